# A/B: the small class at 3 vs 4 waves per SIMD (C2 shape + bench C2)
set -o pipefail
D=gpurun_out/${1:-r3occ}
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 occ3=netrep_amd/_lib/ab/libocc3.so occ4=netrep_amd/_lib/ab/libocc4.so occ3b=netrep_amd/_lib/ab/libocc3.so occ4b=netrep_amd/_lib/ab/libocc4.so > $D/ab_C2.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --lib netrep_amd/_lib/ab/libocc4.so --config C2 --no-secondary --steps 8 --warmup 1 --no-cpu-baseline > $D/C2_occ4.json 2> $D/C2_occ4.err
