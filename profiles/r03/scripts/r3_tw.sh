# A/B: the Gram-table kernel at 4 waves x 3 per CU vs 2 waves x 5 per CU (C3 shape + bench)
set -o pipefail
D=gpurun_out/${1:-r3tw}
mkdir -p $D
timeout -k 10 400 python -u tools/probes/profile_ab.py 500 30 300 50 tw4=netrep_amd/_lib/ab/libtw4.so tw2=netrep_amd/_lib/ab/libtw2.so tw4b=netrep_amd/_lib/ab/libtw4.so tw2b=netrep_amd/_lib/ab/libtw2.so > $D/ab_C3.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --lib netrep_amd/_lib/ab/libtw2.so --steps 4 --warmup 1 --no-secondary --no-cpu-baseline > $D/bench_tw2.json 2> $D/bench_tw2.err
