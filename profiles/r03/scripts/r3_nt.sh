# A/B: Gram-table gathers with and without the non-temporal hint (C3 shape)
set -o pipefail
D=gpurun_out/${1:-r3nt}
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 plain=netrep_amd/_lib/ab/libnont.so nt=netrep_amd/_lib/ab/libnt.so plain2=netrep_amd/_lib/ab/libnont.so nt2=netrep_amd/_lib/ab/libnt.so > $D/ab_C3.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --lib netrep_amd/_lib/ab/libnont.so --steps 2 --warmup 1 --no-cpu-baseline > $D/bench_plain.json 2> $D/bench_plain.err && \
timeout -k 10 300 python -u bench.py --lib netrep_amd/_lib/ab/libnetnt.so --steps 2 --warmup 1 --no-cpu-baseline > $D/bench_netnt.json 2> $D/bench_netnt.err
