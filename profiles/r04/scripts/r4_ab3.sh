# Round 4: LDS prefix sized to keep three workgroups per CU (lds2), and the
# Gram table in uncached memory (unc: its random gathers no longer allocate
# lines, so the slots' Gram scratch may stay in L2 / the Infinity Cache).
set -o pipefail
D=gpurun_out/${1:-r4ab3}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 400 python -u tools/probes/profile_ab.py 500 30 300 50 tree=- lds2=$L/liblds2.so unc=$L/libunc.so > $D/ab.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 6 > $D/bench_tree.json 2> $D/bench_tree.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 6 --lib $L/libunc.so > $D/bench_unc.json 2> $D/bench_unc.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 6 --lib $L/liblds2.so > $D/bench_lds2.json 2> $D/bench_lds2.err
