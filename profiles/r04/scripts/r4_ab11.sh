# Round 4: Gram-table chunk size (pairs per lane per gather burst) now that
# each chunk ends in the segmented column flush: 2 (tree) vs 1 and 3.
set -o pipefail
D=gpurun_out/${1:-r4ab11}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 500 python -u tools/probes/profile_ab.py 500 30 300 50 tree=- u1=$L/libu1.so u3=$L/libu3.so tree2=- > $D/ab.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 10 --lib $L/libu3.so > $D/bench_u3.json 2> $D/bench_u3.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 10 > $D/bench_tree.json 2> $D/bench_tree.err
