# Round 4: C3's table kernel against the early-round-4 build (lib6ab, commit
# 6ab38f8, whose run gave 265.7 ms per 5,120 perms) -- later rounds measured
# 271-274 ms. head = the tree before the Gram-store LDS branch was compiled
# out; tree = without it.
set -o pipefail
D=gpurun_out/${1:-r4ab9}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 400 python -u tools/probes/profile_ab.py 500 30 300 50 tree=- head=$L/libhead.so r6ab=$L/lib6ab.so > $D/ab.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 10 > $D/bench_tree.json 2> $D/bench_tree.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 10 --lib $L/lib6ab.so > $D/bench_6ab.json 2> $D/bench_6ab.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 10 --lib $L/libhead.so > $D/bench_head.json 2> $D/bench_head.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 10 > $D/bench_tree2.json 2> $D/bench_tree2.err
