# Round 4: packed Gram diagonal chunks without the upper-triangle zeros (tree)
# vs HEAD (rows unpadded, zeros stored); the -m gpu suite on the tree first.
set -o pipefail
D=gpurun_out/${1:-r4ab14}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $D/pytest.log 2>&1 && \
timeout -k 10 500 python -u tools/probes/profile_ab.py 500 30 300 50 tree=- head=$L/libhead.so tree2=- head2=$L/libhead.so > $D/ab_C3.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 10 > $D/bench_tree.json 2> $D/bench_tree.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 10 --lib $L/libhead.so > $D/bench_head.json 2> $D/bench_head.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 > $D/c2_tree.json 2> $D/c2_tree.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 --lib $L/libhead.so > $D/c2_head.json 2> $D/c2_head.err
