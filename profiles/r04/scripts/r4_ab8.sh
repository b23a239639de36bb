# Round 4: network kernels specialised on the pairs' layout (packed / full at
# compile time) and the two-wave pipelined items flushing directly; the
# packed pairs beyond 8,192 nodes (tree) vs never (pack0) at C5 and C4; the
# whole -m gpu suite on the tree.
set -o pipefail
D=gpurun_out/${1:-r4ab8}
mkdir -p $D
L=netrep_amd/_lib/ab
C5="--config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $D/pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py $C5 > $D/c5_tree.json 2> $D/c5_tree.err && \
timeout -k 10 400 python -u bench.py $C5 --lib $L/libpack0.so > $D/c5_pack0.json 2> $D/c5_pack0.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 > $D/bench_tree.json 2> $D/bench_tree.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 --lib $L/libpack0.so > $D/bench_pack0.json 2> $D/bench_pack0.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 > $D/c2_tree.json 2> $D/c2_tree.err
