# Round 4: the 128 x 128 Gram tile with global loads two K steps ahead (tree)
# vs one step ahead (pf1) vs the per-wave 64 x 64 tiles (g64), C5; the packed
# pairs beyond 8,192 nodes (tree) vs never (pack0) at C5 and C4; C2 on the
# new rule (full array); parity of the large-module and configuration tests.
set -o pipefail
D=gpurun_out/${1:-r4ab6}
mkdir -p $D
L=netrep_amd/_lib/ab
C5="--config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dual.py tests/test_gpu_configs.py -x -v --timeout 400 --timeout-method thread > $D/pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py $C5 > $D/c5_tree.json 2> $D/c5_tree.err && \
timeout -k 10 400 python -u bench.py $C5 --lib $L/libpf1.so > $D/c5_pf1.json 2> $D/c5_pf1.err && \
timeout -k 10 400 python -u bench.py $C5 --lib $L/libg64.so > $D/c5_g64.json 2> $D/c5_g64.err && \
timeout -k 10 400 python -u bench.py $C5 --lib $L/libpack0.so > $D/c5_pack0.json 2> $D/c5_pack0.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 > $D/bench_tree.json 2> $D/bench_tree.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 --lib $L/libpack0.so > $D/bench_pack0.json 2> $D/bench_pack0.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 > $D/c2_tree.json 2> $D/c2_tree.err
