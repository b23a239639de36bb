# Round 4: the 128 x 128 Gram tile in its own kernel (big128), global loads
# two K steps ahead (tree) vs one (pf1) vs the per-wave 64 x 64 tiles (g64);
# the network kernel's segmented column flush (tree) vs direct atomics (noseg)
# at C5 (the C5 network launch measured 36 G reads/s this round vs 41 in round 3).
set -o pipefail
D=gpurun_out/${1:-r4ab7}
mkdir -p $D
L=netrep_amd/_lib/ab
C5="--config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dual.py tests/test_gpu_configs.py -x -v --timeout 400 --timeout-method thread -k "dual or big or c5 or large or beyond" > $D/pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py $C5 > $D/c5_tree.json 2> $D/c5_tree.err && \
timeout -k 10 400 python -u bench.py $C5 --lib $L/libpf1.so > $D/c5_pf1.json 2> $D/c5_pf1.err && \
timeout -k 10 400 python -u bench.py $C5 --lib $L/libg64.so > $D/c5_g64.json 2> $D/c5_g64.err && \
timeout -k 10 400 python -u bench.py $C5 --lib $L/libnoseg.so > $D/c5_noseg.json 2> $D/c5_noseg.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 --lib $L/libnoseg.so > $D/c2_noseg.json 2> $D/c2_noseg.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 > $D/c2_tree.json 2> $D/c2_tree.err
