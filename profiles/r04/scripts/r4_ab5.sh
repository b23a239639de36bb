# Round 4: the large modules' Gram in 128 x 128 LDS-staged workgroup tiles
# (NR_BIG_G128, tree) against the per-wave 64 x 64 tiles (g64): parity of the
# large-module kernel (small/dual/C5 tests) and C5 (one resident dataset,
# 64-permutation launches).
set -o pipefail
D=gpurun_out/${1:-r4ab5}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 900 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_dual.py tests/test_gpu_configs.py -x -v \
    --timeout 400 --timeout-method thread -k "large or beyond or c5 or size_classes" > $D/pytest.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline > $D/c5_tree.json 2> $D/c5_tree.err && \
timeout -k 10 400 python -u bench.py --config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline --lib $L/libg64.so > $D/c5_g64.json 2> $D/c5_g64.err
