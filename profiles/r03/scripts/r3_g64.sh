# The large-module kernel's 64 x 64 super-tile Gram: big-module parity tests,
# then C5 (one dataset) with 32 x 32 vs 64 x 64 super-tiles
set -o pipefail
D=gpurun_out/${1:-r3g64}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_dual.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --lib netrep_amd/_lib/ab/libg32.so --config C5 --c5-single --steps 3 --warmup 1 --perms-per-step 512 --batch 64 --no-cpu-baseline > $D/C5s_g32.json 2> $D/C5s_g32.err && \
timeout -k 10 400 python -u bench.py --lib netrep_amd/_lib/ab/libg64.so --config C5 --c5-single --steps 3 --warmup 1 --perms-per-step 512 --batch 64 --no-cpu-baseline > $D/C5s_g64.json 2> $D/C5s_g64.err
