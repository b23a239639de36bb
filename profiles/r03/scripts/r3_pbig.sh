# Large modules on the packed Gram: parity tests of the big-module paths, then
# C5 (one dataset, engine layer) with and without it
set -o pipefail
D=gpurun_out/${1:-r3pbig}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_dual.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_small.py -x -v --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1 && \
timeout -k 10 400 python -u bench.py --lib netrep_amd/_lib/ab/libnopbig.so --config C5 --c5-single --steps 3 --warmup 1 --perms-per-step 512 --batch 64 --no-cpu-baseline > $D/C5s_full.json 2> $D/C5s_full.err && \
timeout -k 10 400 python -u bench.py --lib netrep_amd/_lib/ab/libpbig.so --config C5 --c5-single --steps 3 --warmup 1 --perms-per-step 512 --batch 64 --no-cpu-baseline > $D/C5s_packed.json 2> $D/C5s_packed.err
