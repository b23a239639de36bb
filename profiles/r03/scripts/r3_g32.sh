# new large-module tests; A/B (C3 shape): the table kernel without its fp32 Gram copy
set -o pipefail
D=gpurun_out/${1:-r3g32}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py -x -v --timeout 300 --timeout-method thread > $D/pytest_small.txt 2>&1 && \
timeout -k 10 400 python -u tools/probes/profile_ab.py 500 30 300 50 g32=netrep_amd/_lib/ab/libg32on.so nog32=netrep_amd/_lib/ab/libg32off.so g32b=netrep_amd/_lib/ab/libg32on.so nog32b=netrep_amd/_lib/ab/libg32off.so > $D/ab_C3.txt 2>&1
