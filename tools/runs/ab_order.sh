set -o pipefail
D=gpurun_out/order; mkdir -p $D
B="python -u bench.py --steps 8 --no-secondary --no-cpu-baseline"
timeout -k 10 300 $B > $D/base.json 2> $D/base.err && \
NETREP_PROFILE_ORDER_TAIL=0 timeout -k 10 300 $B > $D/modmajor.json 2> $D/modmajor.err && \
NETREP_PROFILE_ORDER_TAIL=100 timeout -k 10 300 $B > $D/tail100.json 2> $D/tail100.err
