set -o pipefail
D=gpurun_out/s3d; mkdir -p $D
B="python -u bench.py --steps 10 --no-secondary --no-cpu-baseline"
timeout -k 10 200 $B > $D/base.json 2> $D/base.err && \
NETREP_PROFILE_WG_PER_CU=4 timeout -k 10 200 $B > $D/wg4.json 2> $D/wg4.err && \
NETREP_RELAX=0 timeout -k 10 200 $B > $D/norelax.json 2> $D/norelax.err && \
timeout -k 10 200 $B --stamps > $D/stamps.json 2> $D/stamps.err
