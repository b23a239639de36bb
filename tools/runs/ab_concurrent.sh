set -o pipefail
D=gpurun_out/conc; mkdir -p $D
B="python -u bench.py --steps 8 --no-secondary --no-cpu-baseline"
timeout -k 10 300 $B > $D/base.json 2> $D/base.err && \
NETREP_CONCURRENT=1 timeout -k 10 300 $B > $D/conc.json 2> $D/conc.err && \
NETREP_FUSE=1 timeout -k 10 300 $B > $D/fuse.json 2> $D/fuse.err
