set -o pipefail
D=gpurun_out/batch; mkdir -p $D
B="python -u bench.py --steps 12 --perms-per-step 8192 --no-secondary --no-cpu-baseline"
timeout -k 10 200 $B --launch-batch 1024 > $D/b1024.json 2> $D/b1024.err && \
timeout -k 10 200 $B --launch-batch 2048 > $D/b2048.json 2> $D/b2048.err && \
timeout -k 10 200 $B --launch-batch 4096 > $D/b4096.json 2> $D/b4096.err && \
timeout -k 10 200 $B --launch-batch 8192 > $D/b8192.json 2> $D/b8192.err
