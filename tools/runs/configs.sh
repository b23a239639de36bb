set -o pipefail
D=gpurun_out/cfg3; mkdir -p $D
timeout -k 10 300 python -u bench.py --config C2 --no-secondary --no-cpu-baseline > $D/C2.json 2> $D/C2.err && \
timeout -k 10 500 python -u bench.py --config C5 --no-secondary --no-cpu-baseline --steps 4 > $D/C5.json 2> $D/C5.err
