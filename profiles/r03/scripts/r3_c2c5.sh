set -o pipefail
D=gpurun_out/${1:-r3cc}; mkdir -p $D
timeout -k 10 300 python -u bench.py --config C2 --no-secondary --no-cpu-baseline > $D/C2.json 2> $D/C2.err && \
timeout -k 10 120 ./tools/probes/gather_probe 40000 > $D/gather_probe_40k.txt 2>&1 && \
timeout -k 10 900 python -u bench.py --config C5 --steps 2 --warmup 1 --perms-per-step 512 > $D/C5.json 2> $D/C5.err
