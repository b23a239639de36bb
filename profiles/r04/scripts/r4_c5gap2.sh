# C5 network launch: 64- vs 66-permutation launches on one box.
set -o pipefail
D=gpurun_out/${1:-r4c5gap2}
mkdir -p $D
timeout -k 10 400 python -u bench.py --config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline > $D/c5_b64.json 2> $D/c5_b64.err && \
timeout -k 10 400 python -u bench.py --config C5 --c5-single --batch 66 --perms-per-step 264 --steps 3 --warmup 1 --no-cpu-baseline > $D/c5_b66.json 2> $D/c5_b66.err && \
timeout -k 10 400 python -u bench.py --config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline > $D/c5_b64b.json 2> $D/c5_b64b.err
