# C5 network launch: the three-dataset line's compute-alone pass vs the
# resident single-dataset run, on one box.
set -o pipefail
D=gpurun_out/${1:-r4c5gap}
mkdir -p $D
timeout -k 10 400 python -u bench.py --config C5 --c5-single --batch 66 --perms-per-step 264 --steps 3 --warmup 1 --no-cpu-baseline > $D/c5_single.json 2> $D/c5_single.err && \
timeout -k 10 600 python -u bench.py --config C5 --steps 1 --warmup 1 --perms-per-step 1980 --no-cpu-baseline > $D/c5_three.json 2> $D/c5_three.err
