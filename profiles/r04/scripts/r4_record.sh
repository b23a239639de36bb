# Round 4 record lines: the default bench (C3 + C4 secondary + CPU baseline), C2 with its CPU
# baseline, and C5 (three host datasets, null = "all") at the reference's default of
# 10,000 permutations per dataset, with its CPU baseline.
set -o pipefail
D=gpurun_out/${1:-r4rec}
mkdir -p $D
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-secondary > $D/C2.json 2> $D/C2.err && \
timeout -k 10 900 python -u bench.py --config C5 --steps 1 --warmup 1 --perms-per-step 10000 > $D/C5.json 2> $D/C5.err
