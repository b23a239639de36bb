# Round 4 final tree, part 3: the record lines (default bench with the C4
# secondary and CPU baseline; C2; C5 at 10,000 perms per dataset).
set -o pipefail
D=gpurun_out/${1:-r4fin3}
mkdir -p $D
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-secondary > $D/C2.json 2> $D/C2.err && \
timeout -k 10 900 python -u bench.py --config C5 --steps 1 --warmup 1 --perms-per-step 10000 > $D/C5.json 2> $D/C5.err
