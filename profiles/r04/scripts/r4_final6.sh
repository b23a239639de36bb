# Round 4 final tree: the C5 record line again (three host datasets, 10,000
# permutations each, 64-permutation automatic launches) with its CPU baseline.
set -o pipefail
D=gpurun_out/${1:-r4fin6}
mkdir -p $D
timeout -k 10 900 python -u bench.py --config C5 --steps 1 --warmup 1 --perms-per-step 10000 > $D/C5.json 2> $D/C5.err
