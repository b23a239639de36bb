# Round 4 final tree, part 2: the C5 PMC passes on the three-dataset command
# (the reference interface's own 66-permutation launches).
set -o pipefail
D=gpurun_out/${1:-r4fin2}
mkdir -p $D
bash tools/collect_pmc.sh $D/C5 --config C5 --steps 1 --warmup 1 --perms-per-step 1980 && \
python3 tools/summarize_pmc.py $D/C5 --json $D/C5_summary.json > $D/C5_summary.txt
