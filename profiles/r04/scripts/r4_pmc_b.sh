# Round 4 final-tree PMC passes (part B): C4 (network only, 1,024-permutation launches as the
# bench's secondary record) and C5 (one resident dataset, 64-permutation launches)
set -o pipefail
D=gpurun_out/${1:-r4pmcB}
mkdir -p $D
bash tools/collect_pmc.sh $D/C4 --config C4 --batch 1024 --perms-per-step 16384 --steps 4 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C4 --json $D/C4_summary.json > $D/C4_summary.txt && \
bash tools/collect_pmc.sh $D/C5 --config C5 --c5-single --batch 64 --steps 2 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C5 --json $D/C5_summary.json > $D/C5_summary.txt
