# Round 4 final tree, part 2b: the C2 and C4 PMC passes.
set -o pipefail
D=gpurun_out/${1:-r4fin2b}
mkdir -p $D
bash tools/collect_pmc.sh $D/C2 --config C2 --no-secondary --steps 3 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C2 --json $D/C2_summary.json > $D/C2_summary.txt && \
bash tools/collect_pmc.sh $D/C4 --config C4 --batch 1024 --perms-per-step 16384 --steps 4 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C4 --json $D/C4_summary.json > $D/C4_summary.txt
