# Round 4 final-tree PMC passes (part A): C3 (Gram-table kernel) and C2 (small class + network kernel)
set -o pipefail
D=gpurun_out/${1:-r4pmcA}
mkdir -p $D
bash tools/collect_pmc.sh $D/C3 --config C3 --no-secondary --steps 3 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C3 --json $D/C3_summary.json > $D/C3_summary.txt && \
bash tools/collect_pmc.sh $D/C2 --config C2 --no-secondary --steps 3 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C2 --json $D/C2_summary.json > $D/C2_summary.txt
