# kernel trace + PMC passes of the final tree: C3 (Gram-table kernel) and C5 (large-module kernel)
set -o pipefail
D=gpurun_out/${1:-r3pmcF}
mkdir -p $D
bash tools/collect_pmc.sh $D/C3 --config C3 --no-secondary --steps 3 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C3 --json $D/C3_summary.json > $D/C3_summary.txt && \
bash tools/collect_pmc.sh $D/C5 --config C5 --c5-single --batch 64 --steps 2 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C5 --json $D/C5_summary.json > $D/C5_summary.txt
