# rocprofv3 kernel trace + PMC passes (tools/collect_pmc.sh) of the C3 bench
# (Gram-table kernel) and the C2 bench (small class), bench launch of 5,120
set -o pipefail
D=gpurun_out/${1:-r3pmc2}
mkdir -p $D
bash tools/collect_pmc.sh $D/C3 --config C3 --no-secondary --steps 3 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C3 --json $D/C3_summary.json > $D/C3_summary.txt && \
bash tools/collect_pmc.sh $D/C2 --config C2 --no-secondary --steps 3 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C2 --json $D/C2_summary.json > $D/C2_summary.txt
