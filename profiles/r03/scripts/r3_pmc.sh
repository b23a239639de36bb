# rocprofv3 PMC passes (tools/collect_pmc.sh) for C2 and C5 (engine layer,
# the launch size of the three-dataset run)
set -o pipefail
D=gpurun_out/${1:-r3pmc}
mkdir -p $D
bash tools/collect_pmc.sh $D/C2 --config C2 --no-secondary --steps 3 --warmup 1 && \
bash tools/collect_pmc.sh $D/C5 --config C5 --c5-single --steps 1 --warmup 1 --perms-per-step 512 --batch 64 && \
python3 tools/summarize_pmc.py $D/C2 --json $D/C2_summary.json > $D/C2_summary.txt && \
python3 tools/summarize_pmc.py $D/C5 --json $D/C5_summary.json > $D/C5_summary.txt
