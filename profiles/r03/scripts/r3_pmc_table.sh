# rocprofv3 kernel trace + PMC passes of the default C3 bench on the Gram-table
# kernel (bench default launch of 5,120 permutations), then its summary
set -o pipefail
D=gpurun_out/${1:-r3pmc_table}
mkdir -p $D
bash tools/collect_pmc.sh $D/C3 --config C3 --no-secondary --steps 3 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C3 --json $D/C3_summary.json > $D/C3_summary.txt
