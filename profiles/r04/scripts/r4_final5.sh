# Round 4 final tree with 64-permutation automatic launches: the whole -m gpu
# suite, then the C5 PMC passes on the three-dataset command.
set -o pipefail
D=gpurun_out/${1:-r4fin5}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $D/pytest.log 2>&1 && \
bash tools/collect_pmc.sh $D/C5 --config C5 --steps 1 --warmup 1 --perms-per-step 1920 && \
python3 tools/summarize_pmc.py $D/C5 --json $D/C5_summary.json > $D/C5_summary.txt
