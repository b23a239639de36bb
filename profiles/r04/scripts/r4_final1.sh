# Round 4 final tree, part 1: smoke, the extended parity sweep (1,024 C3 and
# 2,048 C2 permutations against the C++ LAPACK restatement), the C3 PMC passes.
set -o pipefail
D=gpurun_out/${1:-r4fin1}
mkdir -p $D
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.txt 2>&1 && \
timeout -k 10 600 python -u tools/parity_sweep.py 1024 2048 > $D/parity_sweep.json 2> $D/parity_sweep.err && \
bash tools/collect_pmc.sh $D/C3 --config C3 --no-secondary --steps 3 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C3 --json $D/C3_summary.json > $D/C3_summary.txt
