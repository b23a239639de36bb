# Round 4 final tree (unpadded packed Gram): the extended parity sweep, the C3
# PMC passes, and a repeat of the C2-shaped small-launch probe (ab12 anomaly).
set -o pipefail
D=gpurun_out/${1:-r4fin1b}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.txt 2>&1 && \
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 pad=$L/libpad.so tree=- pad2=$L/libpad.so tree2=- > $D/ab_C2.txt 2>&1 && \
timeout -k 10 600 python -u tools/parity_sweep.py 1024 2048 > $D/parity_sweep.json 2> $D/parity_sweep.err && \
bash tools/collect_pmc.sh $D/C3 --config C3 --no-secondary --steps 3 --warmup 1 && \
python3 tools/summarize_pmc.py $D/C3 --json $D/C3_summary.json > $D/C3_summary.txt
