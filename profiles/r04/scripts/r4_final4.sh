# Round 4 final tree: the whole -m gpu suite once more (its parity_maxerr.json
# is the record quoted in DESIGN.md section 2) and the smoke entry point.
set -o pipefail
D=gpurun_out/${1:-r4fin4}
mkdir -p $D
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $D/pytest.log 2>&1 && \
cp gpurun_out/parity_maxerr.json $D/ && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.txt 2>&1 && \
bash profiles/r04/scripts/r4_stamps.sh r4stamps
