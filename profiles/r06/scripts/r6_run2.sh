# Round 6: smoke + the whole GPU suite on the committed tree (r6_run1.sh's first
# half), then A/B 2 (r6_ab2.sh) in the same call.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6run1
mkdir -p $D
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/ || true
bash tools/runs/r6_ab2.sh
