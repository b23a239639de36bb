# Round 6: the ADVICE r5 fixes and the new parity tests on the GPU, then the
# props record (Scale through pinned staging, the fingerprint at C5 shape).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6check1
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_fallbacks.py tests/test_gpu_residency.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
D=$D/props bash tools/props_record.sh
