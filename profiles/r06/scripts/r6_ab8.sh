# Round 6 A/B 8 on C5 (10,000 permutations per dataset): the large modules'
# dual Gram in 64 x 96 super-tiles per wave with a rolling operand buffer
# (g96: 24 tiles per 10 operand blocks, 192 accumulator registers), or in
# 64 x 64 with the rolling buffer (g64r), against the in-tree 64 x 64
# double-buffered tile (ritz). Then g96 in place of the in-tree library for
# the large-module parity tests.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab8
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
A=netrep_amd/_lib/ab
B5="python -u bench.py --config C5 --perms-per-step 10000 --steps 1 --warmup 1 --no-secondary --no-cpu-baseline"
for v in ritz g96 g64r ritz g96; do
  timeout -k 10 300 $B5 --lib $A/lib$v.so > $D/${v}_C5.$(date +%s).json 2> $D/${v}_C5.err
done
cp $A/libg96.so netrep_amd/_lib/libnetrep_amd.so
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 700 python -u -m pytest tests/test_gpu_dual.py tests/test_gpu_small.py tests/test_gpu_configs.py -m gpu -x -v -k "dual or large or big or c5 or lanczos" --timeout 500 --timeout-method thread > $D/pytest.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
