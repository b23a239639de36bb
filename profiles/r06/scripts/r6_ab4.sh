# Round 6 A/B 4, alternating on one box:
#  base   the round-5 kernels
#  check2 cheaper Ritz checks (r6_ab3's `check`), with a check predicted to end
#         the run taking its eigenvalue to full precision in one stage
#  sweep2 check2 + the column sweep's first-after-diagonal term and tail split
#         out of the per-pair loop
# C3: base / check2; C2: base / check2 / sweep2; C4: check2 / sweep2. Then
# sweep2 in place of the in-tree library for the parity tests and the sweep.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab4
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
A=netrep_amd/_lib/ab
for i in 1 2; do
  timeout -k 10 300 $B --lib $A/libbase.so > $D/base_C3.$i.json 2> $D/base_C3.$i.err
  timeout -k 10 300 $B --lib $A/libcheck2.so > $D/check2_C3.$i.json 2> $D/check2_C3.$i.err
  for v in base check2 sweep2; do
    timeout -k 10 300 $B --config C2 --lib $A/lib$v.so > $D/${v}_C2.$i.json 2> $D/${v}_C2.$i.err
  done
  for v in check2 sweep2; do
    timeout -k 10 300 $B --config C4 --lib $A/lib$v.so > $D/${v}_C4.$i.json 2> $D/${v}_C4.$i.err
  done
done
cp $A/libsweep2.so netrep_amd/_lib/libnetrep_amd.so
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_gpu_fallbacks.py tests/test_gpu_configs.py tests/test_gpu_small.py -m gpu -x -v --timeout 500 --timeout-method thread > $D/pytest.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
timeout -k 10 700 python -u tools/parity_sweep.py 1024 2048 0 > $D/parity_sweep.json 2> $D/parity_sweep.err
