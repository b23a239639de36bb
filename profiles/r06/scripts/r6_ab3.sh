# Round 6 A/B 3: cheaper Ritz checks (check: the top eigenvalue to 1e-9 of the
# scale unless the run may stop, power-of-two multisection points, DPP
# Gershgorin bounds, the residual recurrence reading 8 steps ahead, fp32 log2
# step predictions) against the round-5 kernel (base), alternating on C3 and
# C2; C5 once each; then `check` in place of the in-tree library for the
# full-size parity tests and the parity sweep (C3 1,024, C2 2,048 permutations),
# and phase stamps of its diagnostic build.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab3
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
for i in 1 2; do
  for c in C3 C2; do
    timeout -k 10 300 $B --config $c --lib netrep_amd/_lib/ab/libbase.so > $D/base_$c.$i.json 2> $D/base_$c.$i.err
    timeout -k 10 300 $B --config $c --lib netrep_amd/_lib/ab/libcheck.so > $D/check_$c.$i.json 2> $D/check_$c.$i.err
  done
done
timeout -k 10 400 $B --config C5 --steps 4 --lib netrep_amd/_lib/ab/libbase.so > $D/base_C5.json 2> $D/base_C5.err
timeout -k 10 400 $B --config C5 --steps 4 --lib netrep_amd/_lib/ab/libcheck.so > $D/check_C5.json 2> $D/check_C5.err
S="python -u bench.py --no-secondary --no-cpu-baseline --steps 3 --stamps --lib netrep_amd/_lib/diag/libstamps.so"
timeout -k 10 300 $S > $D/stamps_C3.json 2> $D/stamps_C3.err
timeout -k 10 300 $S --config C2 > $D/stamps_C2.json 2> $D/stamps_C2.err
cp netrep_amd/_lib/ab/libcheck.so netrep_amd/_lib/libnetrep_amd.so
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 700 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_small.py tests/test_gpu_dual.py -m gpu -x -v --timeout 500 --timeout-method thread > $D/pytest_cfg.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
timeout -k 10 700 python -u tools/parity_sweep.py 1024 2048 0 > $D/parity_sweep.json 2> $D/parity_sweep.err
