# Round 6 A/B 10 on C2: the wave class's Gram with one register set of
# operands refilled column by column (wave, the in-tree build, which also has
# the 64 x 112 dual Gram of the large modules, r6_ab9's gB) against ritz,
# alternating; one C5 line of the in-tree build; then the wave-class and
# large-module parity tests on it.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab10
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
A=netrep_amd/_lib/ab
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10 --config C2"
for i in 1 2; do
  for v in ritz wave; do
    timeout -k 10 300 $B --lib $A/lib$v.so > $D/${v}_C2.$i.json 2> $D/${v}_C2.$i.err
  done
done
timeout -k 10 300 python -u bench.py --config C5 --perms-per-step 10000 --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > $D/wave_C5.json 2> $D/wave_C5.err
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 800 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_dual.py -m gpu -x -v -k "c2 or small or wave or bundled or golden or driver or dual or large or big or c5 or lanczos" --timeout 500 --timeout-method thread > $D/pytest.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
