# Round 6 A/B 1: an extra Ritz check at the predicted crossing of the fp32
# threshold (new) against the round-5 kernel (base), same box, alternating;
# then the C3 parity test (256 permutations) on the new build.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab1
mkdir -p $D
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
for i in 1 2; do
  timeout -k 10 300 $B --lib netrep_amd/_lib/ab/libbase.so > $D/base$i.json 2> $D/base$i.err
  timeout -k 10 300 $B > $D/new$i.json 2> $D/new$i.err
done
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -k "c3_nulls" --timeout 500 --timeout-method thread > $D/pytest_c3.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
