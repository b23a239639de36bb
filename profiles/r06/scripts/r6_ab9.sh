# Round 6 A/B 9 on C5 (10,000 permutations per dataset), large-module Gram
# tiles: g96 (dual 64 x 96, r6_ab8's winner), gB (dual 64 x 112), gC (g96 +
# primal 64 x 80 with the rolling buffer), gD (g96 + primal 64 x 64 rolling);
# then gC in place of the in-tree library for the large-module parity tests.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6ab9
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
A=netrep_amd/_lib/ab
B5="python -u bench.py --config C5 --perms-per-step 10000 --steps 1 --warmup 1 --no-secondary --no-cpu-baseline"
i=0
for v in g96 gB gC gD g96 gC; do
  i=$((i+1))
  timeout -k 10 300 $B5 --lib $A/lib$v.so > $D/${v}_C5.$i.json 2> $D/${v}_C5.$i.err
done
cp $A/libgC.so netrep_amd/_lib/libnetrep_amd.so
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 700 python -u -m pytest tests/test_gpu_dual.py tests/test_gpu_small.py tests/test_gpu_configs.py -m gpu -x -v -k "dual or large or big or c5 or lanczos" --timeout 500 --timeout-method thread > $D/pytest.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
