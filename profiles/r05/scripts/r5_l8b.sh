# Round 5: sweep with 8 lanes per occurrence + eight-value finite-data records: parity subset, A/B vs 16 lanes.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5l8b
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edge.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
for v in def l16 def2 l162; do
  L=""; case $v in l16*) L="--lib netrep_amd/_lib/ab/l16.so";; esac
  timeout -k 10 300 python -u bench.py --config C4 --steps 4 --warmup 1 --no-cpu-baseline $L > $D/C4_$v.json 2> $D/C4_$v.err
  timeout -k 10 300 python -u bench.py --config C2 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary $L > $D/C2_$v.json 2> $D/C2_$v.err
done
