# Round 5: column sweep v9 (scatter fused into the per-item prep, 32-byte slot records):
# parity subset; C4 / C2 bench lines for prefetch depth 6 (default), 4, 8; C4 kernel stats.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5s7
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edge.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.txt 2>&1
for v in def; do
  L=""; [ $v != def ] && L="--lib netrep_amd/_lib/ab/$v.so"
  timeout -k 10 300 python -u bench.py --config C4 --steps 4 --warmup 1 --no-cpu-baseline $L > $D/C4_$v.json 2> $D/C4_$v.err
  timeout -k 10 300 python -u bench.py --config C2 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary $L > $D/C2_$v.json 2> $D/C2_$v.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o c4 --output-format csv -- python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $D/C4_prof.json 2> $D/C4_prof.err
