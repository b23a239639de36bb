# Round 5: finish kernel with two nodes per lane pass; record-memory bound per sub-batch;
# parity subset + the new mixed-size variant-6 test; C4 / C2 lines.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5fin2
mkdir -p $D
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edge.py "tests/test_gpu_dual.py::test_lanczos_beyond_lds_mixed_sizes_multi_slot" -m gpu -x -v --timeout 400 --timeout-method thread > $D/pytest.txt 2>&1
for v in a b; do
  timeout -k 10 300 python -u bench.py --config C4 --steps 4 --warmup 1 --no-cpu-baseline > $D/C4_$v.json 2> $D/C4_$v.err
  timeout -k 10 300 python -u bench.py --config C2 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $D/C2_$v.json 2> $D/C2_$v.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c4 -- python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $D/C4_prof.json 2> $D/C4_prof.err
rm -f $D/prof/c4_kernel_trace.csv
