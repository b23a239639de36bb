# Round 6 final tree (the fp32-crossing Ritz check back on, with the cheaper
# checks), part 1: smoke, the whole GPU suite, the driver's default bench
# command, the C2 / C4 / C5 lines, the kernel trace of the default command.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6final4
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 python -u bench.py --config C2 > $D/C2.json 2> $D/C2.err
timeout -k 10 300 python -u bench.py --config C4 --no-cpu-baseline > $D/C4.json 2> $D/C4.err
timeout -k 10 400 python -u bench.py --config C5 --perms-per-step 10000 --steps 1 --warmup 1 --no-cpu-baseline > $D/C5.json 2> $D/C5.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --no-cpu-baseline > $D/trace_bench.json 2> $D/trace_bench.err
cp $D/trace/run_kernel_stats.csv $D/kernel_stats_default_cmd.csv
rm -rf $D/trace
du -sh gpurun_out
