# Round 6 final tree (the Ritz residual guard by selects, the tridiagonal
# eigenvector reading ahead): smoke, the whole GPU suite, the default bench
# command, the C2 / C4 / C5 lines, the kernel trace, the C3 PMC passes.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6final5
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
bash tools/collect_pmc.sh $D/C3 --config C3 --no-secondary --steps 3 --warmup 1
python3 tools/summarize_pmc.py $D/C3 --json $D/C3/summary.json > $D/C3/summary.txt
cp $D/C3/trace/run_kernel_stats.csv $D/C3/kernel_stats.csv
find $D/C3 -name '*.csv' ! -name 'kernel_stats.csv' -delete
find $D/C3 -name '*.db' -delete
du -sh gpurun_out
