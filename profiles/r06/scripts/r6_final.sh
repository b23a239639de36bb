# Round 6 final tree, part 1: A/B 7 on C3, smoke, the whole GPU suite, the
# driver's default bench command and the C2 / C4 lines, the kernel trace of the
# default command (part 2: r6_final2.sh).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r6final
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
# A/B 7 first: the multi-wave kernels' Ritz vector with eight basis loads in
# flight (the in-tree build) against sweep2 (without it), alternating on C3
B="python -u bench.py --no-secondary --no-cpu-baseline --steps 10"
for i in 1 2; do
  timeout -k 10 300 $B --lib netrep_amd/_lib/ab/libsweep2.so > $D/ab7_sweep2_C3.$i.json 2> $D/ab7_sweep2_C3.$i.err
  timeout -k 10 300 $B > $D/ab7_ritz_C3.$i.json 2> $D/ab7_ritz_C3.$i.err
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1
rm -f gpurun_out/parity_maxerr.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1
cp gpurun_out/parity_maxerr.json $D/
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 python -u bench.py --config C2 > $D/C2.json 2> $D/C2.err
timeout -k 10 300 python -u bench.py --config C4 --no-cpu-baseline > $D/C4.json 2> $D/C4.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --no-cpu-baseline > $D/trace_bench.json 2> $D/trace_bench.err
cp $D/trace/run_kernel_stats.csv $D/kernel_stats_default_cmd.csv
rm -rf $D/trace
du -sh gpurun_out
