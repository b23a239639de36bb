# Round 5: same-box A/B of the two-node finish kernel (current tree) against HEAD (ab/head.so), C4 / C2, with kernel stats.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5fin3
mkdir -p $D
for v in cur head cur2 head2; do
  L=""; case $v in head*) L="--lib netrep_amd/_lib/ab/head.so";; esac
  timeout -k 10 300 python -u bench.py --config C4 --steps 4 --warmup 1 --no-cpu-baseline $L > $D/C4_$v.json 2> $D/C4_$v.err
  timeout -k 10 300 python -u bench.py --config C2 --steps 5 --warmup 1 --no-cpu-baseline --no-secondary $L > $D/C2_$v.json 2> $D/C2_$v.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o cur -- python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline > $D/C4_pc.json 2> $D/C4_pc.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o head -- python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --lib netrep_amd/_lib/ab/head.so > $D/C4_ph.json 2> $D/C4_ph.err
rm -f $D/prof/*_kernel_trace.csv
