# bench.py's default command after the value_incl_table_build field (short run)
set -o pipefail
D=gpurun_out/${1:-r4benchchk}
mkdir -p $D
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline --secondary-steps 2 > $D/bench.json 2> $D/bench.err && \
# then the dual-Gram index prefetch A/B (profiles/r04/scripts/r4_ab16.sh)
[ -s $D/bench.json ] && bash profiles/r04/scripts/r4_ab16.sh r4ab16
