# A/B: the network kernel's gather chunk (7 / 4 / 3 pairs): bench C3 (+ the C4
# network-only record) and C2; the table kernel at 2-pair chunks in every build
set -o pipefail
D=gpurun_out/${1:-r3netu}
mkdir -p $D
for u in 7 4 3; do
  timeout -k 10 300 python -u bench.py --lib netrep_amd/_lib/ab/libnet$u.so --steps 4 --warmup 1 --no-cpu-baseline > $D/bench_u$u.json 2> $D/bench_u$u.err || exit 1
  timeout -k 10 300 python -u bench.py --lib netrep_amd/_lib/ab/libnet$u.so --config C2 --no-secondary --steps 8 --warmup 1 --no-cpu-baseline > $D/C2_u$u.json 2> $D/C2_u$u.err || exit 1
done
