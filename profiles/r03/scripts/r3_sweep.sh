# C3 bench sweeps on the table kernel: launch batch and queue order
set -o pipefail
D=gpurun_out/${1:-r3sweep}
mkdir -p $D
for b in 2560 10240; do
  timeout -k 10 400 python -u bench.py --batch $b --perms-per-step $b --steps $((102400 / b / 2)) --warmup 1 --no-secondary --no-cpu-baseline > $D/batch$b.json 2> $D/batch$b.err || exit 1
done
for o in 1 2; do
  timeout -k 10 400 python -u bench.py --lib netrep_amd/_lib/ab/libord$o.so --steps 8 --warmup 1 --no-secondary --no-cpu-baseline > $D/order$o.json 2> $D/order$o.err || exit 1
done
timeout -k 10 400 python -u bench.py --steps 8 --warmup 1 --no-secondary --no-cpu-baseline > $D/default.json 2> $D/default.err
