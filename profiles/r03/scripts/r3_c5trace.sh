# C5 three-dataset pipeline timeline: kernel, copy and HIP API trace
set -o pipefail
D=gpurun_out/${1:-r3c5t}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --stats --output-format csv -d $D/trace -o run -- \
  python3 bench.py --config C5 --steps 2 --warmup 0 --perms-per-step 512 > $D/C5.json 2> $D/C5.err
