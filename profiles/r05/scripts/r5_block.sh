# Round 5: the block Lanczos probe (b = 16, G V on the matrix cores), modes 0 and 1.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5block
mkdir -p $D
timeout -k 10 400 python -u tools/probes/block_probe.py tools/probes/bp_kernel.so 100 256000 2 0 > $D/mode0.log 2>&1
timeout -k 10 400 python -u tools/probes/block_probe.py tools/probes/bp_kernel.so 100 256000 2 1 > $D/mode1.log 2>&1
