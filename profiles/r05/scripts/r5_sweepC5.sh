# Round 5 final tree: the extended C5 parity sweep (64 permutations, large-module kernels,
# the sweep's 16-lane path for modules beyond 1,024 nodes) against the C++ oracle.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5sweepC5
mkdir -p $D
timeout -k 10 1000 python -u tools/parity_sweep.py 0 0 64 > $D/parity_sweep_C5.json 2> $D/parity_sweep_C5.err
