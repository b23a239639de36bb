# Round 4 final tree: the parity sweep extended to C5 (64 permutations of 40
# modules up to 2,000 nodes at S = 1,000: large-module kernels, dual Grams).
set -o pipefail
D=gpurun_out/${1:-r4sweep5}
mkdir -p $D
timeout -k 10 1000 python -u tools/parity_sweep.py 0 0 64 > $D/parity_sweep_C5.json 2> $D/parity_sweep_C5.err
