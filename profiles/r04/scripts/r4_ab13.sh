# Round 4: table-kernel retuning on the final tree: the next gather chunk in
# flight (pipe) and two fp64 matvec units in flight (uf2) vs the tree.
set -o pipefail
D=gpurun_out/${1:-r4ab13}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 500 python -u tools/probes/profile_ab.py 500 30 300 50 tree=- pipe=$L/libpipe.so uf2=$L/libuf2.so tree2=- > $D/ab.txt 2>&1
