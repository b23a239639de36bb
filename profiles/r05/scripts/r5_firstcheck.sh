# Round 5: the wave class's first Ritz check at step 20 / 24 instead of 16 (C2 shape).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5firstcheck
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 600 python -u tools/probes/profile_ab.py 100 30 300 20 fc16=$L/prev.so fc20=$L/fc20.so fc24=$L/fc24.so > $D/ab_C2.txt 2>&1
