# Round 5: the wave class's largest step between Ritz checks, 8 / 12 / 16 (C2 shape).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5checkcap
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 600 python -u tools/probes/profile_ab.py 100 30 300 20 cap8=$L/prev.so cap12=$L/cap12.so cap16=$L/cap16.so > $D/ab_C2.txt 2>&1
