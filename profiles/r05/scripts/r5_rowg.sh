# Round 5: the wave matvec's tile rows in groups of 2 / 3 / 4 (C2 shape).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5rowg
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 600 python -u tools/probes/profile_ab.py 100 30 300 20 g2=$L/pairs.so g3=$L/rowg3.so g4=$L/rowg4.so > $D/ab_C2.txt 2>&1
