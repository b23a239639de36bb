# Round 5: the wave matvec's tile rows in pairs (C2 shape) against the previous commit.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5pairs
mkdir -p $D
timeout -k 10 600 python -u tools/probes/profile_ab.py 100 30 300 20 prev=netrep_amd/_lib/ab/prev.so pairs=- > $D/ab_C2.txt 2>&1
