# Round 5: wave class phase stamps (LDS-accumulated) on the C2 shape.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5wave6
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 wave_st=netrep_amd/_lib/diag/wave_stamps.so > $D/stamps_C2.txt 2>&1
