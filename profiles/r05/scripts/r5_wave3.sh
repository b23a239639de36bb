# Round 5: phase stamps of the wave class on the C2 shape (diagnostic build).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5wave3
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 wave_st=netrep_amd/_lib/diag/wave_stamps.so > $D/stamps_C2.txt 2>&1
