# Round 5: the Gram-table kernel at two workgroups per CU (256 VGPRs) with more matvec
# units in flight per wave, against the shipped three per CU (C3 shape, profile_ab).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5tableocc
mkdir -p $D
( while sleep 50; do date >> $D/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
L=netrep_amd/_lib/ab
timeout -k 10 600 python -u tools/probes/profile_ab.py 500 30 300 50 tree=- o2u1=$L/occ2_u1_2.so o2u2=$L/occ2_u2_4.so o2u3=$L/occ2_u3_4.so o3u2=$L/occ3_u2_2.so > $D/ab_C3.txt 2>&1
