# A/B: modules of 330-700 nodes at S = 600 (two workgroups per CU fit): the packed
# runtime-layout kernel (32 x 32 Gram, 2 per CU) vs the large-module kernel (64 x 64, 1 per CU)
set -o pipefail
D=gpurun_out/${1:-r3bigall}
mkdir -p $D
timeout -k 10 400 python -u tools/probes/profile_ab.py 600 330 700 12 two=netrep_amd/_lib/ab/libpp0.so one=netrep_amd/_lib/ab/libbigall.so > $D/ab_mid.txt 2>&1
