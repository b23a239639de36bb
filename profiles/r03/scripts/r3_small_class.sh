# A/B: C2 (S = 100) on the packed 4-wave kernel vs the small class at 1 and 2
# waves per item
set -o pipefail
D=gpurun_out/${1:-r3small}
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 eig=netrep_amd/_lib/ab/libeig.so small1=netrep_amd/_lib/ab/libsmall1.so small2=netrep_amd/_lib/ab/libsmall2.so > $D/ab_C2.txt 2>&1
