# A/B: Ritz coefficients by the backward recurrence vs inverse iteration (C3, C2, large modules)
set -o pipefail
D=gpurun_out/${1:-r3rec}
mkdir -p $D
timeout -k 10 400 python -u tools/probes/profile_ab.py 500 30 300 50 inv=netrep_amd/_lib/ab/libinv.so rec=netrep_amd/_lib/ab/librec.so inv2=netrep_amd/_lib/ab/libinv.so rec2=netrep_amd/_lib/ab/librec.so > $D/ab_C3.txt 2>&1 && \
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 inv=netrep_amd/_lib/ab/libinv.so rec=netrep_amd/_lib/ab/librec.so > $D/ab_C2.txt 2>&1 && \
timeout -k 10 400 python -u tools/probes/profile_ab.py 1000 330 2000 12 inv=netrep_amd/_lib/ab/libinv.so rec=netrep_amd/_lib/ab/librec.so > $D/ab_big.txt 2>&1
