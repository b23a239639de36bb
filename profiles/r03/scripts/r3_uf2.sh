# A/B: two fp64 matvec units in flight per wave (C3 and C2 shapes + bench C3)
set -o pipefail
D=gpurun_out/${1:-r3uf2}
mkdir -p $D
timeout -k 10 400 python -u tools/probes/profile_ab.py 500 30 300 50 uf1=netrep_amd/_lib/ab/libnet7.so uf2=netrep_amd/_lib/ab/libuf2.so uf1b=netrep_amd/_lib/ab/libnet7.so uf2b=netrep_amd/_lib/ab/libuf2.so > $D/ab_C3.txt 2>&1 && \
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 uf1=netrep_amd/_lib/ab/libnet7.so uf2=netrep_amd/_lib/ab/libuf2.so > $D/ab_C2.txt 2>&1
