# A/B: HEAD vs the burst basis combine (reorthogonalisation + Ritz vector),
# 16 and 32 basis entries in flight; finer phase stamps
set -o pipefail
D=gpurun_out/${1:-r3reorth}
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 head=netrep_amd/_lib/ab/libhead.so tree b32=netrep_amd/_lib/ab/libb32.so > $D/ab_C3.txt 2>&1 && \
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 head=netrep_amd/_lib/ab/libhead.so tree b32=netrep_amd/_lib/ab/libb32.so > $D/ab_C2.txt 2>&1
