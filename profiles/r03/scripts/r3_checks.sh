# A/B: HEAD vs read-ahead Sturm counts + reciprocal omega, stamps compiled out
set -o pipefail
D=gpurun_out/${1:-r3checks2}
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 head=netrep_amd/_lib/ab/libhead.so eig=netrep_amd/_lib/ab/libeig.so head2=netrep_amd/_lib/ab/libhead.so eig2=netrep_amd/_lib/ab/libeig.so > $D/ab_C3.txt 2>&1 && \
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 head=netrep_amd/_lib/ab/libhead.so eig=netrep_amd/_lib/ab/libeig.so > $D/ab_C2.txt 2>&1
