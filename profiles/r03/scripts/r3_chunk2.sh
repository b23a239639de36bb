# A/B (C3 shape): smaller table-gather chunks
set -o pipefail
D=gpurun_out/${1:-r3chunk2}
mkdir -p $D
timeout -k 10 500 python -u tools/probes/profile_ab.py 500 30 300 50 pipe2=netrep_amd/_lib/ab/libpipe2.so u3=netrep_amd/_lib/ab/libu3.so u2=netrep_amd/_lib/ab/libu2.so u1=netrep_amd/_lib/ab/libu1.so pipe1=netrep_amd/_lib/ab/libpipe1.so pipe2b=netrep_amd/_lib/ab/libpipe2.so > $D/ab_C3.txt 2>&1
