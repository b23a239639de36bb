# A/B (C3 shape): the table gathers' chunking with selective zeroing in every build
set -o pipefail
D=gpurun_out/${1:-r3chunk}
mkdir -p $D
timeout -k 10 500 python -u tools/probes/profile_ab.py 500 30 300 50 u7=netrep_amd/_lib/ab/libzero.so u3=netrep_amd/_lib/ab/libu3.so u4=netrep_amd/_lib/ab/libu4.so pipe2=netrep_amd/_lib/ab/libpipe2.so pipe3=netrep_amd/_lib/ab/libpipe3.so u5=netrep_amd/_lib/ab/libu5.so pipe3b=netrep_amd/_lib/ab/libpipe3.so > $D/ab_C3.txt 2>&1
