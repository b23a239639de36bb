# A/B (C3 shape): selective zeroing of the table items' packed Gram, and the
# table gathers' chunking (5 pairs; 3 pairs with the next chunk in flight)
set -o pipefail
D=gpurun_out/${1:-r3zero}
mkdir -p $D
timeout -k 10 400 python -u tools/probes/profile_ab.py 500 30 300 50 head=netrep_amd/_lib/ab/libhead.so zero=netrep_amd/_lib/ab/libzero.so u5=netrep_amd/_lib/ab/libu5.so pipe3=netrep_amd/_lib/ab/libpipe3.so head2=netrep_amd/_lib/ab/libhead.so zero2=netrep_amd/_lib/ab/libzero.so > $D/ab_C3.txt 2>&1
