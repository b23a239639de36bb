# Phase stamps of the small class (C2 shape) and of the table kernel (C3 shape), diagnostic build
set -o pipefail
D=gpurun_out/${1:-r3small_stamps}
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 stamps=netrep_amd/_lib/ab/libstamps.so > $D/ab_C2.txt 2>&1 && \
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 stamps=netrep_amd/_lib/ab/libstamps.so > $D/ab_C3.txt 2>&1
