# Phase stamps of the profile kernel (Gram-table build at C3, dual Gram at C2
# sizes) and the Lanczos-tolerance A/B build
set -o pipefail
D=gpurun_out/${1:-r3stamps}
mkdir -p $D
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 tree tol14=netrep_amd/_lib/ab/libtol14.so > $D/ab_C3.txt 2>&1 && \
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 tree > $D/ab_C2.txt 2>&1
