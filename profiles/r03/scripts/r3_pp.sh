# A/B: the large modules' 64 x 64 Gram with the prefetched step used in turn vs copied
set -o pipefail
D=gpurun_out/${1:-r3pp}
mkdir -p $D
timeout -k 10 400 python -u tools/probes/profile_ab.py 1000 330 2000 12 pp1=netrep_amd/_lib/ab/libpp1.so pp0=netrep_amd/_lib/ab/libpp0.so pp1b=netrep_amd/_lib/ab/libpp1.so pp0b=netrep_amd/_lib/ab/libpp0.so > $D/ab_big.txt 2>&1
