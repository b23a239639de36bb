# phase stamps of the large-module (packed, scratch per-node arrays) items at S = 1,000
set -o pipefail
D=gpurun_out/${1:-r3c5stamps}
mkdir -p $D
timeout -k 10 400 python -u tools/probes/profile_ab.py 1000 330 2000 12 stamps=netrep_amd/_lib/ab/libstamps.so > $D/ab_big.txt 2>&1
