# Round 4 final tree: per-phase cycle stamps (diagnostic build) of the table
# kernel (C3 shape), the small class (C2 shape) and the large modules (C5 shape).
set -o pipefail
D=gpurun_out/${1:-r4stamps}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 stamps=$L/libstamps.so > $D/stamps_C3.txt 2>&1 && \
timeout -k 10 300 python -u tools/probes/profile_ab.py 100 30 300 20 stamps=$L/libstamps.so > $D/stamps_C2.txt 2>&1 && \
timeout -k 10 400 python -u tools/probes/profile_ab.py 1000 330 2000 12 stamps=$L/libstamps.so > $D/stamps_big.txt 2>&1
