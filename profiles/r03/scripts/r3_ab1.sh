set -o pipefail
mkdir -p gpurun_out/r3ab1
timeout -k 10 600 python -u tools/probes/profile_ab.py 500 30 300 50 packed4 reg reg12 reg16 > gpurun_out/r3ab1/ab.txt 2>&1
