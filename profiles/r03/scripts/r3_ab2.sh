set -o pipefail
mkdir -p gpurun_out/r3ab2
timeout -k 10 600 python -u tools/probes/profile_ab.py 500 30 300 50 packed4 rg4 reg > gpurun_out/r3ab2/ab.txt 2>&1
