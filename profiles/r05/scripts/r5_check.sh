# Round 5: GPU regression suite on the current tree (+ the eigen probe's stamped runs).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5/pytest_gpu.txt 2>&1
P=tools/probes
timeout -k 10 200 python -u $P/eig_probe.py $P/eig_probe_m0.so 1000 256000 2 > gpurun_out/r5/ek_s0.log 2>&1
timeout -k 10 200 python -u $P/eig_probe.py $P/eig_probe_m1.so 1000 256000 2 > gpurun_out/r5/ek_s1.log 2>&1
timeout -k 10 200 python -u $P/eig_probe.py $P/eig_probe_m0.so 1000 256000 2 230 > gpurun_out/r5/ek_s0k.log 2>&1
timeout -k 10 200 python -u $P/eig_probe.py $P/eig_probe_m1.so 1000 256000 2 230 > gpurun_out/r5/ek_s1k.log 2>&1
