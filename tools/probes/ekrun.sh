set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=tools/probes
timeout -k 10 200 python -u $P/eig_probe.py $P/eig_probe_m0.so 1000 256000 2 > gpurun_out/ek_s0.log 2>&1
timeout -k 10 200 python -u $P/eig_probe.py $P/eig_probe_m1.so 1000 256000 2 > gpurun_out/ek_s1.log 2>&1
timeout -k 10 200 python -u $P/eig_probe.py $P/eig_probe_m0.so 1000 256000 2 230 > gpurun_out/ek_s0k.log 2>&1
timeout -k 10 200 python -u $P/eig_probe.py $P/eig_probe_m1.so 1000 256000 2 230 > gpurun_out/ek_s1k.log 2>&1
