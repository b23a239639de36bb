# full GPU suite, smoke, C5 with three host datasets, stamps of the large-module items
set -o pipefail
D=gpurun_out/${1:-r3check3}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 && \
timeout -k 10 900 python -u bench.py --config C5 --steps 2 --warmup 1 --perms-per-step 512 > $D/C5.json 2> $D/C5.err && \
timeout -k 10 400 python -u tools/probes/profile_ab.py 1000 330 2000 12 stamps=netrep_amd/_lib/ab/libstamps.so > $D/stamps_big.txt 2>&1
