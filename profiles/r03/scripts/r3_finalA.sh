# final validation: GPU suite, smoke, extended parity sweep (C3 1,024 / C2 2,048 permutations)
set -o pipefail
D=gpurun_out/${1:-r3finalA}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $D/pytest_gpu.txt 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 && \
timeout -k 10 360 python -u tools/parity_sweep.py 1024 2048 > $D/parity_sweep.json 2> $D/parity_sweep.err
