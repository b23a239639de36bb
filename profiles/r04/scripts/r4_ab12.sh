# Round 4: the packed Gram without row padding (tree) vs rows padded to a
# multiple of 16 (pad = the previous commit); the whole -m gpu suite on the tree.
set -o pipefail
D=gpurun_out/${1:-r4ab12}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $D/pytest.log 2>&1 && \
timeout -k 10 500 python -u tools/probes/profile_ab.py 500 30 300 50 tree=- pad=$L/libpad.so > $D/ab_C3.txt 2>&1 && \
timeout -k 10 500 python -u tools/probes/profile_ab.py 100 30 300 20 tree=- pad=$L/libpad.so > $D/ab_C2.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 > $D/c2_tree.json 2> $D/c2_tree.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 --lib $L/libpad.so > $D/c2_pad.json 2> $D/c2_pad.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 10 > $D/bench_tree.json 2> $D/bench_tree.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 10 --lib $L/libpad.so > $D/bench_pad.json 2> $D/bench_pad.err && \
timeout -k 10 400 python -u bench.py --config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline > $D/c5_tree.json 2> $D/c5_tree.err && \
timeout -k 10 400 python -u bench.py --config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline --lib $L/libpad.so > $D/c5_pad.json 2> $D/c5_pad.err
