# Round 4: the segmented column flush by DPP moves (tree) vs ds_bpermute
# (prev = the previous commit); the whole -m gpu suite on the tree; then the
# C5 record line again (its traffic now read from the 64-permutation PMC pass
# scaled to the reference interface's 66-permutation launches).
set -o pipefail
D=gpurun_out/${1:-r4ab10}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $D/pytest.log 2>&1 && \
timeout -k 10 400 python -u tools/probes/profile_ab.py 500 30 300 50 tree=- prev=$L/libprev.so > $D/ab.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > $D/bench_tree.json 2> $D/bench_tree.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --lib $L/libprev.so > $D/bench_prev.json 2> $D/bench_prev.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 > $D/c2_tree.json 2> $D/c2_tree.err && \
timeout -k 10 900 python -u bench.py --config C5 --steps 1 --warmup 1 --perms-per-step 10000 > $D/C5.json 2> $D/C5.err
