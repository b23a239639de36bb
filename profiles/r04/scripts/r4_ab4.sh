# Round 4: whole -m gpu suite on the tree (small symmetric datasets now use the
# packed-triangle pairs), then A/Bs: C3 LDS prefix (lds2) and uncached table
# (unc); C2 packed vs full pairs (pack0); C4 with every symmetric dataset
# packed (pack2).
set -o pipefail
D=gpurun_out/${1:-r4ab4}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $D/pytest.log 2>&1 && \
timeout -k 10 400 python -u tools/probes/profile_ab.py 500 30 300 50 tree=- lds2=$L/liblds2.so unc=$L/libunc.so > $D/ab.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 > $D/bench_tree.json 2> $D/bench_tree.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 6 --lib $L/libunc.so > $D/bench_unc.json 2> $D/bench_unc.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 --lib $L/libpack2.so > $D/bench_pack2.json 2> $D/bench_pack2.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 > $D/c2_tree.json 2> $D/c2_tree.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 --lib $L/libpack0.so > $D/c2_pack0.json 2> $D/c2_pack0.err && \
# the large modules' Gram in 128 x 128 LDS-staged workgroup tiles (tree) vs the per-wave 64 x 64 tiles
timeout -k 10 400 python -u bench.py --config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline > $D/c5_tree.json 2> $D/c5_tree.err && \
timeout -k 10 400 python -u bench.py --config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline --lib $L/libg64.so > $D/c5_g64.json 2> $D/c5_g64.err && \
# the unfused network launch on a side stream beside the small-class profiles (C2)
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 --lib $L/libside.so > $D/c2_side.json 2> $D/c2_side.err
