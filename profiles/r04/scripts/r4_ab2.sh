# Round 4: the table kernel's LDS prefix (NR_TABLE_LDS), the segmented column
# flush of the weighted degrees (NR_WD_SEGSCAN) and the small class's fused
# network statistics (NR_SMALL_FUSE), each against the round-3 build
# (base: neither; lds / seg: one each, no small fusion); parity of the tree.
set -o pipefail
D=gpurun_out/${1:-r4ab2}
mkdir -p $D
L=netrep_amd/_lib/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_parity.py tests/test_gpu_small.py tests/test_gpu_configs.py -x -v \
    --timeout 300 --timeout-method thread -k "not c5" > $D/pytest.log 2>&1 && \
timeout -k 10 400 python -u tools/probes/profile_ab.py 500 30 300 50 tree=- base=$L/libbase.so lds=$L/liblds.so seg=$L/libseg.so > $D/ab.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 --lib $L/libbase.so > $D/bench_base.json 2> $D/bench_base.err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 6 > $D/bench_tree.json 2> $D/bench_tree.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 --lib $L/libbase.so > $D/c2_base.json 2> $D/c2_base.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 --lib $L/libseg.so > $D/c2_seg.json 2> $D/c2_seg.err && \
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 6 > $D/c2_tree.json 2> $D/c2_tree.err
