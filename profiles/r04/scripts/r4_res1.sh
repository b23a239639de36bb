# Round 4: the CU-resident Gram-table kernel -- parity (table tests, C3 vs the
# LAPACK restatement, variant 6), A/B against the round-3 table kernel
# (NR_TABLE_RESIDENT=0 build), and the default bench line.
set -o pipefail
D=gpurun_out/${1:-r4res1}
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_configs.py tests/test_gpu_dual.py -x -v \
    --timeout 400 --timeout-method thread -k "table or c3 or beyond" > $D/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/probes/profile_ab.py 500 30 300 50 res=- res0=netrep_amd/_lib/ab/libres0.so > $D/ab.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > $D/bench.json 2> $D/bench.err
