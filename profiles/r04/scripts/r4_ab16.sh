# Round 4: the large modules' dual Gram with node indices a step ahead (tree)
# vs HEAD; large-module parity tests; C5 one dataset; the big-module probe.
set -o pipefail
D=gpurun_out/${1:-r4ab16}
mkdir -p $D
L=netrep_amd/_lib/ab
C5="--config C5 --c5-single --batch 64 --perms-per-step 256 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dual.py tests/test_gpu_configs.py -x -v --timeout 400 --timeout-method thread -k "dual or big or c5 or large or beyond" > $D/pytest.log 2>&1 && \
timeout -k 10 400 python -u tools/probes/profile_ab.py 1000 330 2000 12 tree=- head=$L/libhead.so > $D/ab_big.txt 2>&1 && \
timeout -k 10 400 python -u bench.py $C5 > $D/c5_tree.json 2> $D/c5_tree.err && \
timeout -k 10 400 python -u bench.py $C5 --lib $L/libhead.so > $D/c5_head.json 2> $D/c5_head.err
