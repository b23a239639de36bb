# North-star subsystems outside the permutation loop (Scale / CheckFinite /
# NetProps / IntermediateProperties at 20,000 x 500): kernel trace + one
# FETCH_SIZE and one WRITE_SIZE pass; the traced run also measures the
# residency fingerprint at the C5 shape. D: output directory.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=${D:-gpurun_out/props}
mkdir -p $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 tools/props_record.py --c5-fingerprint > $D/props.json 2> $D/props.err
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 tools/props_record.py > $D/props_fetch.json 2> $D/props_fetch.err
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 tools/props_record.py > $D/props_write.json 2> $D/props_write.err
