# Round 5: kernel trace + one PMC pass of the north star's
# Scale / CheckFinite / NetProps / IntermediateProperties calls at 20,000 x 500.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r5props
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 tools/runs/r5_props.py > $D/props.json 2> $D/props.err
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 tools/runs/r5_props.py > $D/props_fetch.json 2> $D/props_fetch.err
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 tools/runs/r5_props.py > $D/props_write.json 2> $D/props_write.err
