set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/updw_fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench_updw.py > $GRAFT_REPO_ROOT/gpurun_out/updw_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/updw_write -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench_updw.py > $GRAFT_REPO_ROOT/gpurun_out/updw_write.log 2>&1 || exit 1
echo pmc ok
