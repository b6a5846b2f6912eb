set -o pipefail
T=${1:-r01g}
mkdir -p gpurun_out/$T
cd $GRAFT_REPO_ROOT
echo "== pytest"; timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/$T/pytest_gpu.log
echo "== smoke"; timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -30 gpurun_out/$T/smoke.log; exit 1; }
tail -2 gpurun_out/$T/smoke.log
echo "== bench"; timeout -k 10 300 python bench.py > gpurun_out/$T/bench.log 2>&1 || { tail -30 gpurun_out/$T/bench.log; exit 1; }
tail -1 gpurun_out/$T/bench.log
echo "== rocprof"; cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$T/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-e2e > $GRAFT_REPO_ROOT/gpurun_out/$T/kt.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/$T/kt.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/$T/kt.log
find $GRAFT_REPO_ROOT/gpurun_out/$T/kt -name "*stats*"
