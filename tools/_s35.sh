# final check of the round: full GPU suite, smoke, bench
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05d_pytest_gpu.log 2>&1
tail -2 gpurun_out/r05d_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05d_smoke.log 2>&1
tail -1 gpurun_out/r05d_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r05d_bench.log 2>&1
echo final done
