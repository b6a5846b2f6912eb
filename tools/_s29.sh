# round-end set, part 1: full GPU tests, smoke, C2/C5 measurement + bench (measure_round)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_pytest_gpu_final.log 2>&1
tail -3 gpurun_out/r05_pytest_gpu_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05_smoke_final.log 2>&1
tail -1 gpurun_out/r05_smoke_final.log
tools/measure_round.sh r05c
echo part1 done
