set -e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r06z_pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06z_smoke.log 2>&1
bash tools/measure_round.sh r06z > gpurun_out/r06z_measure_round.log 2>&1
bash tools/measure_dec.sh r06z > gpurun_out/r06z_measure_dec.log 2>&1
