#!/bin/bash
# The round-end GPU set (one gpurun call): the whole GPU suite, smoke, then tools/measure_round.sh and
# tools/measure_dec.sh with the same tag. Logs under gpurun_out/TAG_*; usage: round_set.sh TAG   (e.g. r06z)
set -e
TAG=${1:?tag}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
bash tools/measure_round.sh ${TAG} > gpurun_out/${TAG}_measure_round.log 2>&1
bash tools/measure_dec.sh ${TAG} > gpurun_out/${TAG}_measure_dec.log 2>&1
