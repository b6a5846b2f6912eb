#!/bin/bash
# re-entry check: full GPU suite, smoke, bench, kernel-trace profile of the bench
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "900|pytest_gpu|python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread" \
  "300|smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300|bench|python bench.py" \
  "300|prof_kt|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-e2e"
