#!/bin/bash
# ablation: compute floor vs memory floor vs real kernel; SQ counters of the real kernel; DDP tests
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "600|pytest_new|python -m pytest tests/test_reference_suites.py tests/test_gpu_parity.py -k 'reference or ddp' -m gpu -q -rs" \
  "300|ablate|python tools/ubench/ablate.py 12,10,11,9,8 32" \
  "120|list|rocprofv3 -L > gpurun_out/counters.txt 2>&1; grep -c . gpurun_out/counters.txt" \
  "300|sq|rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d gpurun_out/prof_sq -o sq --output-format csv -- python3 tools/ubench/ablate.py 12,10 32" \
  "300|sq2|rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/prof_sq2 -o sq --output-format csv -- python3 tools/ubench/ablate.py 12,10 32"
