#!/bin/bash
# counters for the variable-rate 1-D kernels (C5 shape): instruction mix, busy and wait cycles, LDS conflicts
cd "$(dirname "$0")/.." && tools/gpu_session.sh \
  "120|pmc1|timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_var1 -o pmc --output-format csv -- python3 tools/bench_configs.py c5" \
  "120|pmc2|timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_var2 -o pmc --output-format csv -- python3 tools/bench_configs.py c5"
