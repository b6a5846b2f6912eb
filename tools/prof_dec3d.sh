#!/bin/bash
# SQ counters of the 3-D decoders (prof_cases.py c3dec: k_decode3d_fixed at rate 8, k_decode_staged<3> at 1e-3).
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY -d gpurun_out/dec_sq -o pmc --output-format csv -- python tools/prof_cases.py c3dec --reps 3 > gpurun_out/dec_sq.log 2>&1 || exit $?
python tools/pmc_summary.py gpurun_out/dec_sq > gpurun_out/dec_sq.json
