set -e
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
LDS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for form in sp tp; do
  if [ $form = sp ]; then export GCOW_VAR1D_SINGLE_PASS=1; else unset GCOW_VAR1D_SINGLE_PASS; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$form -o kt --output-format csv -- python tools/prof_cases.py c5 --reps 5 > gpurun_out/kt_$form.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/sq_$form -o pmc --output-format csv -- python tools/prof_cases.py c5 --reps 2 > gpurun_out/sq_$form.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $LDS -d gpurun_out/lds_$form -o pmc --output-format csv -- python tools/prof_cases.py c5 --reps 2 > gpurun_out/lds_$form.log 2>&1
done
python tools/pmc_summary.py gpurun_out/sq_sp gpurun_out/lds_sp > gpurun_out/sum_sp.json
python tools/pmc_summary.py gpurun_out/sq_tp gpurun_out/lds_tp > gpurun_out/sum_tp.json
