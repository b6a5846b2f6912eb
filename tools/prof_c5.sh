# C5 (256 Mi bf16, accuracy 1e-6 / 1e-3) encoder forms: kernel trace, SQ instruction / wait counters, LDS bank
# conflicts, and HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) per kernel. usage: prof_c5.sh [form ...]
# forms: tile (default product form), range, single_pass (prof_cases.py --var1d-form: the test-only variant setter)
set -e
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
LDS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for form in ${@:-tile}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$form -o kt --output-format csv -- python tools/prof_cases.py c5 --var1d-form $form --reps 5 > gpurun_out/kt_$form.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/sq_$form -o pmc --output-format csv -- python tools/prof_cases.py c5 --var1d-form $form --reps 2 > gpurun_out/sq_$form.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $LDS -d gpurun_out/lds_$form -o pmc --output-format csv -- python tools/prof_cases.py c5 --var1d-form $form --reps 2 > gpurun_out/lds_$form.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/fetch_$form -o pmc --output-format csv -- python tools/prof_cases.py c5 --var1d-form $form --reps 2 > gpurun_out/fetch_$form.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/write_$form -o pmc --output-format csv -- python tools/prof_cases.py c5 --var1d-form $form --reps 2 > gpurun_out/write_$form.log 2>&1
  python tools/pmc_summary.py gpurun_out/sq_$form gpurun_out/lds_$form gpurun_out/fetch_$form gpurun_out/write_$form > gpurun_out/sum_$form.json
done
