tools/gpu_session.sh \
 "600|pytest_gpu|python -m pytest tests -m gpu -q -x -p no:cacheprovider -k 'fast1d or c2 or fixture or golden or subnormal or bf16 or tiny'" \
 "300|bench_v1|GCOW_FIXED1D_VARIANT=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-e2e" \
 "300|bench_v2|GCOW_FIXED1D_VARIANT=2 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-e2e" \
 "300|prof_sq2|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/prof_sq2 -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e" \
 "300|prof_grbm2|rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/prof_grbm2 -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e"
