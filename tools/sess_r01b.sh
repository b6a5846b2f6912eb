tools/gpu_session.sh \
 "600|pytest_gpu|python -m pytest tests -m gpu -q -x -p no:cacheprovider --durations=8" \
 "300|bench_v0|GCOW_FIXED1D_VARIANT=0 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-e2e" \
 "300|bench_v1|GCOW_FIXED1D_VARIANT=1 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-e2e" \
 "300|prof_kt|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host-e2e" \
 "300|prof_fetch|rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e" \
 "300|prof_write|rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e" \
 "300|prof_sq|rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/prof_sq -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-e2e"
