#!/bin/bash
# Round-end measurement set (one GPU call): C2 kernel trace + HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes)
# of the bench command, C5 traffic and SQ counters per encode, then the full bench line (which reads the traffic files
# just written). Outputs under gpurun_out/; usage: measure_round.sh TAG   (e.g. r03)
set -e
TAG=${1:-r03}
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/m_kt -o kt --output-format csv -- python bench.py --no-extras > $O/m_kt.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/m_fetch -o pmc --output-format csv -- python bench.py --no-extras > $O/m_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/m_write -o pmc --output-format csv -- python bench.py --no-extras > $O/m_write.log 2>&1
python tools/pmc_traffic.py k_encode_fixed1d_np c2_1d_fp32_fixed_rate16_256Mi_per_gpu $O/m_kt $O/m_fetch $O/m_write $O/${TAG} 5:20 > $O/m_traffic.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/c5_fetch -o pmc --output-format csv -- python tools/prof_cases.py c5 --reps 2 > $O/c5_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/c5_write -o pmc --output-format csv -- python tools/prof_cases.py c5 --reps 2 > $O/c5_write.log 2>&1
python tools/c5_traffic.py $O/c5_fetch $O/c5_write 2 $O/${TAG} > $O/c5_traffic.log
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
timeout -s KILL 120 rocprofv3 --pmc $SQ -d $O/c5_sq -o pmc --output-format csv -- python tools/prof_cases.py c5 --reps 2 > $O/c5_sq.log 2>&1
python tools/pmc_summary.py $O/c5_sq > $O/${TAG}_c5_sq_counters.json
cp $O/${TAG}_pmc_traffic.json $O/${TAG}_c2_kernel_stats.csv $O/${TAG}_c5_acc*_pmc_traffic.json profiles/ 2>/dev/null || true
cp $O/${TAG}_kernel_stats.csv profiles/${TAG}_c2_kernel_stats.csv 2>/dev/null || true
timeout -k 10 300 python bench.py > $O/m_bench.log 2>&1
echo measure_round done
