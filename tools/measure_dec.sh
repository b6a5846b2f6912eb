#!/bin/bash
# C3 encode/decode and receive-side decoder measurement set (one GPU call): kernel trace + stats, HBM traffic
# (separate FETCH_SIZE / WRITE_SIZE passes) and two SQ counter passes over tools/prof_cases.py c3 vdec dmean.
# Outputs under gpurun_out/ and copies the summaries to profiles/TAG_*; usage: measure_dec.sh TAG   (e.g. r04)
set -e
TAG=${1:-r04}
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
CASES="c3 vdec dmean --reps 2"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/d_kt -o kt --output-format csv -- python tools/prof_cases.py $CASES > $O/d_kt.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/d_fetch -o pmc --output-format csv -- python tools/prof_cases.py $CASES > $O/d_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/d_write -o pmc --output-format csv -- python tools/prof_cases.py $CASES > $O/d_write.log 2>&1
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"
timeout -s KILL 240 rocprofv3 --pmc $SQ -d $O/d_sq -o pmc --output-format csv -- python tools/prof_cases.py $CASES > $O/d_sq.log 2>&1
SQ2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM"
timeout -s KILL 240 rocprofv3 --pmc $SQ2 -d $O/d_sq2 -o pmc --output-format csv -- python tools/prof_cases.py $CASES > $O/d_sq2.log 2>&1
python tools/pmc_summary.py $O/d_fetch $O/d_write > $O/${TAG}_dec_traffic_raw.json
python tools/pmc_summary.py $O/d_sq $O/d_sq2 > $O/${TAG}_dec_sq_counters.json
cp $O/d_kt/kt_kernel_stats.csv $O/${TAG}_dec_kernel_stats.csv
echo measure_dec done
