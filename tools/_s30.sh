# round-end set, part 2: decoder / C3 measurement (measure_dec), then the bench line again
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/measure_dec.sh r05c
timeout -k 10 300 python bench.py > gpurun_out/r05c_bench2.log 2>&1
tail -c 300 gpurun_out/r05c_bench2.log
echo part2 done
