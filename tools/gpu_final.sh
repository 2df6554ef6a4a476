#!/bin/bash
# Round-end measurement without the test run: bench line, rocprofv3 kernel stats of the
# bench (parts = 1), PMC passes + summary.  Raw traces are deleted on the box once
# summarised, so what comes back stays under gpurun's 64 MiB merge limit.
# usage: tools/gpu_final.sh TAG
set -u
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_BENCH:-0}" != "1" ]; then
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python -u bench.py --no-cpu --no-latency --steps 5 --warmup 2 --parts 1 --ingest-images 32768 > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
find gpurun_out/prof_$TAG -name '*kernel_trace.csv' -delete
bash tools/pmc_collect.sh gpurun_out/pmc_$TAG -- python -u bench.py --no-cpu --no-latency --ingest-images 0 --jpeg-images 512 --steps 2 --warmup 1 --batch-reps 1 --search-queries 4 --parts 1 || exit $?
python tools/pmc_summary.py gpurun_out/pmc_$TAG --json gpurun_out/pmc_$TAG/summary.json --latest gpurun_out/pmc_$TAG/pmc_latest.json > gpurun_out/pmc_$TAG/summary.txt
echo "pmc summary rc=$?"
rm -rf gpurun_out/pmc_$TAG/p[0-9]*/
du -sh gpurun_out
