#!/bin/bash
# r03b: GPU tests (patch GEMM byte conversion), PMC passes incl. VALU/LDS issue counters, kernel stats.
set -u
TAG=${1:-r03b}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/gemm_ab.py > gpurun_out/gemm_ab_$TAG.log 2>&1
echo "gemm_ab rc=$?"; tail -2 gpurun_out/gemm_ab_$TAG.log
SHORT="--no-cpu --no-latency --steps 2 --warmup 1 --batch-reps 1 --search-queries 4 --parts 1 --ingest-images 4096 --jpeg-images 64"
bash tools/pmc_collect.sh gpurun_out/pmc_$TAG -- python -u bench.py $SHORT || exit $?
python tools/pmc_summary.py gpurun_out/pmc_$TAG --json gpurun_out/pmc_$TAG/summary.json --latest gpurun_out/pmc_$TAG/pmc_latest.json > gpurun_out/pmc_$TAG/summary.txt
echo "pmc summary rc=$?"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python -u bench.py --no-cpu --no-latency --steps 5 --warmup 2 --parts 1 --ingest-images 32768 > gpurun_out/prof_$TAG.log 2>&1
echo "rocprof rc=$?"
