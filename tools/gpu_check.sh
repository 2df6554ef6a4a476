#!/bin/bash
# One GPU call: parity tests, bench line, rocprofv3 kernel-trace stats of the bench.
# usage: tools/gpu_check.sh TAG [bench args...]
set -u
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python -u bench.py --no-cpu --no-latency --steps 5 --warmup 2 --parts 1 --ingest-images 32768 > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
