#!/bin/bash
# Round-6 batch-1 call: embed GPU tests, the latency probe (graphs on/off), the per-request kernel
# table under rocprofv3.  usage: tools/gpu_r06_lat.sh TAG [notests]
set -u
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
if [ "${2:-tests}" = "tests" ]; then
timeout -k 10 600 python -u -m pytest tests/test_embed_gpu.py tests/test_service.py tests/test_index_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/$TAG/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -u tools/search_image_breakdown.py > gpurun_out/$TAG/search_image.json 2> gpurun_out/$TAG/search_image.err
rc=$?; cat gpurun_out/$TAG/search_image.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/$TAG/search_image.err; exit $rc; }
timeout -k 10 300 python -u tools/embed_latency_probe.py > gpurun_out/$TAG/lat.json 2> gpurun_out/$TAG/lat.err
rc=$?; cat gpurun_out/$TAG/lat.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/$TAG/lat.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python -u tools/embed_latency_probe.py --trace-only > gpurun_out/$TAG/trace.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/trace.log; find gpurun_out/$TAG/prof -name '*kernel_trace.csv' -delete; exit $rc
