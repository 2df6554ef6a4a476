#!/bin/bash
# Batch-1 /embed latency breakdown: the probe's phase timings, then a rocprofv3 kernel trace of
# 110 embed_bytes calls (per-kernel totals / 110 = device time per request).
# usage: tools/gpu_embedlat.sh TAG
set -u
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u tools/embed_latency_probe.py > gpurun_out/$TAG/embed_probe.json 2> gpurun_out/$TAG/embed_probe.err
rc=$?; cat gpurun_out/$TAG/embed_probe.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/$TAG/embed_probe.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/$TAG/prof_embed -o run --output-format csv -- python -u tools/embed_latency_probe.py --trace-only > gpurun_out/$TAG/embed_trace.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/embed_trace.log; exit $rc
