#!/bin/bash
# Round-5 GPU call: -m gpu suite, bench line, in-model A/Bs on the diagnostic build: the
# residual-producer GEMM tiles (10 image-aligned 224-row, 8 two-workgroup 128x256, 4 ping-pong
# 256x256) and the attention form (2 = v2, 3 = v3).
# usage: tools/gpu_r05.sh TAG [tests|notests] [bench|nobench] [ab|noab] [jpeg|nojpeg]
set -u
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
DIAG=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib/diag/libretrieval_core.so
if [ "${2:-tests}" = "tests" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/$TAG/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "${3:-bench}" = "bench" ]; then
timeout -k 10 600 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?; head -c 3000 gpurun_out/$TAG/bench.json; echo; [ $rc -ne 0 ] && { tail -20 gpurun_out/$TAG/bench.err; exit $rc; }
fi
if [ "${5:-jpeg}" = "jpeg" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_jpeg -o run --output-format csv -- python -u tools/jpeg_probe.py > gpurun_out/$TAG/jpeg_probe.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/jpeg_probe.log; find gpurun_out/$TAG/prof_jpeg -name '*kernel_trace.csv' -delete; [ $rc -ne 0 ] && exit $rc
fi
if [ "${4:-ab}" = "ab" ]; then
RC_LIB_PATH=$DIAG ROUNDS=5 STEPS=10 PARTS=2 timeout -k 10 300 python -u tools/attn_ab.py > gpurun_out/$TAG/attn_ab_p2.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/attn_ab_p2.log; [ $rc -ne 0 ] && exit $rc
RC_LIB_PATH=$DIAG VARIANTS=${GV:-12,11,10} ROUNDS=5 STEPS=10 PARTS=2 timeout -k 10 400 python -u tools/gemm_ab.py > gpurun_out/$TAG/gemm_ab_p2.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/gemm_ab_p2.log; [ $rc -ne 0 ] && exit $rc
RC_LIB_PATH=$DIAG VARIANTS=${GV:-12,11,10} ROUNDS=5 STEPS=10 PARTS=1 timeout -k 10 400 python -u tools/gemm_ab.py > gpurun_out/$TAG/gemm_ab_p1.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/gemm_ab_p1.log; exit $rc
fi
