#!/bin/bash
# Round-6 GPU call: selected -m gpu tests, the precision probe, and an interleaved A/B of the
# product library against a saved one (lib/<AB_BASE>/), embed-only bench lines at parts = 2.
# usage: tools/gpu_r06.sh TAG "TEST FILES" [AB_BASE]
set -u
TAG=$1; TESTS=$2; BASE=${3:-}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
P=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib
if [ -n "$TESTS" ]; then
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/$TAG/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$BASE" ]; then
timeout -k 10 300 python -u tools/precision_probe.py > gpurun_out/$TAG/precision.log 2>&1
rc=$?; tail -2 gpurun_out/$TAG/precision.log; [ $rc -ne 0 ] && exit $rc
AB_PARTS=2 timeout -k 10 900 bash tools/ab_env.sh 3 "RC_LIB_PATH=$P/$BASE/libretrieval_core.so" "RC_LIB_PATH=$P/libretrieval_core.so" -- --no-latency > gpurun_out/$TAG/ab.log 2>&1
rc=$?; cat gpurun_out/$TAG/ab.log | sed "s#$P/##g"; exit $rc
fi
