#!/bin/bash
# Round-6: interleaved A/B of the product library against lib/ab_base (bench embed lines, parts 2)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/$1
P=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib
AB_PARTS=2 timeout -k 10 900 bash tools/ab_env.sh ${2:-4} "RC_LIB_PATH=$P/ab_base/libretrieval_core.so" "RC_LIB_PATH=$P/libretrieval_core.so" -- --no-latency > gpurun_out/$1/ab.log 2>&1
rc=$?; sed "s#$P/##g" gpurun_out/$1/ab.log; exit $rc
