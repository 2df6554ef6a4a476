#!/bin/bash
# Round-6 in-model A/B on the diagnostic build (same bits asserted): usage TAG VARIANTS
set -u
TAG=$1; V=$2
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
DIAG=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib/diag/libretrieval_core.so
for P in 2 1; do
RC_LIB_PATH=$DIAG VARIANTS=$V ROUNDS=4 STEPS=10 PARTS=$P timeout -k 10 500 python -u tools/gemm_ab.py > gpurun_out/$TAG/gemm_ab_p$P.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/gemm_ab_p$P.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
