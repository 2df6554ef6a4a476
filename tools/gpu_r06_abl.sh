#!/bin/bash
# Round-6 in-model ablations on the diagnostic build (bits change on purpose: NOCHECK=1):
# usage: tools/gpu_r06_abl.sh TAG VARIANTS [PARTS]
set -u
TAG=$1; V=$2; P=${3:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
DIAG=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib/diag/libretrieval_core.so
RC_LIB_PATH=$DIAG NOCHECK=1 VARIANTS=$V ROUNDS=4 STEPS=10 PARTS=$P timeout -k 10 500 python -u tools/gemm_ab.py > gpurun_out/$TAG/gemm_ab.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/gemm_ab.log; exit $rc
