set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c
DIAG=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib/diag/libretrieval_core.so
RC_LIB_PATH=$DIAG VARIANTS=12,13,14,4,10 ROUNDS=4 STEPS=10 PARTS=2 timeout -k 10 400 python -u tools/gemm_ab.py > gpurun_out/r06c/gemm_ab_p2.log 2>&1
rc=$?; tail -1 gpurun_out/r06c/gemm_ab_p2.log; [ $rc -ne 0 ] && exit $rc
RC_LIB_PATH=$DIAG VARIANTS=12,13,14,4,10 ROUNDS=4 STEPS=10 PARTS=1 timeout -k 10 400 python -u tools/gemm_ab.py > gpurun_out/r06c/gemm_ab_p1.log 2>&1
rc=$?; tail -1 gpurun_out/r06c/gemm_ab_p1.log; exit $rc
