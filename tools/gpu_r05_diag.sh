#!/bin/bash
# Round-5 diagnostics: JPEG band kernel phase split (diagnostic build) and PMC counters of the
# batch-1 embed kernels (one counter group per rocprofv3 pass, kernel trace only).
# usage: tools/gpu_r05_diag.sh TAG [phase|nophase] [pmc|nopmc]
set -u
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
DIAG=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib/diag/libretrieval_core.so
if [ "${2:-phase}" = "phase" ]; then
RC_LIB_PATH=$DIAG timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$TAG/prof_phase -o run --output-format csv -- python -u tools/jpeg_phase.py > gpurun_out/$TAG/jpeg_phase.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/jpeg_phase.log; [ $rc -ne 0 ] && exit $rc
python tools/jpeg_phase.py --parse gpurun_out/$TAG/prof_phase/run_kernel_trace.csv > gpurun_out/$TAG/jpeg_phase.json; cat gpurun_out/$TAG/jpeg_phase.json
find gpurun_out/$TAG/prof_phase -name '*kernel_trace.csv' -delete
fi
if [ "${3:-pmc}" = "pmc" ]; then
i=0
for CTR in "TCC_HIT_sum TCC_MISS_sum" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES" "TA_BUSY_avr" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTR -d gpurun_out/$TAG/pmc_embed/p$i -o run --output-format csv -- python -u tools/embed_latency_probe.py --trace-only > gpurun_out/$TAG/pmc_embed/p$i.log 2>&1
  rc=$?
  echo "pass $i ($CTR) rc=$rc"
  [ $rc -ne 0 ] && { tail -3 gpurun_out/$TAG/pmc_embed/p$i.log; exit $rc; }
done
fi
exit 0
