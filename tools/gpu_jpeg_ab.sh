#!/bin/bash
# A/B of band-kernel builds (diagnostic libraries, mask 0 = the product arithmetic): per-launch
# medians of the 256 fixture-shaped JPEG batch under each library.
# usage: tools/gpu_jpeg_ab.sh TAG LIB_DIR... (dirs under the package's lib/)
set -u
TAG=$1; shift
export TMPDIR=/tmp RC_PHASE_MASKS=${RC_PHASE_MASKS:-0}
mkdir -p gpurun_out/$TAG
P=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib
for rep in 1 2; do
for L in "$@"; do
  RC_LIB_PATH=$P/$L/libretrieval_core.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/$TAG/p_${L}_$rep -o run --output-format csv -- python -u tools/jpeg_phase.py > gpurun_out/$TAG/${L}_$rep.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -3 gpurun_out/$TAG/${L}_$rep.log; exit $rc; }
  echo "$L rep $rep: $(python tools/jpeg_phase.py --parse gpurun_out/$TAG/p_${L}_$rep/run_kernel_trace.csv)"
  find gpurun_out/$TAG/p_${L}_$rep -name '*kernel_trace.csv' -delete
done
done
