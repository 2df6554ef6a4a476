#!/bin/bash
# Round-6: batch-1 A/B of the product library against lib/ab_base (tools/embed_b1_time.py, interleaved)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/$1
P=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib
for r in 1 2 3 4; do
  for L in ab_base/libretrieval_core.so libretrieval_core.so; do
    echo "$L $(RC_LIB_PATH=$P/$L timeout -k 10 120 python -u tools/embed_b1_time.py 2>/dev/null | tail -1)" | tee -a gpurun_out/$1/b1.log
  done
done
