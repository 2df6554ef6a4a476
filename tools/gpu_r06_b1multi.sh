#!/bin/bash
# Round-6: interleaved batch-1 A/B of several libraries (lib/<name>/libretrieval_core.so, "." = product)
# usage: tools/gpu_r06_b1multi.sh OUT ROUNDS name1 name2 ...
set -u
export TMPDIR=/tmp
OUT=$1; R=$2; shift 2
mkdir -p gpurun_out/$OUT
P=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib
for r in $(seq $R); do
  for n in "$@"; do
    res=$(RC_LIB_PATH=$P/$n/libretrieval_core.so timeout -k 10 120 python -u tools/embed_b1_time.py 2>gpurun_out/$OUT/err.log | tail -1) || { echo "FAIL $n"; tail -5 gpurun_out/$OUT/err.log; exit 1; }
    echo "$n $res" | tee -a gpurun_out/$OUT/b1.log
  done
done
