#!/bin/bash
# Round-6: per-kernel rocprofv3 stats of tools/embed_b1_time.py for lib/<name> libraries ("." = product)
set -u
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p gpurun_out/$OUT
P=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib
for n in "$@"; do
  d=gpurun_out/$OUT/prof_$(echo $n | tr -d ./)x
  RC_LIB_PATH=$P/$n/libretrieval_core.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 tools/embed_b1_time.py > gpurun_out/$OUT/prof_$(echo $n | tr -d ./)x.log 2>&1 || exit 1
done
find gpurun_out/$OUT -name "*kernel_stats.csv" | head
