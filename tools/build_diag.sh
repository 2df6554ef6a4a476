#!/bin/bash
# Diagnostic build (GEMM ablation variants, A/B knobs) into lib/diag/, loaded with RC_LIB_PATH.
# ONLY="vit index" rebuilds just those sources' objects before relinking.
set -eu
cd "$(dirname "$0")/.."
P=end-to-end-image-retrieval-service-with-k8s-jenkins_amd
mkdir -p $P/lib/diag/obj
pids=
for f in $P/csrc/*.hip; do
  b=$(basename $f .hip)
  if [ -n "${ONLY:-}" ] && ! echo " $ONLY " | grep -q " $b "; then continue; fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Iinclude -I$P/csrc -Wno-unused-result -munsafe-fp-atomics \
    -DRC_GEMM_ABLATION "$@" -c $f -o $P/lib/diag/obj/$(basename $f).o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/lib/diag/libretrieval_core.so $P/lib/diag/obj/*.o
echo built $P/lib/diag/libretrieval_core.so
