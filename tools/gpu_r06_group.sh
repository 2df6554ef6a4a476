#!/bin/bash
# Round-6: tile order (group_m) of QKV / fc1 — timing A/B, then one FETCH_SIZE pass per setting
set -u
export TMPDIR=/tmp
O=gpurun_out/r06p; mkdir -p $O
export RC_LIB_PATH=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib/diag/libretrieval_core.so
timeout -k 10 400 python -u tools/group_m_ab.py > $O/ab.log 2>&1; rc=$?; tail -1 $O/ab.log; [ $rc -ne 0 ] && exit $rc
for G in 8 4 2 16; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_g$G -o run --output-format csv -- python -u tools/group_m_ab.py --one $G > $O/pmc_g$G.log 2>&1 || exit $?
  python - "$O/pmc_g$G" "$G" <<'PY'
import csv, glob, sys, collections
vals = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "gemm_pp_kernel<5" in n or "gemm_pp_kernel<4" in n:
            vals[(n[:40], r["Grid_Size"])].append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    if len(v) >= 6:
        print("group", sys.argv[2], k, "launches", len(v), "read MB (2 x FETCH_SIZE KB)", round(2 * sum(v) / len(v) * 1024 / 1e6, 1))
PY
  find $O/pmc_g$G -name '*.csv' -size +1M -delete
done
