#!/bin/bash
# Round-6: nontemporal C stores (ABL 32) in the bf16 epilogues — in-model A/B, then FETCH/WRITE per launch
set -u
export TMPDIR=/tmp
O=gpurun_out/r06q; mkdir -p $O
export RC_LIB_PATH=$PWD/end-to-end-image-retrieval-service-with-k8s-jenkins_amd/lib/diag/libretrieval_core.so
VARIANTS=12,132 ROUNDS=4 STEPS=10 PARTS=2 timeout -k 10 400 python -u tools/gemm_ab.py > $O/ab_p2.log 2>&1; rc=$?; tail -1 $O/ab_p2.log; [ $rc -ne 0 ] && exit $rc
for V in 12 132; do
  for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C -d $O/pmc_${V}_$C -o run --output-format csv -- python -u tools/gemm_ab_one.py $V > $O/pmc_${V}_$C.log 2>&1 || exit $?
  python - "$O/pmc_${V}_$C" "$V $C" <<'PY'
import csv, glob, sys, collections
vals = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "gemm_pp_kernel" in n and r["Grid_Size"] in ("1210368", "907776", "302592"):
            vals[(n[:40], r["Grid_Size"])].append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    print(sys.argv[2], k, "launches", len(v), "MB per launch", round(sum(v) / len(v) * 1024 / 1e6, 1))
PY
  find $O/pmc_${V}_$C -name '*.csv' -size +1M -delete
  done
done
