#!/bin/bash
# Collect PMC counters in separate rocprofv3 passes (one counter group per pass,
# kernel-trace only — never combined with sys/runtime traces).
# usage: tools/pmc_collect.sh OUTDIR -- python script.py args...
set -u
OUT=$1; shift; shift
export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for CTR in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $CTR -d "$OUT/p$i" -o run --output-format csv -- "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($CTR) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
