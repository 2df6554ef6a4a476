#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only) over tools/jpeg_probe.py:
# the band kernel's instruction mix, waits and HBM bytes.  usage: tools/gpu_jpeg_pmc.sh TAG
set -u
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG/pmc_jpeg
i=0
for CTR in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTR -d gpurun_out/$TAG/pmc_jpeg/p$i -o run --output-format csv -- python -u tools/jpeg_probe.py > gpurun_out/$TAG/pmc_jpeg/p$i.log 2>&1
  rc=$?
  echo "pass $i ($CTR) rc=$rc"
  [ $rc -ne 0 ] && { tail -3 gpurun_out/$TAG/pmc_jpeg/p$i.log; exit $rc; }
done
exit 0
