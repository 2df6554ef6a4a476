#!/bin/bash
# Round-4 GPU call: GEMM lab (main-loop variants + stamps), the full -m gpu suite, smoke, bench.
# usage: tools/gpu_r04.sh TAG   (outputs under gpurun_out/TAG/)
set -u
TAG=$1
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/gemm_lab/lab.py --rounds 3 --variants ${LABV:-0,2,7,8,48} > $O/lab.log 2>&1
echo "lab rc=$?"; tail -2 $O/lab.log | cut -c1-200
VARIANTS=${ABV:-0,10} ROUNDS=3 STEPS=8 timeout -k 10 300 python -u tools/gemm_ab.py > $O/gemm_ab.log 2>&1
echo "gemm_ab rc=$?"; tail -1 $O/gemm_ab.log | cut -c1-600
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; cut -c1-600 $O/bench.json; [ $rc -ne 0 ] && tail -20 $O/bench.err
exit $rc
