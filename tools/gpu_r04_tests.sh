#!/bin/bash
# Round-4 validation call: the full -m gpu suite, smoke, bench (outputs under gpurun_out/TAG/).
# usage: tools/gpu_r04_tests.sh TAG
set -u
TAG=$1
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; cut -c1-600 $O/bench.json; [ $rc -ne 0 ] && tail -20 $O/bench.err
exit $rc
