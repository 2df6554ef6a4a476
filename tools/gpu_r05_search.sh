#!/bin/bash
# Config-3 diagnostics: kernel stats of the single-query scan path (search_micro under rocprofv3)
# and the scan lab's streaming ceiling for the 1M x 512 f32 load shape.
# usage: tools/gpu_r05_search.sh TAG
set -u
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_search -o run --output-format csv -- python -u tools/search_micro.py > gpurun_out/$TAG/search_micro.log 2>&1
rc=$?; grep dtype gpurun_out/$TAG/search_micro.log; find gpurun_out/$TAG/prof_search -name '*kernel_trace.csv' -delete; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/scan_lab/lab.py > gpurun_out/$TAG/scan_lab.json 2> gpurun_out/$TAG/scan_lab.err
rc=$?; cat gpurun_out/$TAG/scan_lab.json; [ $rc -ne 0 ] && tail -5 gpurun_out/$TAG/scan_lab.err
exit $rc
