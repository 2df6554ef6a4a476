set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_i8_filter_gpu.py tests/test_batched_search_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_i8a.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_i8a.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/i8_probe.py > gpurun_out/i8probe_a.json 2> gpurun_out/i8probe_a.err
rc=$?; cat gpurun_out/i8probe_a.json; tail -5 gpurun_out/i8probe_a.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_i8a -o run --output-format csv -- python -u tools/i8_probe.py --reps 2 > gpurun_out/prof_i8a.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
