export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03f_pytest.log 2>&1 || { tail -30 gpurun_out/r03f_pytest.log; exit 1; }
tail -2 gpurun_out/r03f_pytest.log
VARIANTS=104,105,107 ROLES=attention,qkv ROUNDS=5 STEPS=10 timeout -k 10 300 python -u tools/gemm_ab.py > gpurun_out/r03f_attn_ab.log 2>&1 || { tail -20 gpurun_out/r03f_attn_ab.log; exit 1; }
tail -1 gpurun_out/r03f_attn_ab.log
VARIANTS=104,105,107 ROLES=attention ROUNDS=1 STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03f -o run --output-format csv -- python -u tools/gemm_ab.py > gpurun_out/r03f_prof.log 2>&1
echo rocprof=$?
