#!/bin/bash
# GPU tests + a quick bench (per-GEMM HIP-event times) + kernel stats of the bench
set -u
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_embed_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h_pytest.log 2>&1 || { tail -40 gpurun_out/r03h_pytest.log; exit 1; }
tail -1 gpurun_out/r03h_pytest.log
timeout -k 10 400 python -u bench.py --no-cpu --no-latency --ingest-images 32768 > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err || { tail -20 gpurun_out/r03h_bench.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/r03h_bench.json'))
print(d['value'], d['ms_per_step'], d['model_mfma_frac'], {k: round(v['avg_launch_ms']*1e3,1) for k,v in d['gemms'].items()}, d['attention_avg_launch_ms'])"
