#!/bin/bash
# A/B of the ping-pong GEMM's alternating K order (RC_GEMM_KREV) on the batch-256
# shapes (tools/gemm_calib.py, ping-pong only) and on the embed line, interleaved.
# usage: tools/ab_krev.sh TAG
set -u
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/abk_$TAG.jsonl
: > "$OUT"
for r in 1 2; do
  for KR in 0 4 2; do
    RC_GEMM_KREV=$KR VARIANTS=4 ROUNDS=3 timeout -k 10 120 python -u tools/gemm_calib.py > gpurun_out/abk_calib_$KR.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/abk_calib_$KR.log').read().strip().splitlines()[-1]); print(json.dumps({'round': $r, 'krev': $KR, **{k: round(v['rc4']['ms_min']*1e3, 1) for k, v in d.items()}}))" | tee -a "$OUT"
    RC_GEMM_KREV=$KR timeout -k 10 120 python -u bench.py --no-cpu --no-search --ingest-images 0 --jpeg-images 0 --steps 20 \
      --warmup 3 > gpurun_out/abk_tmp.json 2> gpurun_out/abk_$TAG.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/abk_tmp.json')); print(json.dumps({'round': $r, 'krev': $KR, 'img_s': d['value'], 'fc1_ms': d['roofline']['avg_launch_ms']}))" | tee -a "$OUT"
  done
done
