#!/bin/bash
# A/B of the embed path's concurrent batch slices (rc_model_set_parts) and the
# ping-pong GEMM tile grouping (RC_GEMM_GM), embed line only, interleaved rounds.
# usage: tools/ab_parts.sh TAG
set -u
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/ab_$TAG.jsonl
: > "$OUT"
for r in 1 2; do
  for P in 2 3 4; do
    timeout -k 10 120 python -u bench.py --no-cpu --no-search --ingest-images 0 --jpeg-images 0 --steps 20 --warmup 3 \
      --parts $P > gpurun_out/ab_tmp.json 2> gpurun_out/ab_$TAG.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_tmp.json')); print(json.dumps({'round': $r, 'parts': $P, 'gm': '', 'img_s': d['value'], 'ms': d['ms_per_step']}))" | tee -a "$OUT"
  done
  for GM in 0 4 16; do
    RC_GEMM_GM=$GM timeout -k 10 120 python -u bench.py --no-cpu --no-search --ingest-images 0 --jpeg-images 0 --steps 20 \
      --warmup 3 --parts 3 > gpurun_out/ab_tmp.json 2> gpurun_out/ab_$TAG.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_tmp.json')); print(json.dumps({'round': $r, 'parts': 3, 'gm': $GM, 'img_s': d['value'], 'ms': d['ms_per_step']}))" | tee -a "$OUT"
  done
done
