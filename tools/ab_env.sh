#!/bin/bash
# Interleaved A/B of embed throughput under different settings.
# usage: tools/ab_env.sh ROUNDS "VAR=a --flag" "VAR=b" ... [-- extra bench args]
# A setting's VAR=value words go to the environment, its --words to bench.py.
# Prints one line per run: setting, parts, images/s, ms/step.  AB_PARTS="2" limits the parts settings.
set -u
ROUNDS=$1; shift
SETS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SETS+=("$1"); shift; done
[ $# -gt 0 ] && shift
mkdir -p gpurun_out
for r in $(seq "$ROUNDS"); do
  for s in "${SETS[@]}"; do
    for parts in ${AB_PARTS:-1 2}; do
      ev=(); fl=()
      for w in $s; do case $w in --*) fl+=("$w");; *) ev+=("$w");; esac; done
      out=$(env "${ev[@]}" timeout -k 10 300 python -u bench.py --no-cpu --no-search --ingest-images 0 --jpeg-images 0 \
            --steps 30 --warmup 3 --parts $parts "${fl[@]}" "$@" 2>gpurun_out/ab_err.log) || { echo "FAIL $s"; tail -5 gpurun_out/ab_err.log; exit 1; }
      echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$s', 'parts=$parts', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms']*1e3,1))"
    done
  done
done
