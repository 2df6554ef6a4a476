#!/bin/bash
# Round measurement on one GPU box: parity tests, bench line, kernel-trace stats,
# then PMC passes (separate runs, kernel-trace only) over a short bench.
# usage: tools/gpu_round.sh TAG
set -u
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh "$TAG" || exit $?
bash tools/pmc_collect.sh gpurun_out/pmc_$TAG -- python -u bench.py --no-cpu --steps 2 --warmup 1 --batch-reps 1 --search-queries 4 --parts 1 || exit $?
python tools/pmc_summary.py gpurun_out/pmc_$TAG --json gpurun_out/pmc_$TAG/summary.json --latest gpurun_out/pmc_$TAG/pmc_latest.json > gpurun_out/pmc_$TAG/summary.txt
echo "pmc summary rc=$?"
