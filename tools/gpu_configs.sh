#!/bin/bash
# Bench lines (with their rocprofv3 kernel-stats summaries) for the configs.
# usage: tools/gpu_configs.sh TAG "c2 c1 c3 c4 c5" [extra bench args]
TAG=${1:-cfg}; CFGS=${2:-"c2 c1 c3 c4 c5"}; shift 2
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in $CFGS; do
  PQG_BENCH_PROF_DIR=gpurun_out/${TAG}_prof timeout -k 10 600 python -u bench.py --config $c --steps 10 --warmup 2 "$@" \
    > gpurun_out/${TAG}_${c}_bench.json 2> gpurun_out/${TAG}_${c}_bench.err || exit 1
  echo "$c done" >&2
done
