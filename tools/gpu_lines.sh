#!/bin/bash
# bench lines (no profiler children) and timelines of several configs
# usage: tools/gpu_lines.sh TAG "c2 c3 c4"
TAG=${1:-ln}; CFGS=${2:-"c2 c3 c4"}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for c in $CFGS; do
  timeout -k 10 300 python -u bench.py --config $c --no-prof --cpu-budget 1 > gpurun_out/${TAG}_${c}.json 2> gpurun_out/${TAG}_${c}.err || exit 1
  timeout -k 10 200 python tools/timeline.py $c > gpurun_out/${TAG}_tl_${c}.txt 2>&1 || exit 1
  echo "$c done" >&2
done
