#!/bin/bash
# analysis: Snappy segmentation threshold (PQG_SNAPPY_SEG_MIN) on a config's step
# usage: tools/seg_ab.sh TAG CONFIG "thresholds..."
TAG=${1:-seg}; CFG=${2:-c5}; TH=${3:-"0 262144 524288"}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for t in $TH; do
  if [ "$t" = "0" ]; then unset PQG_SNAPPY_SEG_MIN; else export PQG_SNAPPY_SEG_MIN=$t; fi
  timeout -k 10 300 python -u bench.py --config $CFG --steps 10 --warmup 2 --no-cpu --no-prof > gpurun_out/${TAG}_${CFG}_$t.json 2> gpurun_out/${TAG}_${CFG}_$t.err || exit 1
  timeout -k 10 300 python tools/timeline.py $CFG > gpurun_out/${TAG}_${CFG}_tl_$t.txt 2>&1 || exit 1
done
