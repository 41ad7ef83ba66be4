#!/bin/bash
# analysis: alternating A/B of the large-dictionary job weight in the XCD dealing (C2 decode phase)
TAG=${1:-xw}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for rep in 1 2; do
  for w in 1.0 1.5 2.0; do
    PQG_XCD_WHOLE_W=$w timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-prof > gpurun_out/${TAG}_r${rep}_w$w.json 2> gpurun_out/${TAG}_r${rep}_w$w.err || exit 1
  done
done
