#!/bin/bash
# analysis: alternating A/B of the XCD split threshold on C2 (decode phase)
TAG=${1:-xcdab}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in 0 1024 512; do
    PQG_XCD_SPLIT_KB=$v timeout -k 10 200 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-prof > gpurun_out/${TAG}_r${rep}_split$v.json 2> gpurun_out/${TAG}_r${rep}_split$v.err || exit 1
  done
done
