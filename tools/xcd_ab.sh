#!/bin/bash
# analysis: C2 decode phase with L1/L2 chunks split over XCD residues or kept whole
TAG=${1:-xcd}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for v in ${SPLITS:-0 1024 4096}; do
  PQG_XCD_SPLIT_KB=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-prof > gpurun_out/${TAG}_split$v.json 2> gpurun_out/${TAG}_split$v.err || exit 1
done
