#!/bin/bash
# analysis: decode phase per dictionary bit width under LDS-group size limits
# (PQG_LD_MAX_KB), single-bw files
TAG=${1:-ld}; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
LDS=${LDS:-"32 96 160"}; BWS=${BWS:-"13 14 15"}
for ld in $LDS; do
  for bw in $BWS; do
    PQGPU_LIB=${PQGPU_LIB:-libpqgpu_analysis.so} PQG_LD_MAX_KB=$ld timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-prof --rows ${ROWS:-25165824} --bw $bw "$@" \
      > gpurun_out/${TAG}_ld${ld}_bw$bw.json 2> gpurun_out/${TAG}_ld${ld}_bw$bw.err || exit 1
  done
done
