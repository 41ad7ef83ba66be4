#!/bin/bash
# analysis: decode-kernel time per dictionary bit width (single-bw files, 20M rows)
TAG=${1:-sweep}; shift
BWS=${BWS:-"1 2 4 8 10 12 13 14 15 16 18 20"}
for bw in $BWS; do
  timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-pmc --rows ${ROWS:-25165824} --bw $bw "$@" > gpurun_out/${TAG}_bw$bw.json 2>&1 || exit 1
done
