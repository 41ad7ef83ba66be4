#!/bin/bash
# analysis: k_expand rows-per-wave variants on the bench workload and single-bw files
TAG=${1:-var}
for r in 8 16 32; do
  PQG_EX_ROWS=$r timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/${TAG}_r${r}.json 2>&1 || exit 1
  for bw in 2 20; do
    PQG_EX_ROWS=$r timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --rows 20000000 --bw $bw > gpurun_out/${TAG}_r${r}_bw$bw.json 2>&1 || exit 1
  done
done
