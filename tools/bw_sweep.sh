#!/bin/bash
# analysis: decode time per dictionary bit width (single-bw files, 20M rows)
for bw in 2 8 12 16 20; do
  timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --rows 20000000 --bw $bw > gpurun_out/sweep_bw$bw.json 2>&1 || exit 1
done
