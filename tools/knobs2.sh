#!/bin/bash
for k in 5 4 3 0; do
  for bw in 2 20; do
    PQG_KNOB=$k timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-pmc --rows 20000000 --bw $bw > gpurun_out/knob${k}_bw$bw.json 2>&1 || exit 1
  done
done
