#!/bin/bash
# analysis: k_expand with parts disabled (PQG_KNOB: 1 no gathers, 2 no stores, 3 neither)
for k in 0 1 2 3; do
  for bw in 2 20; do
    PQG_KNOB=$k timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-pmc --rows 20000000 --bw $bw > gpurun_out/knob${k}_bw$bw.json 2>&1 || exit 1
  done
  PQG_KNOB=$k timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-pmc > gpurun_out/knob${k}_full.json 2>&1 || exit 1
done
