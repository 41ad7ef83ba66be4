#!/bin/bash
# LDS-group sizing A/B: PQG_LD_AMORT (group output >= AMORT x dictionary) at group minimum 4
TAG=${1:-gm}
for v in ${AMS:-4 2 1 4 2 1}; do
  PQG_LD_AMORT=$v timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-pmc > gpurun_out/${TAG}_$v.$RANDOM.json 2>&1 || exit 1
done
