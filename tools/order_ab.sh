#!/bin/bash
TAG=${1:-mo}
for v in ${ORS:-0 1 2 0 1 2}; do
  PQG_MIX_ORDER=$v timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-pmc > gpurun_out/${TAG}_$v.$RANDOM.json 2>&1 || exit 1
done
