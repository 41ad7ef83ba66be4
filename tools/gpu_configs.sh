#!/bin/bash
# Bench lines + rocprofv3 kernel stats for the non-headline configs.
# usage: tools/gpu_configs.sh TAG "c1 c3 c4 c5"
TAG=${1:-cfg}; CFGS=${2:-"c1 c3 c4 c5"}
mkdir -p gpurun_out
for c in $CFGS; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 2 > gpurun_out/${TAG}_${c}_bench.json 2> gpurun_out/${TAG}_${c}_bench.err || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${c}_prof -o run -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-pmc > gpurun_out/${TAG}_${c}_prof.log 2>&1 || exit 1
done
