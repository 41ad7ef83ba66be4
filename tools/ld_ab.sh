#!/bin/bash
# GPU tests, then the C2 bench and single-width files with / without k_expand_ld
TAG=${1:-ld}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-pmc > gpurun_out/${TAG}_bench.json 2>&1 || exit 1
PQG_NO_LDS_DICT=1 timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-pmc > gpurun_out/${TAG}_bench_nold.json 2>&1 || exit 1
for bw in ${BWS:-8 12 14 15}; do
  timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-pmc --rows 20000000 --bw $bw > gpurun_out/${TAG}_bw$bw.json 2>&1 || exit 1
  PQG_NO_LDS_DICT=1 timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-pmc --rows 20000000 --bw $bw > gpurun_out/${TAG}_bw${bw}_nold.json 2>&1 || exit 1
done
