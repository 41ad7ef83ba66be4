#!/bin/bash
# tests + bench (no cpu) + bw2/bw20 single-width files
TAG=${1:-q}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
echo "TESTS EXIT $?" >> gpurun_out/${TAG}_tests.log
timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-pmc > gpurun_out/${TAG}_bench.json 2>&1 || exit 1
for bw in 2 20; do
  timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-pmc --rows 20000000 --bw $bw > gpurun_out/${TAG}_bw$bw.json 2>&1 || exit 1
done
