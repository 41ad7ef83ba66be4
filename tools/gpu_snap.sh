#!/bin/bash
# parity tests, then short bench lines of the snappy-heavy configs (+ per-phase times)
TAG=${1:-snap}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc" >> gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit 1
for c in ${CFGS:-c3 c5 c2}; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --no-cpu --no-pmc > gpurun_out/${TAG}_${c}.json 2> gpurun_out/${TAG}_${c}.err || exit 1
  PQG_SEGMENT_TIMES=1 timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-pmc > gpurun_out/${TAG}_${c}_seg.json 2>&1 || exit 1
done
