#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel-trace stats of the bench.
# usage: tools/gpu_round.sh TAG [bench args...]
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
echo "TESTS EXIT $?" >> gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-pmc > gpurun_out/${TAG}_prof.log 2>&1
echo "PROF EXIT $?" >> gpurun_out/${TAG}_prof.log
