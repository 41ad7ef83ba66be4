#!/bin/bash
# GPU parity suite (optionally a -k filter), then a C2 bench line without the profiler children
# usage: tools/gpu_quick.sh TAG [pytest -k expr]
TAG=${1:-quick}; K=${2:-}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${KA[@]}" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc" >> gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-prof --cpu-budget 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
