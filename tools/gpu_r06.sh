#!/bin/bash
# Round-6 GPU session helper: parity tests for a -k filter, then A/B lines.
# usage: tools/gpu_r06.sh TAG "pytest -k expr"   (then the caller's own steps)
TAG=${1:-r06}; K=${2:-}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread "${KA[@]}" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc" >> gpurun_out/${TAG}_tests.log; exit $rc
