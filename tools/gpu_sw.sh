#!/bin/bash
# GPU session: a pytest -k subset, then one config's bench line (no profiler children) and its timeline
# usage: tools/gpu_sw.sh TAG CONFIG "pytest -k expr"
TAG=${1:-sw}; CFG=${2:-c5}; K=${3:-}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${KA[@]}" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc" >> gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config $CFG --no-prof --cpu-budget 1 > gpurun_out/${TAG}_${CFG}.json 2> gpurun_out/${TAG}_${CFG}.err || exit 1
timeout -k 10 200 python tools/timeline.py $CFG > gpurun_out/${TAG}_tl_${CFG}.txt 2>&1
