#!/bin/bash
# Round-5 GPU session: optional pytest -k filter, then bench lines with their own rocprofv3 outputs.
# usage: tools/gpu_r04.sh TAG "CFGS" [pytest -k expr | ALL | NONE] [extra bench args...]
TAG=${1:-r04}; CFGS=${2:-c2}; K=${3:-NONE}; shift 3; EXTRA=("$@")
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
if [ "$K" != "NONE" ]; then
  if [ "$K" = "ALL" ]; then KA=(); else KA=(-k "$K"); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; echo "TESTS EXIT $rc" >> gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for c in $CFGS; do
  [ "$c" = "-" ] && continue
  PQG_BENCH_PROF_DIR=gpurun_out/${TAG}_prof timeout -k 10 600 python -u bench.py --config $c --steps 20 --warmup 3 "${EXTRA[@]}" \
    > gpurun_out/${TAG}_${c}_bench.json 2> gpurun_out/${TAG}_${c}_bench.err || exit 1
  echo "$c done" >&2
done
