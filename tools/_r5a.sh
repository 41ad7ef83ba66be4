#!/bin/bash
# round-5 scratch: focused parity tests, C2 bench line, single-width decode times
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
T=${1:-r5a}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "dictionary or golden or big or tiled or c5_lineitem_shape" > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc" >> gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-prof --cpu-budget 1 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
BWS="${BWS:-13 14 15 16 17 18}" tools/bw_sweep.sh ${T}sw
PQG_LD_MAX_KB=0 timeout -k 10 300 python -u bench.py --no-prof --no-parity --no-cpu > gpurun_out/${T}_bench_ld0.json 2> gpurun_out/${T}_bench_ld0.err || exit 1
PQG_BIG_ORDER=2 timeout -k 10 300 python -u bench.py --no-prof --no-parity --no-cpu > gpurun_out/${T}_bench_side.json 2> gpurun_out/${T}_bench_side.err || exit 1
