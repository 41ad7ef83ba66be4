#!/bin/bash
# round-5 scratch: k_expand_wg after the readlane fix: focused parity, the high-word layout test, then variants
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
T=${1:-r5f}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_guard.py -x -q --timeout 120 --timeout-method thread \
  -k "c2_dict_bw12 or high_low_word or high or dictionary or golden or big or tiled" > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc" >> gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
for v in libpqgpu.so libpqgpu_wg12.so libpqgpu_wg8.so; do
  PQGPU_LIB=$v timeout -k 10 300 python -u bench.py --no-prof --no-parity --no-cpu > gpurun_out/${T}_c2_$v.json 2> gpurun_out/${T}_c2_$v.err || exit 1
  for bw in 13 15 16 17; do
    PQGPU_LIB=$v timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-prof --no-parity --rows 25165824 --bw $bw > gpurun_out/${T}_bw${bw}_$v.json 2>&1 || exit 1
  done
done
for g in 16 32; do
  PQG_WG_JOBS=$g timeout -k 10 300 python -u bench.py --no-prof --no-parity --no-cpu > gpurun_out/${T}_c2_g$g.json 2> gpurun_out/${T}_c2_g$g.err || exit 1
done
PQG_LD_MAX_KB=0 timeout -k 10 300 python -u bench.py --no-prof --no-parity --no-cpu > gpurun_out/${T}_ld0.json 2> gpurun_out/${T}_ld0.err || exit 1
