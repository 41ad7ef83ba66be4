#!/bin/bash
# analysis: k_expand_big placement on C2 (decode phase per variant) + stream trace
TAG=${1:-bigab}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
F=/tmp/pqgpu_bench_c2_100000000_1048576_0.parquet
for v in "PQG_NO_BIG=1" "PQG_BIG=1 PQG_BIG_ORDER=0" "PQG_BIG=1 PQG_BIG_ORDER=1" "PQG_BIG=1 PQG_BIG_ORDER=2"; do
  env $v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-prof > "gpurun_out/${TAG}_${v// /_}.json" 2> "gpurun_out/${TAG}_${v// /_}.err" || exit 1
done
for v in "PQG_NO_BIG=1" "PQG_BIG=1 PQG_BIG_ORDER=0" "PQG_BIG=1 PQG_BIG_ORDER=2"; do
  env $v timeout -k 10 200 python -u tools/timeline.py c2 > "gpurun_out/${TAG}_tl_${v// /_}.txt" 2>&1 || exit 1
done
PQG_TRACE_CREATE=1 timeout -k 10 120 python -u tools/trace_stream.py $F 8 2 > gpurun_out/${TAG}_stream.txt 2>&1 || exit 1
