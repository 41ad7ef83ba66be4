#!/bin/bash
# analysis: pqg_stream slice size / depth / workers on the C2 bench file
# usage: tools/stream_ab.sh TAG   (VARIANTS="per,depth,workers ..." to choose)
TAG=${1:-sab}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
F=/tmp/pqgpu_bench_c2_100000000_1048576_0.parquet
[ -f $F ] || timeout -k 10 300 python -c "import sys; sys.path.insert(0,'tools'); import synth; synth.make('c2','$F',100000000,1<<20)" || exit 1
VARIANTS=${VARIANTS:-"4,4,3 8,4,3 4,6,4 2,8,4 8,2,1"}
for v in $VARIANTS; do
  IFS=, read per depth workers <<< "$v"
  PQG_STREAM_WORKERS=$workers timeout -k 10 120 python -u tools/trace_stream.py $F $per $depth > gpurun_out/${TAG}_p${per}_d${depth}_w${workers}.txt 2>&1 || exit 1
done
