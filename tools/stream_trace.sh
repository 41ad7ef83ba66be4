#!/bin/bash
# analysis: per-slice host phases of pqg_stream (PQG_TRACE_CREATE=1) and one
# whole-shard batch creation, on a bench config's file
# usage: tools/stream_trace.sh TAG CFG "rgs_per_slice ..." [depth]
TAG=${1:-st}; CFG=${2:-c1}; PERS=${3:-"1 5"}; DEPTH=${4:-8}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
F=$(python -c "import sys; sys.path.insert(0,'tools'); import synth; r,g=synth.DEFAULTS['$CFG']; print('/tmp/pqgpu_bench_%s_%d_%d_0.parquet' % ('$CFG', r, g))")
[ -f $F ] || timeout -k 10 300 python -c "import sys; sys.path.insert(0,'tools'); import synth; r,g=synth.DEFAULTS['$CFG']; synth.make('$CFG','$F',r,g)" || exit 1
for per in $PERS; do
  PQG_TRACE_CREATE=1 timeout -k 10 120 python -u tools/trace_stream.py $F $per $DEPTH > gpurun_out/${TAG}_${CFG}_p${per}.txt 2>&1 || exit 1
done
PQG_TRACE_CREATE=1 timeout -k 10 120 python -u - $F > gpurun_out/${TAG}_${CFG}_oneshot.txt 2>&1 <<'PY' || exit 1
import sys, time
sys.path.insert(0, "parquet-go_amd")
import pqgpu
r = pqgpu.FileReader(sys.argv[1])
r.batch(0, 1).close()
for rep in range(3):
    t = time.perf_counter(); b = r.batch(); tc = time.perf_counter() - t
    b.decode(); b.sync(); tt = time.perf_counter() - t
    print("one-shot %d: create %.2f ms, create+decode+sync %.2f ms" % (rep, tc * 1e3, tt * 1e3), flush=True)
    b.close()
PY
