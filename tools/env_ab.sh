#!/bin/bash
# Step time (and parity) of one config under several environment settings.
# usage: tools/env_ab.sh TAG CFG "none|VAR=v[,VAR2=v2] ..." [extra bench args]
# Each setting runs bench.py --no-prof --no-cpu once; the kernel trace of
# each run is kept when PROF=1 (rocprofv3 child, gpurun_out/TAG_prof_<i>/).
# The analysis knobs are read only by libpqgpu_analysis.so (make -C
# parquet-go_amd/csrc analysis), the library these runs load unless PQGPU_LIB
# names another.
TAG=$1; CFG=${2:-c2}; SETS=${3:-none}; shift 3
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
i=0
for set in $SETS; do
  envs=()
  [ "$set" != "none" ] && IFS=',' read -ra envs <<< "$set"
  noprof=--no-prof; pd=
  [ "${PROF:-0}" = "1" ] && noprof= && pd=gpurun_out/${TAG}_prof_$i
  env PQGPU_LIB=${PQGPU_LIB:-libpqgpu_analysis.so} "${envs[@]}" PQG_BENCH_PROF_DIR=$pd timeout -k 10 300 python -u bench.py --config $CFG --steps 20 --warmup 3 \
    --no-cpu $noprof "$@" > gpurun_out/${TAG}_${CFG}_$i.json 2> gpurun_out/${TAG}_${CFG}_$i.err
  rc=$?
  echo "[$i] $set rc=$rc $(python -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_${CFG}_$i.json').read().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['roofline'].get('frac'), d['config'].get('parity','')[:40])" 2>/dev/null)"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
  i=$((i+1))
done
exit 0
