#!/bin/bash
# C2 bench with the built library, then with each variant library (LIBS) in its place
TAG=${1:-lab}
run() {
  for v in "PQG_NO_LDS_DICT=1 PQG_OLD_EXPAND=1" "PQG_LD_MAX_KB=32"; do
    n=$(echo "x$v" | tr -c 'a-zA-Z0-9\n' '_')
    env $v timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-pmc > gpurun_out/${TAG}_$1$n.json 2>&1 || exit 1
  done
}
run base
for l in ${LIBS:-v1}; do
  cp parquet-go_amd/libpqgpu_$l.so parquet-go_amd/libpqgpu.so && run $l || exit 1
done
