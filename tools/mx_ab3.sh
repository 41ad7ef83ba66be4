#!/bin/bash
# GPU tests, then the C2 bench under LDS-dictionary caps
TAG=${1:-mx}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
for v in "PQG_LD_MAX_KB=32" "PQG_LD_MAX_KB=22" "PQG_LD_MAX_KB=26" "PQG_LD_MAX_KB=32"; do
  n=$(echo "x$v" | tr -c 'a-zA-Z0-9\n' '_')
  env $v timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-pmc > gpurun_out/${TAG}_bench$n.json 2>&1 || exit 1
  cp gpurun_out/${TAG}_bench$n.json gpurun_out/${TAG}_bench$n.$RANDOM.json
done
