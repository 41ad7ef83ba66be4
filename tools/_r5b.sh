#!/bin/bash
# round-5 scratch: C2 bench lines with the bench's own rocprofv3 kernel trace (default, NO_BIG), one-shot stall A/B
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
T=${1:-r5b}
PQG_BENCH_PROF_DIR=gpurun_out/${T}_prof timeout -k 10 300 python -u bench.py --no-parity --cpu-budget 1 > gpurun_out/${T}_c2.json 2> gpurun_out/${T}_c2.err || exit 1
PQG_NO_BIG=1 PQG_BENCH_PROF_DIR=gpurun_out/${T}_profnb timeout -k 10 300 python -u bench.py --no-parity --no-cpu > gpurun_out/${T}_c2nb.json 2> gpurun_out/${T}_c2nb.err || exit 1
PQG_LD_MAX_KB=0 PQG_RING_POLL=1 timeout -k 10 300 python -u bench.py --no-prof --no-parity --no-cpu > gpurun_out/${T}_ld0poll.json 2> gpurun_out/${T}_ld0poll.err || exit 1
PQG_LD_MAX_KB=0 timeout -k 10 300 python -u bench.py --no-prof --no-parity --no-cpu > gpurun_out/${T}_ld0.json 2> gpurun_out/${T}_ld0.err || exit 1
