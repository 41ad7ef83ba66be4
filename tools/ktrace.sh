#!/bin/bash
# kernel trace of a short bench run: per-dispatch durations (tools/ktrace_summary.py)
TAG=${1:-kt}; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG} -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-pmc "$@" > gpurun_out/${TAG}.log 2>&1
