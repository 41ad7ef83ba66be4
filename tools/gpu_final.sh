#!/bin/bash
# Round-end evidence: the GPU suite, then every config's bench line with its
# rocprofv3 kernel trace / stats and FETCH_SIZE / WRITE_SIZE passes.
# usage: tools/gpu_final.sh TAG "CFGS"
TAG=${1:-r05}; CFGS=${2:-"c1 c2 c3 c4 c5"}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
if [ "${SUITE:-1}" = "1" ]; then
  bash tools/gpu_suite.sh ${TAG} || exit 1
fi
bash tools/gpu_r05.sh ${TAG} "$CFGS" NONE || exit 1
