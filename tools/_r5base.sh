set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
tools/gpu_quick.sh r5base && BWS="1 2 3 4 5 6 7 8 9 10 11 12 13 14 15 16 17 18 19 20" tools/bw_sweep.sh r5sw
