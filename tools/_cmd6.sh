cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1 || { tail -30 gpurun_out/r04f_tests.log; exit 1; }
tail -2 gpurun_out/r04g_tests.log
PROF=1 bash tools/env_ab.sh r04c3bo c3 "none PQG_LEVEL_BYTES=1 PQG_LEVELS_LATE=1" > gpurun_out/r04c3bo_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c3bo_summary.txt
