cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "list or nest or part or level or corrupt or key" > gpurun_out/r04c_tests.log 2>&1 || { tail -30 gpurun_out/r04c_tests.log; exit 1; }
tail -2 gpurun_out/r04c_tests.log
PROF=1 bash tools/env_ab.sh r04c4p c4 "none PQG_PART_RESCAN=1 PQG_NEST_PART=4096 PQG_NEST_PART=2048 PQG_NEST_PART=1024" > gpurun_out/r04c4p_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c4p_summary.txt
PROF=1 bash tools/env_ab.sh r04c2lc c2 "none PQG_LEVEL_CHECK=1" > gpurun_out/r04c2lc_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c2lc_summary.txt
PROF=1 bash tools/env_ab.sh r04c3b c3 "none PQG_LEVEL_BYTES=1" > gpurun_out/r04c3b_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c3b_summary.txt
PROF=1 bash tools/env_ab.sh r04c2pp c2 "none PQGPU_LIB=libpqgpu_prepser.so" > gpurun_out/r04c2pp_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c2pp_summary.txt
