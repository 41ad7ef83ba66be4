cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "snappy or Snappy or c5 or guard or mix or golden" > gpurun_out/r04i_tests.log 2>&1 || { tail -30 gpurun_out/r04i_tests.log; exit 1; }
tail -2 gpurun_out/r04i_tests.log
PROF=1 bash tools/env_ab.sh r04c5tl c5 "none PQGPU_LIB=libpqgpu_tok0.so PQGPU_LIB=libpqgpu_sh8.so PQGPU_LIB=libpqgpu_sh32.so" > gpurun_out/r04c5tl_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c5tl_summary.txt
PROF=1 bash tools/env_ab.sh r04c3tl c3 "none PQGPU_LIB=libpqgpu_sh8.so PQGPU_LIB=libpqgpu_sh32.so" > gpurun_out/r04c3tl_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c3tl_summary.txt
