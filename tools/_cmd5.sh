cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1 || { tail -30 gpurun_out/r04e_tests.log; exit 1; }
tail -2 gpurun_out/r04e_tests.log
PROF=1 bash tools/env_ab.sh r04c3far c3 "none PQGPU_LIB=libpqgpu_farnow.so" > gpurun_out/r04c3far_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c3far_summary.txt
PROF=1 bash tools/env_ab.sh r04c5far c5 "none PQGPU_LIB=libpqgpu_farnow.so PQGPU_LIB=libpqgpu_dictoff.so" > gpurun_out/r04c5far_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c5far_summary.txt
PROF=1 bash tools/env_ab.sh r04c4d c4 "none PQGPU_LIB=libpqgpu_dictoff.so" > gpurun_out/r04c4d_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c4d_summary.txt
