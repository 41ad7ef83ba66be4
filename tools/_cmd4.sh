cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1 || { tail -30 gpurun_out/r04d_tests.log; exit 1; }
tail -2 gpurun_out/r04d_tests.log
PROF=1 bash tools/env_ab.sh r04c2pq c2 "none PQGPU_LIB=libpqgpu_prepser.so" > gpurun_out/r04c2pq_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c2pq_summary.txt
PROF=1 bash tools/env_ab.sh r04c3lv c3 "none PQGPU_LIB=libpqgpu_lvnow.so PQGPU_LIB=libpqgpu_lvwpe1.so" > gpurun_out/r04c3lv_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c3lv_summary.txt
PROF=1 bash tools/env_ab.sh r04c4lv c4 "PQG_NEST_PART=4096 PQG_NEST_PART=4096,PQGPU_LIB=libpqgpu_lvnow.so PQG_NEST_PART=4096,PQGPU_LIB=libpqgpu_lvwpe1.so PQG_NEST_PART=4096,PQGPU_LIB=libpqgpu_dictoff.so none PQG_NEST_PART=16384" > gpurun_out/r04c4lv_summary.txt 2>&1 || exit 1
cat gpurun_out/r04c4lv_summary.txt
PQG_SNAPPY_V1=1 timeout -k 10 300 python -u tools/diag_snappy.py c3 > gpurun_out/r04sd1_c3.txt 2>&1 || exit 1
PQG_SNAPPY_V1=1 timeout -k 10 300 python -u tools/diag_snappy.py c5 > gpurun_out/r04sd1_c5.txt 2>&1 || exit 1
