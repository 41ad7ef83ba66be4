cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
PQG_SNAPPY_V1=1 timeout -k 10 300 python -u tools/diag_snappy.py c3 > gpurun_out/r04sd1_c3.txt 2>&1 || exit 1
PQG_SNAPPY_V1=1 timeout -k 10 300 python -u tools/diag_snappy.py c5 > gpurun_out/r04sd1_c5.txt 2>&1 || exit 1
