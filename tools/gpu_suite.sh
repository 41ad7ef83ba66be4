cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${1:-suite}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc" >> gpurun_out/${1:-suite}_tests.log; exit $rc
