set -u
mkdir -p gpurun_out/r06s4
timeout -k 10 600 python -u -m pytest tests/test_dist.py tests/test_fullsize.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r06s4/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06s4/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/debug_suite.sh r06s4
