set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tp8
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_tp_gpu.py -k tp8 > gpurun_out/tp8/tests.log 2>&1
rc=$?; tail -25 gpurun_out/tp8/tests.log; exit $rc
