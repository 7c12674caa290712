set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pattn
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill" > gpurun_out/pattn/tests.log 2>&1 || { tail -30 gpurun_out/pattn/tests.log; exit 1; }
tail -1 gpurun_out/pattn/tests.log
timeout -k 10 200 python -u tools/bench_ops.py prefill > gpurun_out/pattn/bench.log 2>&1 || exit 1
grep '^{' gpurun_out/pattn/bench.log
