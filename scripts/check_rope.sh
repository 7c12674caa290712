set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/rope
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rope" > gpurun_out/rope/tests.log 2>&1 || { tail -30 gpurun_out/rope/tests.log; exit 1; }
tail -1 gpurun_out/rope/tests.log
for t in 1 0; do HIPSERVE_ROPE_TILE=$t timeout -k 10 100 python -u tools/bench_rope.py >> gpurun_out/rope/bench.log 2>&1 || exit 1; done
grep '^{' gpurun_out/rope/bench.log
