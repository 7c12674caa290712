set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/dec
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_decode_gpu.py -k "decode" > gpurun_out/dec/tests.log 2>&1 || { tail -30 gpurun_out/dec/tests.log; exit 1; }
tail -1 gpurun_out/dec/tests.log
DECODE_COLD=1 DECODE_PARTS=2048 timeout -k 10 120 python -u tools/bench_ops.py decode > gpurun_out/dec/ops.log 2>&1 || exit 1
grep '^{' gpurun_out/dec/ops.log | head -3
timeout -k 10 240 python -u tools/decode_gap.py > gpurun_out/dec/gap.log 2>&1 || exit 1
tail -1 gpurun_out/dec/gap.log
