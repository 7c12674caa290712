set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/qx
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gguf_gpu.py tests/test_quant_moe_gpu.py tests/test_fused_decode_gpu.py > gpurun_out/qx/tests.log 2>&1 || { tail -30 gpurun_out/qx/tests.log; exit 1; }
tail -1 gpurun_out/qx/tests.log
timeout -k 10 200 python -u tools/bench_gguf.py --m 64 > gpurun_out/qx/gguf.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_gguf.py --m 64 --fp8 > gpurun_out/qx/fp8.log 2>&1 || exit 1
grep '^{' gpurun_out/qx/gguf.log gpurun_out/qx/fp8.log | cut -c1-160
timeout -k 10 300 python -u bench.py --path engine --quantization q4_k_m --steps 2 --warmup 1 > gpurun_out/qx/bench_q4.log 2>&1 || exit 1
tail -1 gpurun_out/qx/bench_q4.log | cut -c1-200
