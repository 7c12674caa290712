# qgemm2 deep weight ring (HIPSERVE_QGEMM_M64=2, default) vs the two-set body (0): correctness, kernel, engine
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/deep
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gguf_gpu.py tests/test_quant_moe_gpu.py > gpurun_out/deep/tests.log 2>&1 || { tail -30 gpurun_out/deep/tests.log; exit 1; }
tail -2 gpurun_out/deep/tests.log
for v in 2 0; do
  HIPSERVE_QGEMM_M64=$v timeout -k 10 200 python -u tools/bench_gguf.py --m 64 > gpurun_out/deep/gguf_m64_v$v.log 2>&1 || exit 1
  HIPSERVE_QGEMM_M64=$v timeout -k 10 200 python -u tools/bench_gguf.py --m 64 --fp8 > gpurun_out/deep/fp8_m64_v$v.log 2>&1 || exit 1
done
for v in 2 0; do
  HIPSERVE_QGEMM_M64=$v timeout -k 10 300 python -u bench.py --path engine --quantization q4_k_m --steps 2 --warmup 1 > gpurun_out/deep/bench_q4_v$v.log 2>&1 || exit 1
  tail -1 gpurun_out/deep/bench_q4_v$v.log | cut -c1-200
done
timeout -k 10 200 python -u tools/bench_mall.py > gpurun_out/deep/mall.log 2>&1 || exit 1
cat gpurun_out/deep/mall.log
