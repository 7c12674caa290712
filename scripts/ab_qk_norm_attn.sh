# Qwen3 per-head q/k norm inside the fused decode attention: kernel/model tests, then the
# Qwen3-30B-A3B INT8 bench with the fused attention on / off
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/qn
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_decode_gpu.py \
  > gpurun_out/qn/tests.log 2>&1 || { tail -40 gpurun_out/qn/tests.log; exit 1; }
tail -1 gpurun_out/qn/tests.log
for v in 1 0; do
  HIPSERVE_FUSED_QKV_ATTN=$v timeout -k 10 600 python -u bench.py --tp-phase off --model qwen3-30b-a3b --quantization int8 \
    --out gpurun_out/qn/bench_q3int8_$v.json > gpurun_out/qn/bench_$v.log 2>&1 || { tail -20 gpurun_out/qn/bench_$v.log; exit 1; }
  echo "fused=$v $(python -c "import json;d=json.load(open('gpurun_out/qn/bench_q3int8_$v.json'));print(d['value'], d.get('p50_ttft_ms'))")"
done
