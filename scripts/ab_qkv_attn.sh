# fused qkv partials -> RoPE + KV write + attention (prefetched first chunk, shared q) vs separate RoPE kernel
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/qa
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_decode_gpu.py > gpurun_out/qa/tests.log 2>&1 || { tail -30 gpurun_out/qa/tests.log; exit 1; }
tail -1 gpurun_out/qa/tests.log
for v in 1 0 1 0; do
  HIPSERVE_FUSED_QKV_ATTN=$v timeout -k 10 240 python -u tools/decode_gap.py > gpurun_out/qa/gap_$v.log 2>&1 || exit 1
  echo "fused=$v $(tail -1 gpurun_out/qa/gap_$v.log)"
done
