# fused qkv attention gated to one context partition: tests, headline decode step, long-context A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/op
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_decode_gpu.py \
  > gpurun_out/op/tests.log 2>&1 || { tail -40 gpurun_out/op/tests.log; exit 1; }
tail -1 gpurun_out/op/tests.log
timeout -k 10 240 python -u tools/decode_gap.py > gpurun_out/op/gap.log 2>&1 || { tail -20 gpurun_out/op/gap.log; exit 1; }
echo "headline decode $(tail -1 gpurun_out/op/gap.log)"
bash scripts/ab_qkv_attn_long.sh
