# fused qkv attention on / off at long context (many decode partitions, small batches)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ql
for v in 0 1; do
  for cfg in "8k 8192 16" "32k 32768 4"; do
    set -- $cfg
    HIPSERVE_FUSED_QKV_ATTN=$v timeout -k 10 400 python -u bench.py --tp-phase off --model llama-3.1-8b --input-len $2 --output-len 256 \
      --concurrency $3 --max-num-batched-tokens 8192 --steps 2 --out gpurun_out/ql/b_$1_$v.json > gpurun_out/ql/b_$1_$v.log 2>&1 || { tail -20 gpurun_out/ql/b_$1_$v.log; exit 1; }
    echo "fused=$v ctx=$1 $(python -c "import json;d=json.load(open('gpurun_out/ql/b_$1_$v.json'));print(d['value'], d['p50_ttft_ms'])")"
  done
done
