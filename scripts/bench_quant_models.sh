# refresh the quantised-model benches on the current tree (gateway path, 64 x 1024 / 256)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/qm
timeout -k 10 600 python -u bench.py --model qwen3-30b-a3b --quantization int8 --out gpurun_out/qm/qwen3_int8.json > gpurun_out/qm/qwen3_int8.log 2>&1 || { tail -5 gpurun_out/qm/qwen3_int8.log; exit 1; }
tail -1 gpurun_out/qm/qwen3_int8.log | cut -c1-200
timeout -k 10 600 python -u bench.py --model gemma-3-27b --quantization fp8 --out gpurun_out/qm/gemma_fp8.json > gpurun_out/qm/gemma_fp8.log 2>&1 || { tail -5 gpurun_out/qm/gemma_fp8.log; exit 1; }
tail -1 gpurun_out/qm/gemma_fp8.log | cut -c1-200
