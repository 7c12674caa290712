#!/bin/bash
# One gpurun call: GPU tests, smoke, decode-GEMM sweep, 1-GPU bench, rocprofv3 kernel stats.
# usage (from the build container):
#   gpurun --timeout 1100 -- 'bash scripts/gpu_check.sh [tests|bench|prof|sweep ...]'
# Every GPU step has its own time limit and the steps are chained with &&:
# the first failure / timeout ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export PYTHONUNBUFFERED=1
steps="${*:-tests smoke sweep bench prof}"

run_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
  local rc=$?
  tail -n 15 $OUT/pytest_gpu.log
  return $rc
}
run_one() {  # one GPU test file
  local n; n=$(basename "$1" .py)
  timeout -k 10 300 python -u -m pytest "$1" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/$n.log 2>&1
  local rc=$?; tail -n 15 $OUT/$n.log; return $rc
}
run_smoke() {
  timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  local rc=$?; tail -n 3 $OUT/smoke.log; return $rc
}
run_sweep() {
  timeout -k 10 300 python -u tools/bench_ops.py sweep 16,32,64 > $OUT/gemm_sweep.log 2>&1
  local rc=$?; cat $OUT/gemm_sweep.log; return $rc
}
run_ops() {
  timeout -k 10 300 python -u tools/bench_ops.py ${OPS:-all} > $OUT/bench_ops.log 2>&1
  local rc=$?; cat $OUT/bench_ops.log; return $rc
}
run_bench() {
  timeout -k 10 480 python -u bench.py --out $OUT/bench.json > $OUT/bench.log 2>&1
  local rc=$?; tail -n 2 $OUT/bench.log; return $rc
}
run_bench_q4() {
  timeout -k 10 480 python -u bench.py --quantization q4_k_m --out $OUT/bench_q4km.json > $OUT/bench_q4km.log 2>&1
  local rc=$?; tail -n 2 $OUT/bench_q4km.log; return $rc
}
# prof_run <name> <bench args...>: kernel trace of one engine-path bench step,
# summarised by tools/prof_db.py into $OUT/<name>_summary.md.
prof_run() {
  local here=$PWD name=$1; shift
  # an unprofiled start first fills the tuning cache, so the profiled run replays the
  # decode GEMM choices of an unprofiled engine (kernel tracing skews start-up timings)
  timeout -k 10 480 python -u bench.py --path engine --steps 1 --warmup 0 --tp-phase off "$@" \
    > $OUT/${name}_tune.log 2>&1 || return $?
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 480 rocprofv3 --kernel-trace --stats -d $here/$OUT/$name \
     -o run -- python3 $here/bench.py --path engine --steps 1 --warmup 1 --tp-phase off "$@" > $here/$OUT/$name.log 2>&1)
  local rc=$?; tail -n 3 $OUT/$name.log
  [ $rc -eq 0 ] || return $rc
  local db; db=$(find $OUT/$name -name '*results.db' | head -n 1)
  [ -n "$db" ] && (cd tools && python prof_db.py "$here/$db" "$here/$OUT/${name}_summary.md" "bench.py --path engine $*" > /dev/null)
  find $OUT/$name -name '*kernel_stats.csv' -exec cp {} $OUT/${name}_kernel_stats.csv \;
  rm -rf $OUT/$name  # raw traces exceed gpurun's 64 MiB copy-back limit
  return 0
}
run_pgemm() {
  local m=${1:-8b}
  timeout -k 10 300 python -u tools/bench_pgemm.py --model $m --fp8 > $OUT/bench_pgemm_$m.log 2>&1
  local rc=$?; tail -n 8 $OUT/bench_pgemm_$m.log; return $rc
}
# bench_named <name> <env assignments...> -- <bench args...>
bench_named() {
  local name=$1; shift
  local envs=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  timeout -k 10 600 env "${envs[@]}" python -u bench.py --tp-phase off --out $OUT/bench_$name.json "$@" \
    > $OUT/bench_$name.log 2>&1
  local rc=$?; tail -n 2 $OUT/bench_$name.log; return $rc
}
run_bench_mixtral() {
  timeout -k 10 600 python -u bench.py --model mixtral-8x7b --concurrency 32 --out $OUT/bench_mixtral.json \
    > $OUT/bench_mixtral.log 2>&1
  local rc=$?; tail -n 2 $OUT/bench_mixtral.log; return $rc
}

for s in $steps; do
  echo "=== $s ($(date +%T))"
  case $s in
    tests) run_tests ;;
    smoke) run_smoke ;;
    sweep) run_sweep ;;
    ops) run_ops ;;
    bench) run_bench ;;
    bench_q4) run_bench_q4 ;;
    bench_mixtral) run_bench_mixtral ;;
    pgemm) run_pgemm 8b ;;
    gguf) timeout -k 10 300 python -u tools/bench_gguf.py --m 1 16 64 > $OUT/bench_gguf.log 2>&1; rc=$?; tail -n 30 $OUT/bench_gguf.log; [ $rc -eq 0 ] ;;
    g27fp8) bench_named g27fp8 HIPSERVE_FP8_PREFILL=1 -- --model gemma-3-27b --quantization fp8 ;;
    b8a) bench_named b8a -- ;;
    b8b) bench_named b8b -- ;;
    untile) timeout -k 10 120 python -u -c "
import torch, time
from hipserve.ops import load_library
load_library()
for N, K in ((43008, 5376), (5376, 21504), (8192, 5376)):
    q = torch.randint(0, 256, (N // 16, K // 256, 4096), dtype=torch.uint8, device='cuda')
    out = torch.empty(N, K, dtype=torch.uint8, device='cuda')
    for _ in range(3): torch.ops.hipserve.fp8_untile(out, q, N, K)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(20): torch.ops.hipserve.fp8_untile(out, q, N, K)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 20
    print(N, K, round(dt * 1e6, 1), 'us', round(2 * N * K / dt / 1e12, 2), 'TB/s (read + write)')
" ;;
    attntest) timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_long_context_gpu.py -x -q --timeout 120 \
                --timeout-method thread -p no:cacheprovider -k "prefill_attention or 32k" > $OUT/attn_test.log 2>&1; rc=$?; tail -n 3 $OUT/attn_test.log; [ $rc -eq 0 ] ;;
    attnbench) BENCH_PREFILL_LONG=1 BENCH_PREFILL_VERS=v2w8 timeout -k 10 300 python -u tools/bench_ops.py prefill > $OUT/attn_bench.log 2>&1; rc=$?; cat $OUT/attn_bench.log; [ $rc -eq 0 ] ;;
    b8_chunk16k) bench_named b8_chunk16k -- --max-num-batched-tokens 16384 ;;
    q4km_chunk8k) bench_named q4km_chunk8k -- --quantization q4_k_m --max-num-batched-tokens 8192 ;;
    q4km_default) bench_named q4km_default -- --quantization q4_k_m ;;
    hosttime) bench_named hosttime_engine HIPSERVE_PROFILE=timing -- --path engine && bench_named hosttime_gw HIPSERVE_PROFILE=timing -- ;;
    q80) bench_named q80 X=1 -- --quantization q8_0 ;;
    q3bf16) bench_named q3bf16 X=1 -- --model qwen3-30b-a3b ;;
    q3int8_8k) bench_named q3int8_8k X=1 -- --model qwen3-30b-a3b --quantization int8 --max-num-batched-tokens 8192 ;;
    q3int8_16k) bench_named q3int8_16k X=1 -- --model qwen3-30b-a3b --quantization int8 --max-num-batched-tokens 16384 ;;
    mixtral16k) bench_named mixtral16k X=1 -- --model mixtral-8x7b --concurrency 32 --max-num-batched-tokens 16384 ;;
    mixtral32k) bench_named mixtral32k X=1 -- --model mixtral-8x7b --concurrency 32 --max-num-batched-tokens 32768 ;;
    q3int8_noshadow16k) bench_named q3int8_noshadow16k HIPSERVE_QUANT_SHADOW=0 -- --model qwen3-30b-a3b --quantization int8 --max-num-batched-tokens 16384 ;;
    q3int8_noshadow32k) bench_named q3int8_noshadow32k HIPSERVE_QUANT_SHADOW=0 -- --model qwen3-30b-a3b --quantization int8 --max-num-batched-tokens 32768 ;;
    g27fp8_16k) bench_named g27fp8_16k X=1 -- --model gemma-3-27b --quantization fp8 --max-num-batched-tokens 16384 ;;
    b8_chunk4k) bench_named b8_chunk4k -- --max-num-batched-tokens 4096 ;;
    enginetest) run_one tests/test_engine_gpu.py ;;
    decsweep) DECODE_COLD=1 DECODE_SHAPES=8x1152x32x4,16x1152x32x4,32x1152x32x4,64x1152x32x4,16x4096x32x4,32x4096x32x4,64x4096x32x4,8x1152x32x8,16x1152x32x8,32x1152x32x8,32x4096x32x8 DECODE_PARTS=512,1024,2048 \
      timeout -k 10 300 python -u tools/bench_ops.py decode > $OUT/decsweep.log 2>&1; rc=$?; cat $OUT/decsweep.log; [ $rc -eq 0 ] ;;
    decq3) for w in 4 8; do HIPSERVE_DECODE_WAVES=$w DECODE_COLD=1 DECODE_SHAPES=64x1152x32x4,64x1152x32x8 DECODE_PARTS=256,512,1024,2048 \
      timeout -k 10 300 python -u tools/bench_ops.py decode > $OUT/decq3_w$w.log 2>&1 || exit 1; echo waves $w; cat $OUT/decq3_w$w.log; done ;;
    prof_moeprefill) cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_moeprefill -o run -- python3 -u tools/bench_moe_prefill.py > $OUT/prof_moeprefill.log 2>&1; rc=$?; cat $OUT/prof_moeprefill.log; [ $rc -eq 0 ] ;;
    moeprefill) timeout -k 10 300 python -u tools/bench_moe_prefill.py > $OUT/bench_moe_prefill.log 2>&1; rc=$?; cat $OUT/bench_moe_prefill.log; [ $rc -eq 0 ] ;;
    tuneprobe) timeout -k 10 300 python -u tools/tune_probe.py > $OUT/tune_probe.log 2>&1; rc=$?; cat $OUT/tune_probe.log; [ $rc -eq 0 ] ;;
    blocking) HIP_LAUNCH_BLOCKING=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py \
      tests/test_fused_decode_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > $OUT/pytest_blocking.log 2>&1; rc=$?; tail -n 5 $OUT/pytest_blocking.log; [ $rc -eq 0 ] ;;
    attnchunk) timeout -k 10 300 python -u tools/bench_ops.py prefill_chunked > $OUT/attn_chunked.log 2>&1; rc=$?; cat $OUT/attn_chunked.log; [ $rc -eq 0 ] ;;
    g27fp8_res) bench_named g27fp8_res HIPSERVE_FP8_PREFILL_LIB=resident -- --model gemma-3-27b --quantization fp8 ;;
    q3int8_noshadow) bench_named q3int8_noshadow HIPSERVE_FUSED_DECODE=1 HIPSERVE_QUANT_SHADOW=0 -- --model qwen3-30b-a3b --quantization int8 ;;
    f8test) run_one tests/test_prefill_gemm_f8_gpu.py ;;
    qmoetest) run_one tests/test_quant_moe_gpu.py ;;
    g27fp8_shadow) bench_named g27fp8_shadow HIPSERVE_FP8_PREFILL=0 -- --model gemma-3-27b --quantization fp8 ;;
    g27bf16) bench_named g27bf16 HIPSERVE_FP8_PREFILL=1 -- --model gemma-3-27b ;;
    q3int8) bench_named q3int8 HIPSERVE_FUSED_DECODE=1 -- --model qwen3-30b-a3b --quantization int8 ;;
    q06) bench_named q06 HIPSERVE_FUSED_DECODE=1 -- --model qwen3-0.6b ;;
    g27bf16_unfused) bench_named g27bf16_unfused HIPSERVE_FUSED_DECODE=0 -- --model gemma-3-27b ;;
    g27fp8_unfused) bench_named g27fp8_unfused HIPSERVE_FUSED_DECODE=0 -- --model gemma-3-27b --quantization fp8 ;;
    q4km) bench_named q4km HIPSERVE_QUANT_SHADOW=1 -- --quantization q4_k_m ;;
    q4km_x16off) bench_named q4km_x16off HIPSERVE_QGEMM_X16=0 -- --quantization q4_k_m ;;
    q4km_noshadow) bench_named q4km_noshadow HIPSERVE_QUANT_SHADOW=0 -- --quantization q4_k_m ;;
    pgemm_g27) run_pgemm gemma27b ;;
    f8test) run_one tests/test_prefill_gemm_f8_gpu.py ;;
    f16test) run_one tests/test_gguf_gpu.py ;;
    fusedtest) run_one tests/test_fused_decode_gpu.py ;;
    pwtest) run_one tests/test_prefill_gemm_packed_gpu.py ;;
    longtest) run_one tests/test_long_context_gpu.py ;;
    kerneltest) run_one tests/test_kernels_gpu.py ;;
    attnab) HIPSERVE_PREFILL_ATTN_PRIO=0 BENCH_PREFILL_LONG=1 BENCH_PREFILL_VERS=v2w8 timeout -k 10 300 python -u tools/bench_ops.py prefill > $OUT/attn_prio0.log 2>&1 && \
            HIPSERVE_PREFILL_ATTN_PRIO=1 BENCH_PREFILL_LONG=1 BENCH_PREFILL_VERS=v2w8 timeout -k 10 300 python -u tools/bench_ops.py prefill > $OUT/attn_prio1.log 2>&1; rc=$?; cat $OUT/attn_prio0.log $OUT/attn_prio1.log | grep prefill_attention; [ $rc -eq 0 ] ;;
    gguf64) timeout -k 10 300 python -u tools/bench_gguf.py --m ${GGUF_M:-64} > $OUT/bench_gguf64.log 2>&1; rc=$?; cat $OUT/bench_gguf64.log; [ $rc -eq 0 ] ;;
    gguf64v2) HIPSERVE_QGEMM_M64=2 timeout -k 10 300 python -u tools/bench_gguf.py --m 64 > $OUT/bench_gguf64_v2.log 2>&1; rc=$?; grep v2_partial $OUT/bench_gguf64_v2.log; [ $rc -eq 0 ] ;;
    qpftest) run_one tests/test_gguf_prefill_gpu.py ;;
    attnpmc) for S in 1024 32768; do
          PMC_PY=tools/attn_pmc.py PG_SHAPE=$S bash scripts/pg_pmc.sh > $OUT/attn_pmc_$S.log 2>&1 || { tail -5 $OUT/attn_pmc_$S.log; exit 1; }
          tail -n 9 $OUT/attn_pmc_$S.log; done ;;
    rope) timeout -k 10 180 python -u tools/bench_rope.py > $OUT/bench_rope.log 2>&1 && \
          HIPSERVE_ROPE_VFAST=0 timeout -k 10 180 python -u tools/bench_rope.py > $OUT/bench_rope_v0.log 2>&1; rc=$?
          cat $OUT/bench_rope.log $OUT/bench_rope_v0.log; [ $rc -eq 0 ] ;;
    qpfpmc) PMC_PY=tools/qpf_pmc.py PG_SHAPE=8192 bash scripts/pg_pmc.sh > $OUT/qpf_pmc.log 2>&1; rc=$?; tail -n 12 $OUT/qpf_pmc.log; [ $rc -eq 0 ] ;;
    qpfbench) timeout -k 10 300 python -u tools/bench_gguf.py --prefill --no-mtiled --m 2048 8192 > $OUT/bench_qpf.log 2>&1; rc=$?; tail -n 40 $OUT/bench_qpf.log; [ $rc -eq 0 ] ;;
    enginetest) run_one tests/test_engine_gpu.py ;;
    pglbench) timeout -k 10 300 python -u tools/bench_pgl.py --model ${PGL_MODEL:-both} > $OUT/bench_pgl.log 2>&1; rc=$?; cat $OUT/bench_pgl.log; [ $rc -eq 0 ] ;;
    tptest) timeout -k 10 1000 python -u -m pytest tests/test_tp_gpu.py -x -v --timeout 420 --timeout-method thread \
              -p no:cacheprovider > $OUT/test_tp_gpu.log 2>&1; rc=$?; tail -n 20 $OUT/test_tp_gpu.log; [ $rc -eq 0 ] ;;
    prof_q4) prof_run profq --quantization q4_k_m ;;
    prof_g27) prof_run profg27 --model gemma-3-27b ;;
    prof_q3int8) prof_run profq3 --model qwen3-30b-a3b --quantization int8 ;;
    prof_g27fp8) prof_run profg27f8 --model gemma-3-27b --quantization fp8 ;;
    prof) prof_run prof ;;
    prof_mixtral) prof_run profmx --model mixtral-8x7b --concurrency 32 ;;
    prof70) prof_run prof70 --model llama-3-70b ;;
    prof32k) prof_run prof32k --model llama-3.1-8b --input-len 32768 --output-len 64 --concurrency 4 --max-num-batched-tokens 8192 ;;
    long8k) bench_named long8k X=1 -- --model llama-3.1-8b --input-len 8192 --output-len 256 --concurrency 16 --max-num-batched-tokens 8192 --steps 2 ;;
    long32k) bench_named long32k X=1 -- --model llama-3.1-8b --input-len 32768 --output-len 256 --concurrency 4 --max-num-batched-tokens 8192 --steps 2 ;;
    long32k_p0) bench_named long32k_p0 HIPSERVE_PREFILL_ATTN_PRIO=0 -- --model llama-3.1-8b --input-len 32768 --output-len 256 --concurrency 4 --max-num-batched-tokens 8192 --steps 2 ;;
    long32k_p1) bench_named long32k_p1 HIPSERVE_PREFILL_ATTN_PRIO=1 -- --model llama-3.1-8b --input-len 32768 --output-len 256 --concurrency 4 --max-num-batched-tokens 8192 --steps 2 ;;
    bench_mixtral_packed) bench_named mixtral_packed HIPSERVE_MOE_PACKED_PREFILL=1 -- --model mixtral-8x7b --concurrency 32 ;;
    bench_mixtral_old) bench_named mixtral_old HIPSERVE_MOE_PACKED_PREFILL=0 -- --model mixtral-8x7b --concurrency 32 ;;
    prof_qwen3moe) prof_run profqm --model qwen3-30b-a3b ;;
    prof_gemma3) prof_run profg3 --model gemma-3-27b ;;
    prof_g27fp8) prof_run profg3f8 --model gemma-3-27b --quantization fp8 ;;
    g27fp8d) bench_named g27fp8d X=1 -- --model gemma-3-27b --quantization fp8 ;;
    fp8dtest) run_one tests/test_fp8_decode_gpu.py ;;
    famtest) run_one tests/test_families_gpu.py ;;
    kvf8test) run_one tests/test_kv_fp8_gpu.py ;;
    b8kvf8) bench_named b8kvf8 X=1 -- --kv-cache-dtype fp8 ;;
    g27fp8kvf8) bench_named g27fp8kvf8 X=1 -- --model gemma-3-27b --quantization fp8 --kv-cache-dtype fp8 ;;
    prof_kvf8) prof_run profkvf8 --kv-cache-dtype fp8 ;;
    deckv) for kv in bf16 fp8; do for w in 4 8; do DECODE_KV=$kv HIPSERVE_DECODE_WAVES=$w DECODE_COLD=1 DECODE_SHAPES=64x1152x32x8,64x1152x32x16 DECODE_PARTS=512,2048 \
      timeout -k 10 300 python -u tools/bench_ops.py decode > $OUT/deckv_${kv}_w$w.log 2>&1 || exit 1; echo "kv $kv waves $w"; grep paged_decode $OUT/deckv_${kv}_w$w.log; done; done ;;
    prefkv) for kv in bf16 fp8; do DECODE_KV=$kv BENCH_PREFILL_VERS=v2w8 timeout -k 10 300 python -u tools/bench_ops.py prefill > $OUT/prefkv_$kv.log 2>&1 || exit 1; echo "kv $kv"; grep prefill_attention $OUT/prefkv_$kv.log; done ;;
    deckvnt) for nt in 1 0; do DECODE_KV=fp8 HIPSERVE_DECODE_NT=$nt DECODE_COLD=1 DECODE_SHAPES=64x1152x32x8,64x1152x32x16,64x4096x32x8 DECODE_PARTS=2048 \
      timeout -k 10 300 python -u tools/bench_ops.py decode > $OUT/deckv_nt$nt.log 2>&1 || exit 1; echo "fp8 nt $nt"; grep paged_decode $OUT/deckv_nt$nt.log; done ;;
    prof_q80) prof_run profq80 --quantization q8_0 ;;
    g27fp8c256) bench_named g27fp8c256 X=1 -- --model gemma-3-27b --quantization fp8 --concurrency 256 --steps 1 ;;
    prof_g27c256) prof_run profg27c256 --model gemma-3-27b --quantization fp8 --concurrency 256 ;;
    ropet) for t in 1 0; do HIPSERVE_ROPE_TILE=$t timeout -k 10 180 python -u tools/bench_rope.py --T 128 256 512 1024 2048 4096 > $OUT/ropet$t.log 2>&1 || exit 1; grep '"aligned"' $OUT/ropet$t.log; done ;;
    b8c256) bench_named b8c256 X=1 -- --concurrency 256 --steps 2 ;;
    q4c256) bench_named q4c256 X=1 -- --quantization q4_k_m --concurrency 256 --steps 2 ;;
    q3int8c256) bench_named q3int8c256 X=1 -- --model qwen3-30b-a3b --quantization int8 --concurrency 256 --steps 2 ;;
    prof_b8c256) prof_run profb8c256 --concurrency 256 ;;
    hosttime256) bench_named hosttime256 HIPSERVE_PROFILE=timing -- --path engine --concurrency 256 --steps 1 ;;
    decblas) timeout -k 10 600 python -u tools/bench_decode_blas.py > $OUT/decblas.log 2>&1; rc=$?; cat $OUT/decblas.log; [ $rc -eq 0 ] ;;
    coalab) for r in 1 2; do bench_named coal_off_$r HIPSERVE_COALESCE_MAX_MS=0 -- --steps 5 --tp-phase off && \
              bench_named coal_def_$r X=1 -- --steps 5 --tp-phase off || exit 1; done
            for f in coal_off_1 coal_def_1 coal_off_2 coal_def_2; do grep -o '"value": [0-9.]*\|"p50_ttft_ms": [0-9.]*' $OUT/bench_$f.json | tr '\n' ' '; echo $f; done ;;
    topktest) timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_quant_moe_gpu.py tests/test_families_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "topk or moe or family" > $OUT/topktest.log 2>&1; rc=$?; tail -n 5 $OUT/topktest.log; [ $rc -eq 0 ] ;;
    int8ctest) timeout -k 10 400 python -u -m pytest tests/test_gguf_gpu.py tests/test_quant_moe_gpu.py tests/test_families_gpu.py tests/test_int_quant.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "int8 or moe or quant or family" > $OUT/int8ctest.log 2>&1; rc=$?; tail -n 5 $OUT/int8ctest.log; [ $rc -eq 0 ] ;;
    qmoebench) timeout -k 10 400 python -u tools/bench_qmoe.py ${QMOE_ARGS:-} > $OUT/qmoebench.log 2>&1; rc=$?; cat $OUT/qmoebench.log | grep -v amdgpu.ids; [ $rc -eq 0 ] ;;
    *) echo "unknown step $s"; false ;;
  esac || { echo "step $s failed (rc=$?)"; exit 1; }
done
echo "=== done ($(date +%T))"
