#!/bin/bash
# One gpurun call: the in-house TP collectives on ONE GPU shared by N ranks.
#   1. tools/bench_allreduce.py --shared-gpu at world 2 and 8, eager and hipGraph,
#      with the add+RMSNorm epilogue sweep (64-block / 512-block classes);
#   2. an 8-rank Llama-3-70B-shape (2 layers) engine, one 8192-token prefill chunk +
#      decode, rank 0 under rocprofv3 --kernel-trace --stats (car_norm vs GEMM time).
# usage: gpurun --timeout 900 -- 'bash scripts/tp_collectives.sh [ar2 ar8 trace8]'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
HERE=$PWD
OUT=gpurun_out/tpc
mkdir -p $OUT
export PYTHONUNBUFFERED=1
steps="${*:-ar2 ar8 trace8}"

ar() {  # ar <world> <hidden>
  local w=$1 h=$2
  # one HW queue per process (see trace8): 8 ranks x 4 queues oversubscribe the
  # device's queue slots and the CP time-slices spin-waiting collective kernels
  export GPU_MAX_HW_QUEUES=1
  for g in "" "--graph"; do
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
      --master-port 29$((500 + w)) tools/bench_allreduce.py --shared-gpu --iters 20 --norm $h $g \
      --out $OUT/ar_w${w}.jsonl > $OUT/ar_w${w}${g}.log 2>&1 || { tail -20 $OUT/ar_w${w}${g}.log; return 1; }
    grep -v "^\[" $OUT/ar_w${w}${g}.log | grep -v Warning | tail -40
  done
}

trace8() {
  # one HW queue per process: 8 processes x the default 4 queues oversubscribe the
  # device's hardware queue slots, and the CP then time-slices queues (~10 ms quanta),
  # so every spin-waiting collective kernel would wait out whole quanta for its peers
  # (measured: 10.6-21 ms per hipGraph all-reduce at 4 queues, 81 us at 1)
  export GPU_MAX_HW_QUEUES=1
  local port=29631 pids=()
  # heartbeat: 8 ranks time-sharing one GPU run for minutes without writing anything
  (while sleep 30; do echo "trace8 heartbeat $(date +%T)"; done) &
  local hb=$!
  for r in 1 2 3 4 5 6 7; do
    RANK=$r WORLD_SIZE=8 MASTER_PORT=$port timeout -k 10 420 python3 tools/tp_shared_gpu.py --model llama-3-70b \
      --layers 2 --batch 8 --input-len 1024 --output-len 32 > $OUT/trace8_r$r.log 2>&1 &
    pids+=($!)
  done
  (cd /tmp && export TMPDIR=/tmp && RANK=0 WORLD_SIZE=8 MASTER_PORT=$port timeout -k 10 420 rocprofv3 --kernel-trace \
     --stats -d $HERE/$OUT/trace8 -o r0 -- python3 $HERE/tools/tp_shared_gpu.py --model llama-3-70b --layers 2 \
     --batch 8 --input-len 1024 --output-len 32 > $HERE/$OUT/trace8_r0.log 2>&1)
  local rc=$?
  for p in "${pids[@]}"; do wait $p || rc=$((rc ? rc : 1)); done
  kill $hb 2>/dev/null
  tail -3 $OUT/trace8_r0.log
  [ $rc -eq 0 ] || return $rc
  local db; db=$(find $OUT/trace8 -name '*results.db' | head -n 1)
  [ -n "$db" ] && (cd tools && python prof_db.py "$HERE/$db" "$HERE/$OUT/trace8_summary.md" \
     "TP=8 shared GPU, Llama-3-70B shapes (2 layers), rank 0" > /dev/null)
  find $OUT/trace8 -name '*kernel_stats.csv' -exec cp {} $OUT/trace8_kernel_stats.csv \;
  rm -rf $OUT/trace8
  return 0
}

for s in $steps; do
  echo "=== $s ($(date +%T))"
  case $s in
    ar2) ar 2 4096 ;;
    ar8) ar 8 8192 ;;
    trace8) trace8 ;;
    *) echo "unknown step $s"; false ;;
  esac || { echo "step $s failed (rc=$?)"; exit 1; }
done
echo "=== done ($(date +%T))"
