#!/bin/bash
# Round-3 evidence runs (one gpurun call, steps chained; each GPU step time-limited):
#   ar8q1      world-8 shared-GPU hipGraph all-reduce sweep with GPU_MAX_HW_QUEUES=1
#              (tests the queue-oversubscription explanation of the 10-20 ms graph calls)
#   mixtral    Mixtral-8x7B bench, grouped prefill GEMM on (default) and off
#   openloop   Llama-3-8B gateway bench, open-loop Poisson at 3 rates
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ev
mkdir -p $OUT
export PYTHONUNBUFFERED=1
steps="${*:-ar8q1 mixtral openloop}"

ar8q1() {
  GPU_MAX_HW_QUEUES=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29611 tools/bench_allreduce.py --shared-gpu --iters 20 --graph \
    > $OUT/ar_w8_graph_q1.log 2>&1 || { tail -20 $OUT/ar_w8_graph_q1.log; return 1; }
  grep "^|" $OUT/ar_w8_graph_q1.log | head -14
}
mixtral() {
  timeout -k 10 600 python -u bench.py --model mixtral-8x7b --concurrency 32 --out $OUT/mixtral_pg.json \
    > $OUT/mixtral_pg.log 2>&1 || { tail -20 $OUT/mixtral_pg.log; return 1; }
  tail -n 1 $OUT/mixtral_pg.log
  HIPSERVE_PREFILL_GEMM=0 timeout -k 10 600 python -u bench.py --model mixtral-8x7b --concurrency 32 \
    --out $OUT/mixtral_blas.json > $OUT/mixtral_blas.log 2>&1 || { tail -20 $OUT/mixtral_blas.log; return 1; }
  tail -n 1 $OUT/mixtral_blas.log
}
openloop() {
  for r in 8 16 24; do
    timeout -k 10 400 python -u bench.py --request-rate $r --steps 2 --tp-phase off --out $OUT/openloop_r$r.json \
      > $OUT/openloop_r$r.log 2>&1 || { tail -20 $OUT/openloop_r$r.log; return 1; }
    tail -n 1 $OUT/openloop_r$r.log
  done
}
for s in $steps; do
  echo "=== $s ($(date +%T))"
  $s || { echo "step $s failed"; exit 1; }
done
echo "=== done ($(date +%T))"
