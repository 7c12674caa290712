# KV block size 16 vs 32 vs 64: paged decode microbench (cold KV) and the engine decode step
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/bs
DECODE_COLD=1 DECODE_PARTS=2048 DECODE_BS=16,32,64 DECODE_SHAPES=64x1152x32x8,64x1280x32x8 \
  timeout -k 10 200 python -u tools/bench_ops.py decode > gpurun_out/bs/ops.log 2>&1 || { tail -20 gpurun_out/bs/ops.log; exit 1; }
grep '^{' gpurun_out/bs/ops.log
for b in 16 32 16 32; do
  timeout -k 10 240 python -u tools/decode_gap.py --block-size $b > gpurun_out/bs/gap_$b.log 2>&1 || { tail -20 gpurun_out/bs/gap_$b.log; exit 1; }
  echo "bs=$b $(tail -1 gpurun_out/bs/gap_$b.log)"
done
