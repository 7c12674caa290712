# decode-attention waves per workgroup 4 vs 8 with the fused qkv attention (engine decode step)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/dw
for w in 4 8 4 8; do
  HIPSERVE_DECODE_WAVES=$w timeout -k 10 240 python -u tools/decode_gap.py > gpurun_out/dw/gap_$w.log 2>&1 || { tail -20 gpurun_out/dw/gap_$w.log; exit 1; }
  echo "waves=$w $(tail -1 gpurun_out/dw/gap_$w.log)"
done
