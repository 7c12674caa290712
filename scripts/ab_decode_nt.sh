# A/B: paged-decode K/V loads non-temporal (default) vs default policy
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/nt
for nt in 1 0; do
  HIPSERVE_DECODE_NT=$nt DECODE_COLD=1 DECODE_PARTS=2048 timeout -k 10 120 python -u tools/bench_ops.py decode > gpurun_out/nt/ops_nt$nt.log 2>&1 || exit 1
done
for nt in 1 0; do
  HIPSERVE_DECODE_NT=$nt timeout -k 10 240 python -u tools/decode_gap.py > gpurun_out/nt/gap_nt$nt.log 2>&1 || exit 1
done
tail -n 3 gpurun_out/nt/*.log
