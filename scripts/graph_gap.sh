set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gg
for k in 30 266; do
  timeout -k 10 120 python -u tools/bench_graph_gap.py --kernels $k >> gpurun_out/gg/gap.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/bench_graph_gap.py --kernels $k --event >> gpurun_out/gg/gap.log 2>&1 || exit 1
done
grep '^{' gpurun_out/gg/gap.log
