set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/probe1
timeout -k 10 300 python -u bench.py --path engine --steps 2 --warmup 1 > gpurun_out/probe1/engine.log 2>&1 && \
HIPSERVE_STEP_LOG=$GRAFT_REPO_ROOT/gpurun_out/probe1/steps_gw.jsonl timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 > gpurun_out/probe1/gw.log 2>&1
tail -1 gpurun_out/probe1/engine.log; tail -1 gpurun_out/probe1/gw.log
