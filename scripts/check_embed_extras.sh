# full GPU suite, decode step wall time, gateway bench, kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ee
bash scripts/gpu_check.sh tests smoke || exit 1
timeout -k 10 240 python -u tools/decode_gap.py > gpurun_out/ee/gap.log 2>&1 || exit 1
tail -1 gpurun_out/ee/gap.log
bash scripts/gpu_check.sh bench prof || exit 1
