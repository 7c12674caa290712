#!/bin/bash
# A/B of the fused decode layer v2 (HIPSERVE_FUSED_V2) by rocprofv3 kernel traces of the
# engine-path bench, plus the prefill GEMM bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
bash scripts/gpu_check.sh pgemm || exit 1
HIPSERVE_FUSED_V2=1 bash scripts/gpu_check.sh prof && mv gpurun_out/prof_summary.md gpurun_out/prof_v2_summary.md || exit 1
HIPSERVE_FUSED_V2=0 bash scripts/gpu_check.sh prof && mv gpurun_out/prof_summary.md gpurun_out/prof_v1_summary.md
