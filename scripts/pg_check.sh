#!/bin/bash
# prefill GEMM: numerics tests + the hipBLASLt comparison bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_prefill_gemm_gpu.py > gpurun_out/pytest_pg.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_pg.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_check.sh pgemm
