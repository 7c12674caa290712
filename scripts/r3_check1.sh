#!/bin/bash
# prefill GEMM (buffer-load staging) + top-logprobs ordering + TP logit bound
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash scripts/pg_check.sh || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "top_logprobs" > gpurun_out/pytest_toplp.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_toplp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 450 --timeout-method thread -p no:cacheprovider \
  tests/test_tp_gpu.py > gpurun_out/pytest_tp.log 2>&1
rc=$?; grep -E "logit bound|exact prefix|PASS|FAIL|Error" gpurun_out/pytest_tp.log | tail -12; exit $rc
