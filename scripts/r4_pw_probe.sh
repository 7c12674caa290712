#!/bin/bash
# Packed-layout prefill GEMM probes: time vs K (persistent / one tile per workgroup,
# weight ring depth 2 / 4) and PMC passes against hipBLASLt. Each GPU step time-limited.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/bench_pw_scaling.py --ks ${PW_KS:-2048,4096,8192} > gpurun_out/pw_scaling.log 2>&1; rc=$?
cat gpurun_out/pw_scaling.log; [ $rc -eq 0 ] || exit $rc
[ "${PW_PMC:-1}" = "1" ] && PG_VARIANTS="${PG_VARIANTS:-p1}" bash scripts/pg_pmc.sh
exit 0
