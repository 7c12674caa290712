#!/bin/bash
# PMC passes: hipBLASLt vs prefill_gemm on one shape (tools/pg_pmc.py); csv under gpurun_out/pmc
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
HERE=$PWD
OUT=$HERE/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
pass() {  # pass <name> <counters...>
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$n -o run -- python3 $HERE/${PMC_PY:-tools/pg_pmc.py} \
    ${PG_SHAPE:-8192 28672 4096} > $OUT/$n.log 2>&1 || { tail -5 $OUT/$n.log; return 1; }
  find $OUT/$n -name '*counter_collection.csv' -exec cp {} $OUT/$n.csv \;
  rm -rf $OUT/$n
}
pass p1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU && \
pass p2 SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT && \
pass p3 SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_WAVES TCC_HIT_sum TCC_MISS_sum && \
cd $HERE && python3 - <<'PY'
import csv, collections, glob
for f in sorted(glob.glob("gpurun_out/pmc/p*.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", f)
    for k, d in agg.items():
        print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
