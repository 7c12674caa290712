#!/bin/bash
# Hardware-counter passes over a short engine-path decode run (one rocprofv3 run per
# counter group: FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950's TCC), then
# tools/pmc_summary.py -> gpurun_out/pmc_summary.md.
#   gpurun --timeout 900 -- 'bash scripts/pmc_passes.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
here=$PWD
OUT=$here/gpurun_out/pmc
mkdir -p $OUT
ARGS="--path engine --steps 1 --warmup 1 --input-len 1024 --output-len 64"
i=0
for counters in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE" \
                "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i + 1))
  echo "=== pass $i: $counters ($(date +%T))"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $counters --output-format csv \
     -d $OUT/p$i -o run -- python3 $here/bench.py $ARGS > $OUT/p$i.log 2>&1) || { tail -5 $OUT/p$i.log; exit 1; }
  tail -n 1 $OUT/p$i.log | cut -c1-160
done
csvs=$(find $OUT -name '*counter_collection.csv' | sort)
(cd tools && python pmc_summary.py $here/gpurun_out/pmc_summary.md \
   "rocprofv3 --pmc: Llama-3-8B engine path, 64 x 1024 in / 64 out" $csvs)
rm -rf $OUT/p1 $OUT/p2 $OUT/p3
