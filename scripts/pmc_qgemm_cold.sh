# PMC passes: v2 (qgemm2) quantised decode GEMM, M=64 Q4_K gate|up, cold blocks
set -o pipefail
cd $GRAFT_REPO_ROOT; here=$PWD; OUT=$here/gpurun_out/pmcq3; mkdir -p $OUT
i=0
for counters in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS" \
                "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d $OUT/p$i -o run -- \
     python3 $here/tools/bench_gguf.py --m 64 --only gate_up --cold --splits 1 2 4 > $OUT/p$i.log 2>&1) || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, os
out = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/pmcq3"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "qgemm" not in k:
            continue
        agg[k[:100]][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(out + "/summary.txt", "w") as fo:
    for k, d in agg.items():
        fo.write(k + "\n")
        for c, v in sorted(d.items()):
            fo.write(f"  {c}: mean per dispatch {sum(v)/len(v):.4g} (n={len(v)})\n")
print(open(out + "/summary.txt").read())
PY
rm -rf $OUT/p1 $OUT/p2
