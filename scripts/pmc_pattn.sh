# PMC passes over the v2 prefill attention (tools/bench_ops.py prefill)
set -o pipefail
cd $GRAFT_REPO_ROOT; here=$PWD; OUT=$here/gpurun_out/pmca; mkdir -p $OUT
i=0
for counters in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS" \
                "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $counters --output-format csv -d $OUT/p$i -o run -- \
     python3 $here/tools/bench_ops.py prefill > $OUT/p$i.log 2>&1) || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, os
out = os.environ.get("GRAFT_REPO_ROOT", ".") + "/gpurun_out/pmca"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "prefill_attn_v2" not in k:
            continue
        agg[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(out + "/summary.txt", "w") as fo:
    for k, d in agg.items():
        fo.write(k + "\n")
        for c, v in sorted(d.items()):
            fo.write(f"  {c}: mean per dispatch {sum(v)/len(v):.4g} (n={len(v)})\n")
print(open(out + "/summary.txt").read())
PY
