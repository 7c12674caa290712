#!/usr/bin/env python3
"""Per-kernel-family hardware-counter summary from rocprofv3 ``--pmc`` CSV output.

usage: python tools/pmc_summary.py out.md title pass1_counter_collection.csv [pass2.csv ...]

Each pass is its own rocprofv3 run (one counter group per run, see
scripts/pmc_passes.sh). Rows are summed per (kernel family, counter) over all
dispatches; with a FETCH_SIZE / WRITE_SIZE pass the table also gives bytes per
call. gfx950 FETCH_SIZE counts half of a wide coalesced stream's bytes
(MI355X_MICROARCH.md), so the "read GB" column doubles it.
"""
import collections
import csv
import sys

from prof_summary import family


def load(paths):
    acc = collections.defaultdict(float)  # (family, counter) -> sum
    calls = collections.defaultdict(set)  # (family, pass) -> dispatch ids
    for p in paths:
        with open(p, newline="") as f:
            for r in csv.DictReader(f):
                fam = family(r["Kernel_Name"])
                acc[(fam, r["Counter_Name"])] += float(r["Counter_Value"])
                calls[(fam, p)].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    per_fam = collections.defaultdict(int)  # dispatches of ONE run (every pass runs the same program)
    for (fam, _), ids in calls.items():
        per_fam[fam] = max(per_fam[fam], len(ids))
    return acc, dict(per_fam)


def main():
    out, title, paths = sys.argv[1], sys.argv[2], sys.argv[3:]
    acc, calls = load(paths)
    counters = sorted({c for _, c in acc})
    fams = sorted(calls, key=lambda f: -max((acc.get((f, c), 0.0) for c in counters), default=0.0))
    L = [f"# {title}", "",
         "Counter sums over every dispatch of a kernel family; `calls` = dispatches in one run",
         "(each counter group is its own run of the same program, engine init incl. the decode",
         "GEMM autotuner). SQ_VALU_MFMA_BUSY_CYCLES counts cycles and SQ_BUSY_CYCLES quad-cycles",
         "summed over SEs, so their ratio is only comparable between kernels.", ""]
    hdr = ["kernel", "calls"] + counters
    have_bytes = "FETCH_SIZE" in counters
    if have_bytes:
        hdr += ["read GB (2x FETCH_SIZE)", "read MB/call"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in counters and "SQ_BUSY_CYCLES" in counters:
        hdr += ["MFMA busy / SQ busy (raw ratio)"]
    if "SQ_LDS_BANK_CONFLICT" in counters and "SQ_LDS_IDX_ACTIVE" in counters:
        hdr += ["LDS conflict / LDS active"]
    L.append("| " + " | ".join(hdr) + " |")
    L.append("|---|" + "---:|" * (len(hdr) - 1))
    for f in fams[:40]:
        row = [f"`{f}`", str(calls[f])] + [f"{acc.get((f, c), 0.0):.4g}" for c in counters]
        if have_bytes:
            gb = 2 * acc.get((f, "FETCH_SIZE"), 0.0) * 1024 / 1e9  # FETCH_SIZE is in KiB
            row += [f"{gb:.2f}", f"{gb * 1e3 / max(calls[f], 1):.2f}"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in counters and "SQ_BUSY_CYCLES" in counters:
            b = acc.get((f, "SQ_BUSY_CYCLES"), 0.0)
            row.append(f"{acc.get((f, 'SQ_VALU_MFMA_BUSY_CYCLES'), 0.0) / b:.3f}" if b else "—")
        if "SQ_LDS_BANK_CONFLICT" in counters and "SQ_LDS_IDX_ACTIVE" in counters:
            a = acc.get((f, "SQ_LDS_IDX_ACTIVE"), 0.0)
            row.append(f"{acc.get((f, 'SQ_LDS_BANK_CONFLICT'), 0.0) / a:.3f}" if a else "—")
        L.append("| " + " | ".join(row) + " |")
    open(out, "w").write("\n".join(L) + "\n")
    print("\n".join(L[:30]))


if __name__ == "__main__":
    main()
