#!/usr/bin/env python3
"""Condense a rocprofv3 ``*_kernel_stats.csv`` into a short per-kernel-family
table (markdown) for ``profiles/``: hipBLASLt GEMM names are grouped by macro
tile, template arguments are dropped."""
import csv
import re
import sys


def family(name: str) -> str:
    if name.startswith(("Cijk", "Custom_Cijk")):
        m = re.search(r"MT(\d+x\d+x\d+)", name)
        return f"hipBLASLt GEMM MT{m.group(1) if m else '?'}"
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    if name.startswith("at::native"):
        name = "torch " + re.sub(r"<.*", "", name).split("::")[-1]
    return name


def main(path, out=None, title="kernel stats"):
    rows = list(csv.DictReader(open(path)))
    agg = {}
    for r in rows:
        f = family(r["Name"])
        a = agg.setdefault(f, [0, 0])
        a[0] += int(r["Calls"])
        a[1] += int(r["TotalDurationNs"])
    total = sum(v[1] for v in agg.values())
    lines = [f"# {title}", "", f"total kernel time: {total / 1e6:.1f} ms", "",
             "| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for f, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| `{f}` | {c} | {t / 1e6:.1f} | {t / c / 1e3:.1f} | {100 * t / total:.1f} |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None,
         sys.argv[3] if len(sys.argv) > 3 else "kernel stats")
