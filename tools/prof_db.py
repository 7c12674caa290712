#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd SQLite database (``--kernel-trace --stats`` writes
``<dir>/<name>_results.db``) into a markdown report for ``profiles/``:

* per-kernel-family totals (same grouping as ``prof_summary.py``),
* the engine timeline split into steps at each ``sample_kernel`` dispatch, with
  decode-only steps (no prefill attention) separated from prefill/mixed steps,
* per-decode-step kernel breakdown and GPU idle time (gaps between kernels,
  i.e. host/launch overhead not hidden by the hipGraph).

usage: python tools/prof_db.py run_results.db [out.md] [title]
"""
import sqlite3
import statistics
import sys

from prof_summary import family


def load(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    return [(family(n), s, e) for n, s, e in rows]


def steps(rows):
    out, cur = [], []
    for r in rows:
        cur.append(r)
        if "sample_kernel" in r[0] or "mc_final_kernel" in r[0]:  # the sampler ends every step
            out.append(cur)
            cur = []
    return out


def summarize(path, title="rocprofv3 kernel trace"):
    rows = load(path)
    tot = {}
    for f, s, e in rows:
        a = tot.setdefault(f, [0, 0])
        a[0] += 1
        a[1] += e - s
    total = sum(v[1] for v in tot.values())
    L = [f"# {title}", "", f"kernels: {len(rows)}, total kernel time {total / 1e6:.1f} ms", "",
         "## all kernels by family", "", "| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for f, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:40]:
        L.append(f"| `{f}` | {n} | {d / 1e6:.1f} | {d / n / 1e3:.1f} | {100 * d / total:.1f} |")
    st = steps(rows)
    dec = [s for s in st if not any("prefill_attn" in r[0] for r in s)]
    pre = [s for s in st if any("prefill_attn" in r[0] for r in s)]
    # one step SHAPE only: decode steps whose kernel sequence (families in dispatch order)
    # is the most common one. Keying on the kernel count alone mixed two graph buckets
    # whose steps had the same count but different kernel instantiations (VERDICT r5
    # weak #8: a Qwen3 table summed to 13.0 ms against a 10.9 ms step)
    if dec:
        sig = [tuple(f for f, _, _ in s) for s in dec]
        mode = statistics.mode(sig)
        n_shapes = len(set(sig))
        dec = [s for s, g in zip(dec, sig) if g == mode]

    def span(s):
        return (s[-1][2] - s[0][1]) / 1e3

    def busy(s):
        return sum(e - b for _, b, e in s) / 1e3

    L += ["", "## engine steps", "",
          f"steps: {len(st)} ({len(pre)} with prefill, {len(dec)} decode-only of the modal shape)"]
    if pre:
        sp = [span(s) for s in pre]
        L.append(f"prefill/mixed step: median span {statistics.median(sp):.0f} us, "
                 f"kernel-busy {statistics.median(busy(s) for s in pre):.0f} us")
        big = [s for s in pre if span(s) >= 0.8 * statistics.median(sp)]
        per = {}
        for s in big:
            acc = {}
            for f, b, e in s:
                a = acc.setdefault(f, [0, 0])
                a[0] += 1
                a[1] += e - b
            for f, (n, d) in acc.items():
                per.setdefault(f, []).append((n, d))
        agg = sorted(((f, v[0][0], statistics.median(d for _, d in v) / 1e3) for f, v in per.items()),
                     key=lambda x: -x[2])
        L += ["", f"### per full prefill step (median over {len(big)} steps)", "",
              "| kernel | calls/step | us/step | avg us |", "|---|---:|---:|---:|"]
        for f, n, d in agg[:25]:
            L.append(f"| `{f}` | {n} | {d:.1f} | {d / n:.2f} |")
        L.append("")
    if dec:
        sp = [span(s) for s in dec]
        bz = [busy(s) for s in dec]
        L += [f"decode step: median span {statistics.median(sp):.0f} us, kernel-busy "
              f"{statistics.median(bz):.0f} us, idle {statistics.median(sp) - statistics.median(bz):.0f} us "
              f"({len(dec[0])} kernels/step)", "", "### per decode step (median over steps)", "",
              "| kernel | calls/step | us/step | avg us |", "|---|---:|---:|---:|"]
        per = {}
        for s in dec:
            acc = {}
            for f, b, e in s:
                a = acc.setdefault(f, [0, 0])
                a[0] += 1
                a[1] += e - b
            for f, (n, d) in acc.items():
                per.setdefault(f, []).append((n, d))
        agg = sorted(((f, v[0][0], statistics.median(d for _, d in v) / 1e3) for f, v in per.items()),
                     key=lambda x: -x[2])
        for f, n, d in agg:
            L.append(f"| `{f}` | {n} | {d:.1f} | {d / n:.2f} |")
        L += ["", f"table sum {sum(d for _, _, d in agg):.0f} us vs median kernel-busy "
              f"{statistics.median(bz):.0f} us ({len(dec)} steps of the modal shape; "
              f"{n_shapes} decode step shapes in the trace)"]
        # where the idle time sits: gap before each kernel family (median step)
        gaps = {}
        for s in dec:
            acc = {}
            for (f0, b0, e0), (f1, b1, e1) in zip(s, s[1:]):
                acc[f1] = acc.get(f1, 0) + max(0, b1 - e0)
            for f, g in acc.items():
                gaps.setdefault(f, []).append(g)
        gl = sorted(((f, statistics.median(v) / 1e3) for f, v in gaps.items()), key=lambda x: -x[1])[:8]
        mid = dec[len(dec) // 2]  # one decode step in dispatch order (first 120 kernels)
        L += ["", "### kernel sequence of one decode step", "", "| # | kernel | us |", "|---:|---|---:|"]
        for j, (f, b, e) in enumerate(mid[:120]):
            L.append(f"| {j} | `{f}` | {(e - b) / 1e3:.1f} |")
        L += ["", "### idle gaps inside a decode step, by the kernel that follows (median us/step)", "",
              "| next kernel | gap us/step |", "|---|---:|"]
        for f, g in gl:
            L.append(f"| `{f}` | {g:.1f} |")
    return "\n".join(L) + "\n"


if __name__ == "__main__":
    text = summarize(sys.argv[1], *(sys.argv[3:4] or []))
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)
