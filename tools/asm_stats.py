#!/usr/bin/env python3
"""Instruction census of the kernels in a hipcc ``-S --cuda-device-only`` listing: per
kernel, the whole body and its innermost loops (a label that a later ``s_cbranch``
jumps back to), counting MFMAs, AGPR <-> VGPR moves, scratch, waits, VMEM and LDS ops.

usage: python tools/asm_stats.py file.s [kernel-substring]
"""
from __future__ import annotations

import re
import sys

PATS = {
    "mfma": r"\bv_mfma", "acc_rd": r"v_accvgpr_read", "acc_wr": r"v_accvgpr_write", "acc_mov": r"v_accvgpr_mov",
    "scratch": r"\bscratch_", "waitcnt": r"\bs_waitcnt", "vmem": r"\b(buffer|global)_load", "store": r"\b(buffer|global)_store",
    "ds_rd": r"\bds_read", "ds_wr": r"\bds_write", "barrier": r"\bs_barrier", "valu": r"^\s*v_(?!mfma|accvgpr)",
    "nop": r"\bs_nop",
}


def census(lines):
    return {k: sum(1 for ln in lines if re.search(p, ln)) for k, p in PATS.items()}


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    text = open(path).read().split("\n")
    kernels = []
    for i, ln in enumerate(text):
        m = re.match(r"^(_Z\S+):\s", ln)
        if m and not ln.startswith("\t"):
            kernels.append((m.group(1), i))
    for k, (name, start) in enumerate(kernels):
        if want not in name:
            continue
        end = kernels[k + 1][1] if k + 1 < len(kernels) else len(text)
        body = text[start:end]
        try:
            body = body[:next(j for j, ln in enumerate(body) if "s_endpgm" in ln) + 1]
        except StopIteration:
            pass
        labels = {}
        for j, ln in enumerate(body):
            m = re.match(r"^(\.LBB\S+):", ln)
            if m:
                labels[m.group(1)] = j
        print(f"{name}: {census(body)}")
        for j, ln in enumerate(body):
            m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)", ln)
            if m and m.group(1) in labels and labels[m.group(1)] < j:
                c = census(body[labels[m.group(1)]:j + 1])
                print(f"  loop {m.group(1)} ({j - labels[m.group(1)]} lines): {c}")


if __name__ == "__main__":
    main()
