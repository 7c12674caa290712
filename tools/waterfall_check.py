#!/usr/bin/env python3
"""Find waterfall loops in the gfx950 device code of ``csrc/kernels/*.hip``.

A buffer load or store needs its 128-bit resource descriptor in SGPRs. If the compiler
thinks the descriptor is divergent, it wraps the access in a loop that runs once per
distinct descriptor value. The loop does ``v_readfirstlane`` into SGPRs, compares, does
``s_and_saveexec``, makes the access and branches back. One common cause is a value
loaded through a generic pointer: flat loads count as divergent.

Round 5 found 32 such loops per grouped MoE prefill kernel. The cause was the expert index
read through ``PwGroup::tile_expert``. With ``readfirstlane`` on that index the grouped
kernel runs at the dense kernel's rate:
* Mixtral 8K: 6.00 -> 4.79 ms per layer.
* Qwen3-30B-A3B 8K: 1.02 -> 0.88 ms per layer.
See ``profiles/r5_moe_grouped_waterfall_fix.log``.

    python tools/waterfall_check.py [file.hip ...]   # default: every kernel source
Exits 1 when any kernel has one and lists them.
"""
from __future__ import annotations

import collections
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics", "-ffp-contract=fast",
         "-I", os.path.join(ROOT, "csrc", "include"), "-S", "--cuda-device-only"]


def waterfalls(asm: str) -> dict[str, int]:
    """kernel symbol -> number of short backward-branch loops that re-read a VGPR into
    SGPRs and narrow exec around the access."""
    lines = asm.split("\n")
    kern, labels, hits = None, {}, collections.Counter()
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            kern = m.group(1)
        m = re.match(r"^(\.LBB\d+_\d+):", ln)
        if m:
            labels[m.group(1)] = i
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)", ln)
        if m and m.group(1) in labels:
            body = lines[labels[m.group(1)]:i + 1]
            if (len(body) < 40 and any("v_readfirstlane" in b for b in body)
                    and any("saveexec" in b for b in body)):
                hits[kern] += 1
    return dict(hits)


def check(src: str) -> dict[str, int]:
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "k.s")
        subprocess.run([HIPCC, *FLAGS, src, "-o", out], check=True, capture_output=True)
        with open(out) as f:
            return waterfalls(f.read())


def main(argv):
    srcs = argv or sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))
    bad = 0
    for s in srcs:
        for k, n in check(s).items():
            print(f"{os.path.basename(s)}: {n} waterfall loop(s) in {k}")
            bad += 1
    print("ok" if not bad else f"{bad} kernel(s) with waterfall loops")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
