"""Device-code regression guard: the kernels that carry per-workgroup indirection
(grouped MoE prefill GEMM, MoE decode GEMM, paged attention) must not compile to
waterfall loops around their buffer loads (tools/waterfall_check.py). Runs hipcc -S on
the CPU; skipped where hipcc is absent."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import waterfall_check as wc  # noqa: E402

pytestmark = pytest.mark.skipif(not os.path.exists(wc.HIPCC), reason="hipcc not installed")


def test_detector_flags_a_waterfall():
    asm = "\n".join(["_Z3fooPi:", ".LBB0_1:", "\tv_readfirstlane_b32 s4, v2", "\tv_cmp_eq_u32_e32 vcc, s4, v2",
                     "\ts_and_saveexec_b64 s[0:1], vcc", "\tbuffer_load_dword v3, v1, s[4:7], 0 offen",
                     "\ts_xor_b64 exec, exec, s[0:1]", "\ts_cbranch_execnz .LBB0_1"])
    assert wc.waterfalls(asm) == {"_Z3fooPi": 1}
    assert wc.waterfalls(asm.replace("v_readfirstlane_b32 s4, v2", "s_mov_b32 s4, s2")) == {}


@pytest.mark.parametrize("src", ["prefill_gemm_packed.hip", "decode_gemm.hip", "attention_decode.hip", "moe.hip"])
def test_no_waterfall_loops(src):
    path = os.path.join(ROOT, "csrc", "kernels", src)
    if not os.path.exists(path):
        pytest.skip(f"{src} not in this tree")
    assert wc.check(path) == {}
