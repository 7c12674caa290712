"""The built kernel library loads on a CPU host (dlopen resolves every symbol: a launcher
declared in kernels.h but left undefined fails here, not on the GPU box) and registers
the ops the Python layer calls."""
import os

import pytest
import torch

from hipserve.ops import library_path


@pytest.mark.skipif(not os.path.exists(library_path()), reason="hipserve/_C.so not built")
def test_library_loads_and_registers_ops():
    from hipserve.ops import load_library

    load_library()
    for op in ("decode_gemm_partial", "gguf_gemm_parts", "fp8_untile", "gguf_dequant_tiled", "paged_decode",
               "splitk_add_rmsnorm", "prefill_gemm_packed", "fp8_decode_gemm"):
        assert hasattr(torch.ops.hipserve, op), op
