# prefill row padding: engine tests, probe table, gateway bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pad
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_families_gpu.py tests/test_vision_gpu.py > gpurun_out/pad/tests.log 2>&1 || { tail -30 gpurun_out/pad/tests.log; exit 1; }
tail -1 gpurun_out/pad/tests.log
HIPSERVE_STEP_LOG=$GRAFT_REPO_ROOT/gpurun_out/pad/steps.jsonl timeout -k 10 480 python -u bench.py --steps 3 --warmup 1 --out gpurun_out/pad/bench.json > gpurun_out/pad/bench.log 2>&1 || exit 1
tail -1 gpurun_out/pad/bench.log | cut -c1-260
timeout -k 10 200 python -u -c "
import torch
from hipserve.config import EngineConfig
from hipserve.engine.model_runner import ModelRunner
from hipserve.config import PRESETS
from hipserve.parallel.comm import TPGroup
cfg = EngineConfig(model='llama-3-8b', load_format='dummy', device='cuda', max_num_seqs=64, max_num_batched_tokens=8192, max_model_len=2048, num_kv_blocks=1024, extra={'gemm_autotune': False})
r = ModelRunner(cfg, PRESETS['llama-3-8b'], TPGroup(0, 1, None, torch.device('cuda', 0)))
print('pad', r.prefill_pad); print('times', r.prefill_pad_times)
" > gpurun_out/pad/probe.log 2>&1 || exit 1
tail -2 gpurun_out/pad/probe.log
