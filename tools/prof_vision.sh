set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vision_gpu.py > gpurun_out/vision_gpu.log 2>&1 && \
timeout -k 10 300 python tools/bench_vision.py --size 1024 --images 4 --iters 10 > gpurun_out/bench_vision.json 2> gpurun_out/bench_vision.err && \
timeout -k 10 300 python tools/bench_vision.py --size 448 --images 16 --iters 10 >> gpurun_out/bench_vision.json 2>> gpurun_out/bench_vision.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/vp -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_vision.py --size 1024 --images 4 --iters 5 > $GRAFT_REPO_ROOT/gpurun_out/vis_prof.log 2>&1 && \
cd $GRAFT_REPO_ROOT && python tools/prof_db.py /tmp/vp/run_results.db gpurun_out/vision_prof.md "Qwen3-VL vision tower, 4 x 1024x1024 images" > /dev/null && tail -2 gpurun_out/vision_gpu.log && cat gpurun_out/bench_vision.json && head -20 gpurun_out/vision_prof.md
