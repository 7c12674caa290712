cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 300 python -u -m cProfile -o gpurun_out/host.prof bench.py --path engine --steps 1 --warmup 1 > gpurun_out/hp.log 2>&1 && python -c "
import pstats; p=pstats.Stats('gpurun_out/host.prof'); p.sort_stats('tottime').print_stats(45)" > gpurun_out/host_tottime.txt && python -c "
import pstats; p=pstats.Stats('gpurun_out/host.prof'); p.sort_stats('cumulative').print_stats(60)" > gpurun_out/host_cum.txt && tail -1 gpurun_out/hp.log
