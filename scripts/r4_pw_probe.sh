set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/bench_pw_scaling.py > gpurun_out/pw_scaling.log 2>&1; cat gpurun_out/pw_scaling.log
PG_VARIANTS="p1 p2" bash scripts/pg_pmc.sh
