#!/bin/bash
# rocprofv3 kernel trace of one engine-path bench wave, summarised by tools/prof_db.py.
#   bash tools/prof_bench.sh <name> <bench.py args...>   ->  gpurun_out/<name>_trace.md
set -o pipefail
name=$1; shift
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/pb_$name -o run -- python3 $GRAFT_REPO_ROOT/bench.py --path engine --steps 1 --warmup 0 "$@" > $GRAFT_REPO_ROOT/gpurun_out/${name}_prof.log 2>&1 && \
cd $GRAFT_REPO_ROOT && python tools/prof_db.py /tmp/pb_$name/run_results.db gpurun_out/${name}_trace.md "$name" > /dev/null && \
grep -A 30 "per decode step" gpurun_out/${name}_trace.md
