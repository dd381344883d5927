#!/bin/bash
# Full GPU-box check: parity tests, the default bench line, a kernel-trace profile of the same bench.
# usage (on the box, from the repo root): tools/round_check.sh <tag>
set -o pipefail
tag=${1:-run}
root=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$tag.log 2>&1 || { tail -n 40 gpurun_out/t_$tag.log; exit 1; }
tail -n 2 gpurun_out/t_$tag.log
timeout -k 10 400 python3 bench.py > gpurun_out/b_$tag.log 2>&1 || { tail -n 20 gpurun_out/b_$tag.log; exit 1; }
tail -n 1 gpurun_out/b_$tag.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/prof_$tag -o run -- python3 $root/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $root/gpurun_out/p_$tag.log 2>&1 || { tail -n 20 $root/gpurun_out/p_$tag.log; exit 1; }
grep '"value"' $root/gpurun_out/p_$tag.log | cut -c1-300
