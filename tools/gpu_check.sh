#!/bin/bash
# GPU-box check used during development: parity tests, then a kernel-trace profile of one bench step.
# usage (on the box, from the repo root): tools/gpu_check.sh <tag> [pytest files...]
set -o pipefail
tag=${1:-run}; shift
files=${@:-tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_vad_gpu.py}
timeout -k 10 300 python -m pytest $files -x -q > gpurun_out/t_$tag.log 2>&1 || { tail -n 30 gpurun_out/t_$tag.log; exit 1; }
tail -n 1 gpurun_out/t_$tag.log
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/prof_$tag -o run -- python3 $root/bench.py --no-cpu-baseline --no-prof --steps 1 --warmup 1 > $root/gpurun_out/p_$tag.log 2>&1 || { tail -n 20 $root/gpurun_out/p_$tag.log; exit 1; }
grep -o '"value": [0-9.]*' $root/gpurun_out/p_$tag.log
