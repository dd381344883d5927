set -o pipefail
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $root/gpurun_out/prof_q -o run -- python3 $root/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $root/gpurun_out/p_q.log 2>&1 || { tail -n 20 $root/gpurun_out/p_q.log; exit 1; }
