set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -n 60 gpurun_out/t_all.log; exit 1; }
tail -n 1 gpurun_out/t_all.log
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -n 20 gpurun_out/b.log; exit 1; }
tail -n 1 gpurun_out/b.log | cut -c1-1500
