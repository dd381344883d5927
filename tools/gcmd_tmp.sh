set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ops.log 2>&1 || { tail -n 40 gpurun_out/t_ops.log; exit 1; }
tail -n 2 gpurun_out/t_ops.log
PATHS=2,18,22,27,28,29,30,43,59 timeout -k 10 300 python -u tools/gemm_tune.py > gpurun_out/tune.log 2>&1 || { tail -n 20 gpurun_out/tune.log; exit 1; }
cat gpurun_out/tune.log
