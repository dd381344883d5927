#!/bin/bash
# Round 3 (session 2): verify-pass drift at the test's inputs; A-stationary GEMM tests + decode-shape sweep.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3j}
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/${tag}_progress.log; exit $rc; }; }
timeout -k 10 300 python3 -u tools/diag_layers.py qwen3-asr-1.7b 4 32 31 2,9 > $out/${tag}_layers.log 2>&1
ok $?; echo "layers done" >> $out/${tag}_progress.log
timeout -k 10 600 python3 -u -m pytest tests/test_ops_gpu.py -q -x -k "as_ or resid_rmsq8" --timeout 240 --timeout-method thread \
    -p no:cacheprovider > $out/${tag}_tests.log 2>&1
ok $?; echo "tests done" >> $out/${tag}_progress.log
CFGS=12,14,15,16,22,24,31,32,33,34,35,36,37 timeout -k 10 600 python3 -u tools/dec_gemm_sweep.py $out/${tag}_sweep.json > $out/${tag}_sweep.log 2>&1
ok $?; echo "sweep done" >> $out/${tag}_progress.log
