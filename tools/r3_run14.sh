#!/bin/bash
# Round 3 (session 2): A-stationary decode GEMM v2 — op tests, exact-row GEMV tests, decode-shape sweep.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3n}
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/${tag}_progress.log; exit $rc; }; }
timeout -k 10 600 python3 -u -m pytest tests/test_ops_gpu.py -q -k "as_ or resid_rmsq8 or gemv" --timeout 240 --timeout-method thread \
    -p no:cacheprovider > $out/${tag}_tests.log 2>&1
ok $?; echo "tests done" >> $out/${tag}_progress.log
CFGS=12,14,15,16,22,24,31,32,33 timeout -k 10 600 python3 -u tools/dec_gemm_sweep.py $out/${tag}_sweep.json > $out/${tag}_sweep.log 2>&1
ok $?; echo "sweep done" >> $out/${tag}_progress.log
