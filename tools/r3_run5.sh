#!/bin/bash
set -o pipefail
out=$(pwd)/gpurun_out
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/r3e_progress.log; exit $rc; }; }
timeout -k 10 200 python3 -u -m pytest tests/test_ops_gpu.py -q -k "verify_rows or exact_rows" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $out/r3e_ops.log 2>&1
rc=$?; echo "ops rc $rc" >> $out/r3e_progress.log; ok $rc
timeout -k 10 500 python3 -u tools/diag_verify.py qwen3-asr-1.7b 20 17 > $out/r3e_diag.log 2>&1
rc=$?; echo "diag rc $rc" >> $out/r3e_progress.log; ok $rc
