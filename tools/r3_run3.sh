#!/bin/bash
# Round 3, GPU pass 3: verify-pass diagnosis at 1.7B / 20 s; the GPU suite; the bench (det tables validated).
set -o pipefail
out=$(pwd)/gpurun_out
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/r3c_progress.log; exit $rc; }; }
timeout -k 10 300 python3 -u tools/diag_verify.py qwen3-asr-1.7b 20 17 > $out/r3c_diag.log 2>&1
rc=$?; echo "diag rc $rc" >> $out/r3c_progress.log; ok $rc
timeout -k 10 300 python3 -u tools/diag_verify.py qwen3-asr-0.6b 20 17 >> $out/r3c_diag.log 2>&1
rc=$?; echo "diag 0.6b rc $rc" >> $out/r3c_progress.log; ok $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --maxfail=25 --timeout 240 --timeout-method thread -p no:cacheprovider \
    > $out/r3c_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $out/r3c_progress.log; ok $rc
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/r3c_bench.log 2>&1
rc=$?; echo "bench rc $rc" >> $out/r3c_progress.log; ok $rc
