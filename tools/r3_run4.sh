#!/bin/bash
# Round 3, GPU pass 4: the row-group diagnosis of the 1.7B verify pass, the GPU suite (parity log kept), the bench.
set -o pipefail
out=$(pwd)/gpurun_out
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/r3d_progress.log; exit $rc; }; }
timeout -k 10 400 python3 -u tools/diag_verify.py qwen3-asr-1.7b 20 17 > $out/r3d_diag.log 2>&1
rc=$?; echo "diag rc $rc" >> $out/r3d_progress.log; ok $rc
QASR_PARITY_LOG=$out/r3d_parity.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --maxfail=25 --timeout 240 \
    --timeout-method thread -p no:cacheprovider > $out/r3d_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $out/r3d_progress.log; ok $rc
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/r3d_bench.log 2>&1
rc=$?; echo "bench rc $rc" >> $out/r3d_progress.log; ok $rc
