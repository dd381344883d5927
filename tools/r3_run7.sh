#!/bin/bash
# Round 3: the layer-by-layer verify-vs-steps diagnosis after pinning the row arithmetic, then the whole GPU suite.
set -o pipefail
out=$(pwd)/gpurun_out
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/r3g_progress.log; exit $rc; }; }
timeout -k 10 300 python3 -u tools/diag_layers.py qwen3-asr-1.7b 20 17 > $out/r3g_layers.log 2>&1
rc=$?; echo "layers rc $rc" >> $out/r3g_progress.log; ok $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --maxfail=25 --timeout 240 --timeout-method thread \
    -p no:cacheprovider > $out/r3g_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $out/r3g_progress.log; ok $rc
