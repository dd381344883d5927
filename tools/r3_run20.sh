#!/bin/bash
# Round 3 (session 2): verify passes through the bucket graphs — tests, in-graph pass cost by row count, C3 sweep.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3t}
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/${tag}_progress.log; exit $rc; }; }
timeout -k 10 600 python3 -u -m pytest tests/test_ops_gpu.py tests/test_model_real_gpu.py tests/test_model_gpu.py tests/test_serve_gpu.py -q \
    -k "exact or verify or draft or streaming or interim or gemv or attention or swiglu" --timeout 240 --timeout-method thread -p no:cacheprovider > $out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $out/${tag}_progress.log; ok $rc
timeout -k 10 300 python3 -u tools/verify_cost.py qwen3-asr-1.7b 1,2,4,8,16,32 > $out/${tag}_verify_cost.log 2>&1
ok $?; echo "cost done" >> $out/${tag}_progress.log
for nz in 0 0.05 0.2 0.5; do
  timeout -k 10 240 python3 -u tools/stream_bench.py --speech-only --draft 1 --draft-noise $nz > $out/${tag}_c3_draft_noise$nz.json 2> $out/${tag}_c3_$nz.err
  ok $?; echo "c3 $nz done" >> $out/${tag}_progress.log
done
