#!/bin/bash
# Round 3 (session 2): decode attention q-row padding + V preload for split-range launches — op tests, then a
# same-box A/B of C2 latency (base = the previous kernels_attn.hip build).
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3o}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_ops_gpu.py tests/test_model_real_gpu.py -q -k "attention or attn or verify or fusion or draft" \
    --timeout 240 --timeout-method thread -p no:cacheprovider > $out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $out/${tag}_progress.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  QASR_LIB=$(pwd)/light-whisper_amd/libqasr_base.so timeout -k 10 240 python3 -u tools/latency.py qwen3-asr-1.7b 1,5,12 > $out/${tag}_lat_base_$r.jsonl 2>&1 || exit 1
  timeout -k 10 240 python3 -u tools/latency.py qwen3-asr-1.7b 1,5,12 > $out/${tag}_lat_new_$r.jsonl 2>&1 || exit 1
  echo "ab $r done" >> $out/${tag}_progress.log
done
