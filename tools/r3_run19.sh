#!/bin/bash
# Round 3 (session 2): exact-row tests after the T=3 fix; kernel stats of verify passes at 8 and 32 rows.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3s}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_ops_gpu.py tests/test_model_real_gpu.py tests/test_model_gpu.py tests/test_serve_gpu.py -q \
    -k "exact or verify or draft or streaming or interim or gemv or attention" --timeout 240 --timeout-method thread -p no:cacheprovider > $out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $out/${tag}_progress.log; [ $rc -le 1 ] || exit $rc
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for n in 1 8 32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_${tag}_$n -o run --output-format csv -- python3 $root/tools/verify_cost.py qwen3-asr-1.7b $n > $out/${tag}_prof_$n.log 2>&1 || exit 1
  cp $(find /tmp/kt_${tag}_$n -name '*kernel_stats.csv' | head -n 1) $out/${tag}_kernel_stats_$n.csv
  echo "prof $n done" >> $out/${tag}_progress.log
done
