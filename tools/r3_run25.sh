#!/bin/bash
# Round 3 (session 3): the 8-wave 256×256 LDS-DMA tile (GEMM config 31) — op tests, then prefill-shape timing against
# the 128×128 tile (config 4) under rocprofv3 kernel trace.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3aa}
root=$(pwd)
mkdir -p $out
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python3 -u -m pytest tests/test_ops_gpu.py -q -k "linear_q8 or chain or fused_epilogues or swiglu" \
    --timeout 240 --timeout-method thread -p no:cacheprovider -x > $out/${tag}_tests.log 2>&1 || { tail -n 30 $out/${tag}_tests.log; exit 1; }
echo "tests ok" > $out/${tag}_progress.log
cd /tmp && export TMPDIR=/tmp
for cfg in 4 31; do
  for shape in "8192 4096 2048 0" "8192 2048 6144 1" "8192 12288 2048 0" "8192 2048 2048 1" "25000 4096 2048 0" "2048 4096 2048 0"; do
    nm=$(echo $shape | tr ' ' '_')
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/kt_${tag}_${cfg}_$nm -o run --output-format csv -- python3 $root/tools/gemm_one.py $shape $((16 + cfg)) 20 > $out/${tag}_${cfg}_$nm.log 2>&1 || exit 1
    cp $(find /tmp/kt_${tag}_${cfg}_$nm -name '*kernel_stats.csv' | head -n 1) $out/${tag}_${cfg}_$nm.csv
  done
  echo "cfg $cfg done" >> $out/${tag}_progress.log
done
