#!/bin/bash
# Round 3 (session 2): kernel stats of 32-row verify passes on the exact-row MFMA linears.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3r}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_$tag -o run --output-format csv -- python3 $OLDPWD/tools/verify_cost.py qwen3-asr-1.7b 32 > $out/${tag}_prof.log 2>&1 || exit 1
cp $(find /tmp/kt_$tag -name '*kernel_stats.csv' | head -n 1) $out/${tag}_kernel_stats.csv
