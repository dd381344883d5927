#!/bin/bash
# Round 3 (session 2): row-level check of the fused norm + QKV GEMV on the verify pass's layer-16 rows.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3k}
mkdir -p $out
timeout -k 10 400 python3 -u tools/diag_gemv_rows.py qwen3-asr-1.7b 16 4 32 31 2,9 > $out/${tag}_gemv_rows.log 2>&1
echo "rc $?" >> $out/${tag}_progress.log
