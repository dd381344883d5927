#!/bin/bash
set -o pipefail
out=$(pwd)/gpurun_out
mkdir -p $out
timeout -k 10 300 python3 -u tools/diag_layers.py qwen3-asr-1.7b 20 17 > $out/r3f_layers.log 2>&1
echo "layers rc $?" >> $out/r3f_progress.log
