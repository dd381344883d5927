#!/bin/bash
# Round 3 (session 2): phase trace of the A-stationary decode GEMM (debug build).
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3m}
mkdir -p $out
export QASR_LIB=$(pwd)/light-whisper_amd/libqasr_trace.so
for a in "32 256 4096 2048" "31 256 4096 2048" "32 16 4096 2048" "35 256 12288 2048"; do
  timeout -k 10 120 python3 -u tools/as_trace.py $a >> $out/${tag}_as_trace.log 2>&1 || { echo "rc $? on $a" >> $out/${tag}_progress.log; exit 1; }
done
echo done >> $out/${tag}_progress.log
