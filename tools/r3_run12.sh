#!/bin/bash
# Round 3 (session 2): after -ffp-contract=off — row-level GEMV check, the verify-pass test, the whole GPU suite, bench.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3l}
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/${tag}_progress.log; exit $rc; }; }
timeout -k 10 400 python3 -u tools/diag_gemv_rows.py qwen3-asr-1.7b 16 4 32 31 2,9 > $out/${tag}_gemv_rows.log 2>&1
ok $?; echo "gemv rows done" >> $out/${tag}_progress.log
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --maxfail=25 --timeout 240 --timeout-method thread \
    -p no:cacheprovider > $out/${tag}_tests.log 2>&1
ok $?; echo "tests done" >> $out/${tag}_progress.log
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $out/${tag}_bench.log 2>&1
ok $?; echo "bench done" >> $out/${tag}_progress.log
