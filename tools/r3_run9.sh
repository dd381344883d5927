#!/bin/bash
# Round 3 (session 2): verify-pass drift diagnosis at 32 rows; same-box A/B of the residual-GEMM norm fusion.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3i}
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || { echo "stopping: rc $rc" >> $out/${tag}_progress.log; exit $rc; }; }
timeout -k 10 300 python3 -u tools/diag_layers.py qwen3-asr-1.7b 4 32 > $out/${tag}_layers.log 2>&1
ok $?; echo "layers done" >> $out/${tag}_progress.log
for r in 1 2; do
  QASR_NO_NORM_FUSE=1 timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $out/${tag}_bench_nofuse_$r.log 2>&1
  ok $?
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $out/${tag}_bench_fuse_$r.log 2>&1
  ok $?; echo "ab $r done" >> $out/${tag}_progress.log
done
