#!/bin/bash
# Round 3 (session 3): decode-tile GEMM with hoisted fragment offsets and a ring-unrolled K loop — GEMM op tests,
# same-box bench A/B against the previous build (light-whisper_amd/libqasr_base.so), decode GEMM kernel stats.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3v}
root=$(pwd)
mkdir -p $out
timeout -k 10 400 python3 -u -m pytest tests/test_ops_gpu.py -q -k "gemm or exact or verify" --timeout 240 \
    --timeout-method thread -p no:cacheprovider > $out/${tag}_tests.log 2>&1 || { tail -n 30 $out/${tag}_tests.log; exit 1; }
echo "tests ok" > $out/${tag}_progress.log
timeout -k 10 1000 bash tools/gpu_ab.sh light-whisper_amd/libqasr_base.so light-whisper_amd/libqasr.so 3 > $out/${tag}_ab.log 2>&1 || exit 1
echo "ab done" >> $out/${tag}_progress.log
cd /tmp && export TMPDIR=/tmp
for L in base new; do
  lib=$root/light-whisper_amd/libqasr.so; [ $L = base ] && lib=$root/light-whisper_amd/libqasr_base.so
  QASR_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_${tag}_$L -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $out/${tag}_bench_$L.log 2>&1 || exit 1
  cp $(find /tmp/kt_${tag}_$L -name '*kernel_stats.csv' | head -n 1) $out/${tag}_kstats_$L.csv
done
echo "kstats done" >> $out/${tag}_progress.log
