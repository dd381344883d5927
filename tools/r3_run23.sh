#!/bin/bash
# Round 3 (session 3): packed-fma rescale (v_pk_fma_f32) in the LDS-DMA GEMM — GEMM op tests, same-box bench A/B of
# base (round-3 final build) / offsets only (QASR_PKFMA=0) / offsets + packed fma, kernel stats of the new build.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3w}
root=$(pwd)
mkdir -p $out
timeout -k 10 400 python3 -u -m pytest tests/test_ops_gpu.py -q -k "gemm or exact or verify or chain" --timeout 240 \
    --timeout-method thread -p no:cacheprovider > $out/${tag}_tests.log 2>&1 || { tail -n 30 $out/${tag}_tests.log; exit 1; }
echo "tests ok" > $out/${tag}_progress.log
L=light-whisper_amd
for i in 1 2; do
  timeout -k 10 1000 bash tools/gpu_ab.sh $L/libqasr_base.so $L/libqasr_nopk.so 1 >> $out/${tag}_ab.log 2>&1 || exit 1
  timeout -k 10 1000 bash tools/gpu_ab.sh $L/libqasr.so "" 1 >> $out/${tag}_ab.log 2>&1 || exit 1
done
echo "ab done" >> $out/${tag}_progress.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_${tag} -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $out/${tag}_bench_new.log 2>&1 || exit 1
cp $(find /tmp/kt_${tag} -name '*kernel_stats.csv' | head -n 1) $out/${tag}_kstats_new.csv
echo "kstats done" >> $out/${tag}_progress.log
