#!/bin/bash
# Round 3 (session 3): packed scale-multiply / fma in the exact-row verify kernel (k_gemm_q8_exact) — exact-row tests
# on the packed build, then C3 streaming A/B (draft noise 0 / 5 %) base vs packed, swapping the engine's libqasr.so.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3ad}
L=light-whisper_amd
mkdir -p $out
cp $L/libqasr_pk.so $L/libqasr.so
timeout -k 10 500 python3 -u -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_model_real_gpu.py -q \
    -k "exact_rows or verify or draft" --timeout 240 --timeout-method thread -p no:cacheprovider -x \
    > $out/${tag}_tests.log 2>&1 || { tail -n 30 $out/${tag}_tests.log; cp $L/libqasr_base.so $L/libqasr.so; exit 1; }
echo "tests ok" > $out/${tag}_progress.log
for i in 1 2; do
  for v in base pk; do
    cp $L/libqasr_$v.so $L/libqasr.so
    for nz in 0 0.05; do
      timeout -k 10 240 python3 -u tools/stream_bench.py --speech-only --draft 1 --draft-noise $nz > $out/${tag}_${v}_${i}_c3_$nz.json 2> $out/${tag}_${v}_${i}_c3_$nz.err || exit 1
    done
    echo "$v $i done" >> $out/${tag}_progress.log
  done
done
cp $L/libqasr_base.so $L/libqasr.so
