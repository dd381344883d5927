#!/bin/bash
# Round 3 (session 3) diagnostic: how much of the Q8 GEMM's time is the exact rescale?  The same GEMM shapes through
# the product library and through light-whisper_amd/libqasr_diag.so (built with -DQASR_DIAG_NORESCALE=1: one integer
# add per MFMA instead of cvt + fma — wrong results, timing only), kernel trace + stats for each.
# libqasr_diag.so: git apply tools/diag_norescale.patch; make -C light-whisper_amd BUILD=build_diag LIB=libqasr_diag.so
#   EXTRA=-DQASR_DIAG_NORESCALE=1 libqasr_diag.so; git checkout light-whisper_amd/csrc/kernels_q8.hip
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3y}
root=$(pwd)
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for L in prod diag; do
  lib=$root/light-whisper_amd/libqasr.so; [ $L = diag ] && lib=$root/light-whisper_amd/libqasr_diag.so
  for shape in "8192 4096 2048 0" "8192 2048 6144 1" "256 4096 2048 0" "128 2048 6144 1"; do
    nm=$(echo $shape | tr ' ' '_')
    QASR_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/kt_${tag}_${L}_$nm -o run --output-format csv -- python3 $root/tools/gemm_one.py $shape 0 20 > $out/${tag}_${L}_$nm.log 2>&1 || exit 1
    cp $(find /tmp/kt_${tag}_${L}_$nm -name '*kernel_stats.csv' | head -n 1) $out/${tag}_${L}_$nm.csv
  done
  echo "$L done" >> $out/${tag}_progress.log
done
