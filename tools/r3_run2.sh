#!/bin/bash
# Round 3, GPU pass 2: fusion diagnosis (current and round-2 builds), the GPU suite, the deterministic bench with the
# deterministic decode tables.
set -o pipefail
out=$(pwd)/gpurun_out
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/r3b_progress.log; exit $rc; }; }
timeout -k 10 200 python3 -u tools/diag_fusion.py > $out/r3b_diag.log 2>&1
rc=$?; echo "diag rc $rc" >> $out/r3b_progress.log; ok $rc
QASR_LIB=$(pwd)/ab/r2/libqasr.so timeout -k 10 200 python3 -u tools/diag_fusion.py >> $out/r3b_diag.log 2>&1
rc=$?; echo "diag r2 rc $rc" >> $out/r3b_progress.log; ok $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --maxfail=25 --timeout 240 --timeout-method thread -p no:cacheprovider \
    > $out/r3b_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $out/r3b_progress.log; ok $rc
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/r3b_bench_det.log 2>&1
rc=$?; echo "bench det rc $rc" >> $out/r3b_progress.log; ok $rc
