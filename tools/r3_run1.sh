#!/bin/bash
# Round 3, first GPU pass: the GPU suite (exact-row / stable-order / streaming identity tests), the bench in the
# default deterministic mode and with f32 split-K atomics (QASR_ATOMICS=1), C2 latency, and the deterministic
# decode-GEMM sweep.  Test failures do not stop the script; a crash, abort or time limit does.
set -o pipefail
out=$(pwd)/gpurun_out
mkdir -p $out
nproc > $out/r3a_nproc.txt
ok() {   # 0 = fine, 1 = assertion failures (go on); anything else (abort, segfault, time limit) = stop
    local rc=$1
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/r3a_progress.log; exit $rc; }
}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --maxfail=25 --timeout 240 --timeout-method thread -p no:cacheprovider \
    > $out/r3a_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $out/r3a_progress.log; ok $rc
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/r3a_bench_det.log 2>&1
rc=$?; echo "bench det rc $rc" >> $out/r3a_progress.log; ok $rc
QASR_ATOMICS=1 timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $out/r3a_bench_atomics.log 2>&1
rc=$?; echo "bench atomics rc $rc" >> $out/r3a_progress.log; ok $rc
timeout -k 10 300 python3 -u tools/latency.py > $out/r3a_latency.jsonl 2> $out/r3a_latency.err
rc=$?; echo "latency rc $rc" >> $out/r3a_progress.log; ok $rc
timeout -k 10 900 python3 -u tools/dec_gemm_sweep.py $out/r3a_dec_sweep_det.json > $out/r3a_dec_sweep_det.log 2>&1
rc=$?; echo "sweep rc $rc" >> $out/r3a_progress.log; ok $rc
