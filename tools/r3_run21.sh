#!/bin/bash
# Round 3 (session 2): exact-row kernel with both row fragments per workgroup — tests, per-bucket pass cost (kernel
# time), C3 draft-noise sweep.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3u}
root=$(pwd)
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/${tag}_progress.log; exit $rc; }; }
timeout -k 10 600 python3 -u -m pytest tests/test_ops_gpu.py tests/test_model_real_gpu.py tests/test_model_gpu.py tests/test_serve_gpu.py -q \
    -k "exact or verify or draft or streaming or interim or gemv or attention or swiglu" --timeout 240 --timeout-method thread -p no:cacheprovider > $out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $out/${tag}_progress.log; ok $rc
cd /tmp && export TMPDIR=/tmp
for n in 1 2 4 8 16 32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/kt_${tag}_$n -o run --output-format csv -- python3 $root/tools/verify_cost.py qwen3-asr-1.7b $n > $out/${tag}_prof_$n.log 2>&1 || exit 1
  cp $(find /tmp/kt_${tag}_$n -name '*kernel_stats.csv' | head -n 1) $out/${tag}_kstats_$n.csv
done
cd $root
python3 tools/pass_cost.py $out/${tag}_kstats_1.csv $out/${tag}_kstats_2.csv $out/${tag}_kstats_4.csv $out/${tag}_kstats_8.csv $out/${tag}_kstats_16.csv $out/${tag}_kstats_32.csv > $out/${tag}_pass_cost.log 2>&1
echo "pass cost done" >> $out/${tag}_progress.log
for nz in 0 0.05 0.2 0.5; do
  timeout -k 10 240 python3 -u tools/stream_bench.py --speech-only --draft 1 --draft-noise $nz > $out/${tag}_c3_draft_noise$nz.json 2> $out/${tag}_c3_$nz.err
  ok $?; echo "c3 $nz done" >> $out/${tag}_progress.log
done
