#!/bin/bash
# Round-end evidence on the GPU box (repo root), in two phases so each fits one gpurun call (round 6: + the C5 line):
#   tools/final_round_r6.sh <tag> a   graph-replayed kernel trace + per-class trace JSON, PMC passes, the default bench
#   tools/final_round_r6.sh <tag> b   32 / 64-segment shares (+ kernel trace of the 32-segment share), C3 streams, C2
set -o pipefail
tag=${1:-r6}; phase=${2:-a}
root=$(pwd)
out=$root/gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
if [ "$phase" = a ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/kt_$tag -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --no-prof --steps 2 --warmup 1 > $out/${tag}_prof_bench.log 2>&1 || { tail -n 20 $out/${tag}_prof_bench.log; exit 1; }
  cp $(find /tmp/kt_$tag -name '*kernel_stats.csv' | head -n 1) $out/${tag}_kernel_stats.csv
  python3 $root/tools/trace_classes.py $out/${tag}_trace_classes.json 4 $(find /tmp/kt_$tag -name '*kernel_trace.csv' | head -n 1) > $out/${tag}_trace_classes.log || exit 1
  echo "kernel trace done" >> $out/${tag}_progress.log
  cd $root
  bash tools/pmc_round.sh $tag > $out/${tag}_pmc.log 2>&1 || { tail -n 20 $out/${tag}_pmc.log; exit 1; }
  cp $out/pmc_$tag.json $out/${tag}_pmc_classes.json
  echo "pmc done" >> $out/${tag}_progress.log
  # the bench line, after the committed-evidence files exist on this box (trace classes + PMC of this very build)
  cp $out/${tag}_trace_classes.json $root/profiles/ && cp $out/${tag}_pmc_classes.json $root/profiles/
  timeout -k 10 400 python3 -u bench.py > $out/${tag}_bench.log 2>&1 || { tail -n 20 $out/${tag}_bench.log; exit 1; }
  echo "bench done" >> $out/${tag}_progress.log
else
  cd $root
  timeout -k 10 400 python3 -u bench.py > $out/${tag}_bench_b.log 2>&1 || exit 1   # (phase a's line is ${tag}_bench.log)
  echo "bench (repeat) done" >> $out/${tag}_progress.log
  timeout -k 10 300 python3 -u bench.py --segments 32 --no-cpu-baseline > $out/${tag}_seg32.log 2>&1 || exit 1
  timeout -k 10 300 python3 -u bench.py --segments 64 --no-cpu-baseline > $out/${tag}_seg64.log 2>&1 || exit 1
  echo "shares done" >> $out/${tag}_progress.log
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt32_$tag -o run --output-format csv -- python3 $root/bench.py --segments 32 --no-cpu-baseline --no-prof --steps 2 --warmup 1 > $out/${tag}_seg32_prof.log 2>&1 || exit 1
  cp $(find /tmp/kt32_$tag -name '*kernel_stats.csv' | head -n 1) $out/${tag}_seg32_kernel_stats.csv
  cd $root
  echo "seg32 trace done" >> $out/${tag}_progress.log
  timeout -k 10 300 python3 -u tools/stream_bench.py --speech-only --draft 1 > $out/${tag}_c3_draft.json 2> $out/${tag}_c3_draft.err || exit 1
  echo "c3 done" >> $out/${tag}_progress.log
  timeout -k 10 300 python3 -u tools/latency.py > $out/${tag}_latency.jsonl 2> $out/${tag}_latency.err || exit 1
  echo "c2 done" >> $out/${tag}_progress.log
  timeout -k 10 400 python3 -u bench.py --workload c5 --no-cpu-baseline > $out/${tag}_c5.log 2>&1 || exit 1
  echo "c5 done" >> $out/${tag}_progress.log
fi
