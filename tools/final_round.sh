#!/bin/bash
# Round-end evidence on the GPU box (repo root): bench kernel trace + stats, per-class PMC passes, the default bench
# line (with the CPU baseline), and the C3 streaming runs.  usage: tools/final_round.sh <tag>
set -o pipefail
tag=${1:-r2f}
root=$(pwd)
out=$root/gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
# graph-replayed steps only (--no-prof: no eager instrumented step): 1 warm-up + 2 timed + the results step = 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/kt_$tag -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --no-prof --steps 2 --warmup 1 > $out/${tag}_prof_bench.log 2>&1 || { tail -n 20 $out/${tag}_prof_bench.log; exit 1; }
cp $(find /tmp/kt_$tag -name '*kernel_stats.csv' | head -n 1) $out/${tag}_kernel_stats.csv
python3 $root/tools/trace_classes.py $out/${tag}_trace_classes.json 4 $(find /tmp/kt_$tag -name '*kernel_trace.csv' | head -n 1) > /dev/null || exit 1
echo "kernel trace done" >> $out/${tag}_progress.log
cd $root
bash tools/pmc_round.sh $tag > $out/${tag}_pmc.log 2>&1 || { tail -n 20 $out/${tag}_pmc.log; exit 1; }
echo "pmc done" >> $out/${tag}_progress.log
timeout -k 10 400 python3 -u bench.py > $out/${tag}_bench.log 2>&1 || { tail -n 20 $out/${tag}_bench.log; exit 1; }
echo "bench done" >> $out/${tag}_progress.log
timeout -k 10 300 python3 -u tools/stream_bench.py --speech-only --draft 1 > $out/${tag}_c3_draft.json 2> $out/${tag}_c3_draft.err || exit 1
timeout -k 10 300 python3 -u tools/stream_bench.py --speech-only --draft 0 > $out/${tag}_c3_nodraft.json 2> $out/${tag}_c3_nodraft.err || exit 1
echo "c3 done" >> $out/${tag}_progress.log
timeout -k 10 300 python3 -u tools/latency.py > $out/${tag}_latency.jsonl 2> $out/${tag}_latency.err || exit 1
echo "c2 done" >> $out/${tag}_progress.log
