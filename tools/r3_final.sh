#!/bin/bash
# Round-3 evidence on the GPU box (repo root): bench kernel trace + stats, per-class PMC passes, the default bench line
# (with the CPU baseline), C3 streaming at draft noise 0 / 5 / 20 / 50 % and without drafts, C2 latency.
# usage: tools/r3_final.sh <tag>
set -o pipefail
tag=${1:-r3f}
root=$(pwd)
out=$root/gpurun_out
mkdir -p $out
prog=$out/${tag}_progress.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/kt_$tag -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $out/${tag}_prof_bench.log 2>&1 || { tail -n 20 $out/${tag}_prof_bench.log; exit 1; }
cp $(find /tmp/kt_$tag -name '*kernel_stats.csv' | head -n 1) $out/${tag}_kernel_stats.csv
echo "kernel trace done" >> $prog
cd $root
bash tools/pmc_round.sh $tag > $out/${tag}_pmc.log 2>&1 || { tail -n 20 $out/${tag}_pmc.log; exit 1; }
echo "pmc done" >> $prog
timeout -k 10 400 python3 -u bench.py > $out/${tag}_bench.log 2>&1 || { tail -n 20 $out/${tag}_bench.log; exit 1; }
echo "bench done" >> $prog
for nz in 0 0.05 0.2 0.5; do
  timeout -k 10 300 python3 -u tools/stream_bench.py --speech-only --draft 1 --draft-noise $nz > $out/${tag}_c3_draft_noise$nz.json 2> $out/${tag}_c3_draft_noise$nz.err || exit 1
  echo "c3 noise $nz done" >> $prog
done
timeout -k 10 300 python3 -u tools/stream_bench.py --speech-only --draft 0 > $out/${tag}_c3_nodraft.json 2> $out/${tag}_c3_nodraft.err || exit 1
echo "c3 done" >> $prog
timeout -k 10 300 python3 -u tools/latency.py > $out/${tag}_latency.jsonl 2> $out/${tag}_latency.err || exit 1
echo "c2 done" >> $prog
