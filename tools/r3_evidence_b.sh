#!/bin/bash
# Round-3 evidence (part B): the default bench line (CPU baseline included), C3 streaming at draft noise 0 / 5 / 20 /
# 50 % and without drafts, C2 single-utterance latency.  usage: tools/r3_evidence_b.sh <tag>
set -o pipefail
tag=${1:-r3s2}
out=$(pwd)/gpurun_out
mkdir -p $out
prog=$out/${tag}_progress_b.log
timeout -k 10 400 python3 -u bench.py > $out/${tag}_bench.log 2>&1 || { tail -n 20 $out/${tag}_bench.log; exit 1; }
echo "bench done" >> $prog
for nz in 0 0.05 0.2 0.5; do
  timeout -k 10 240 python3 -u tools/stream_bench.py --speech-only --draft 1 --draft-noise $nz > $out/${tag}_c3_draft_noise$nz.json 2> $out/${tag}_c3_draft_noise$nz.err || exit 1
  echo "c3 noise $nz done" >> $prog
done
timeout -k 10 240 python3 -u tools/stream_bench.py --speech-only --draft 0 > $out/${tag}_c3_nodraft.json 2> $out/${tag}_c3_nodraft.err || exit 1
echo "c3 done" >> $prog
timeout -k 10 240 python3 -u tools/latency.py > $out/${tag}_latency.jsonl 2> $out/${tag}_latency.err || exit 1
echo "c2 done" >> $prog
