#!/bin/bash
# Round-3 evidence (part A, GPU box, repo root): the whole GPU suite, the bench's kernel trace + stats, the per-class
# PMC passes (tools/pmc_round.sh), then the default bench line (which picks up the per-class file of this very build).
# usage: tools/r3_evidence_a.sh <tag>
set -o pipefail
tag=${1:-r3s2}
root=$(pwd)
out=$root/gpurun_out
mkdir -p $out
prog=$out/${tag}_progress.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --maxfail=25 --timeout 240 --timeout-method thread \
    -p no:cacheprovider > $out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $prog; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/${tag}_smoke.log 2>&1 || { echo "smoke failed" >> $prog; exit 1; }
echo "smoke done" >> $prog
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt_$tag -o run --output-format csv -- python3 $root/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $out/${tag}_prof_bench.log 2>&1 || { tail -n 20 $out/${tag}_prof_bench.log; exit 1; }
cp $(find /tmp/kt_$tag -name '*kernel_stats.csv' | head -n 1) $out/${tag}_kernel_stats.csv
echo "kernel trace done" >> $prog
cd $root
bash tools/pmc_round.sh $tag > $out/${tag}_pmc.log 2>&1 || { tail -n 20 $out/${tag}_pmc.log; exit 1; }
echo "pmc done" >> $prog
