#!/bin/bash
# Round 3 (session 2): smoke, the whole GPU suite, then the default bench line on the current tree.
set -o pipefail
out=$(pwd)/gpurun_out
tag=${1:-r3h}
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stopping: rc $rc" >> $out/${tag}_progress.log; exit $rc; }; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/${tag}_smoke.log 2>&1
rc=$?; echo "smoke rc $rc" >> $out/${tag}_progress.log; ok $rc
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --maxfail=25 --timeout 240 --timeout-method thread \
    -p no:cacheprovider > $out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc $rc" >> $out/${tag}_progress.log; ok $rc
timeout -k 10 400 python3 -u bench.py > $out/${tag}_bench.log 2>&1
rc=$?; echo "bench rc $rc" >> $out/${tag}_progress.log; exit $rc
