#!/bin/bash
# Round profile on the GPU box (from the repo root): kernel-trace + stats of the bench, then the two HBM-traffic
# PMC passes (FETCH_SIZE, WRITE_SIZE) on the Q8 GEMM launches of one bench step.  usage: tools/profile_round.sh <tag>
set -o pipefail
tag=${1:-r1}
root=$(pwd)
out=$root/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_$tag -o run -- python3 $root/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $out/p_$tag.log 2>&1 || { tail -n 20 $out/p_$tag.log; exit 1; }
grep '"metric"' $out/p_$tag.log | cut -c1-400
cmd="python3 bench.py --no-cpu-baseline --no-prof --steps 1 --warmup 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_gemm_q8' -d $out/pmcf_$tag -o run -- python3 $root/bench.py --no-cpu-baseline --no-prof --steps 1 --warmup 0 > $out/pf_$tag.log 2>&1 || { tail -n 20 $out/pf_$tag.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_gemm_q8' -d $out/pmcw_$tag -o run -- python3 $root/bench.py --no-cpu-baseline --no-prof --steps 1 --warmup 0 > $out/pw_$tag.log 2>&1 || { tail -n 20 $out/pw_$tag.log; exit 1; }
ls $out/pmcf_$tag $out/pmcw_$tag $out/prof_$tag
