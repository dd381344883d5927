# same-box kernel-trace A/B of two library builds: tools/gpu_abprof.sh <libA> <libB>
set -o pipefail
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
for L in $1 $2; do
t=$(basename $L .so)
QASR_LIB=$root/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $root/gpurun_out/abprof_$t -o run -- python3 $root/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $root/gpurun_out/abprof_$t.log 2>&1 || { tail -n 20 $root/gpurun_out/abprof_$t.log; exit 1; }
grep '"value"' $root/gpurun_out/abprof_$t.log | cut -c1-150
done
