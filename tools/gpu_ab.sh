# same-box A/B of two library builds on the default bench: tools/gpu_ab.sh <libA> <libB> [rounds]
set -o pipefail
A=$1; B=$2; n=${3:-2}
for i in $(seq $n); do
for L in $A $B; do
[ -z "$L" ] && continue
QASR_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -n 20 gpurun_out/ab.log; exit 1; }
echo "$L $(tail -n 1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["breakdown_ms"]["gemm_q8_decode"], d["roofline"]["breakdown_ms"]["gemm_q8_prefill"])')"
done; done
