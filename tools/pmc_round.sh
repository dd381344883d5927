#!/bin/bash
# Hardware-counter passes over one bench step (run on the GPU box from the repo root):
#   tools/pmc_round.sh <tag> [bench args...]
# One rocprofv3 --pmc pass per counter group (gfx950 slot limits: ≤ 8 SQ, ≤ 4 TCC with FETCH_SIZE = 3 and
# WRITE_SIZE = 2, ≤ 2 GRBM per pass — MI355X_MICROARCH.md), each under its own time limit; then
# tools/pmc_classes.py folds them into per-kernel-class MFMA-busy / HBM / wait figures (gpurun_out/pmc_<tag>.json).
set -o pipefail
tag=${1:-r2}; shift
args=${@:---no-cpu-baseline --no-prof --steps 1 --warmup 0}
root=$(pwd)
out=$root/gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
passes=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
  "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
  "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE"
  "WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE"
)
dbs=""
i=0
work=/tmp/pmc_$tag   # the databases stay on the box (too large to merge back); the per-class JSON is the record
for p in "${passes[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $p -d $work/$i -o run -- python3 $root/bench.py $args > $out/pmc_${tag}_$i.log 2>&1 \
    || { echo "pass $i failed"; tail -n 5 $out/pmc_${tag}_$i.log; exit 1; }
  db=$(find $work/$i -name '*.db' | head -n 1)
  dbs="$dbs $db"
done
python3 $root/tools/pmc_classes.py $out/pmc_$tag.json $dbs
