#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter CSVs per kernel-name pattern and print derived per-instruction ratios.
usage: tools/pmc_kernels.py <pattern> <counter_collection.csv>... (pattern: substring of the kernel name)"""
import csv
import sys
from collections import defaultdict


def main():
    pat = sys.argv[1]
    tot = defaultdict(float)
    disp = set()
    for path in sys.argv[2:]:
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
                if pat not in name:
                    continue
                disp.add((path, r.get("Dispatch_Id") or r.get("Correlation_Id")))
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f"{pat}: {len(disp)} dispatch-passes")
    for k in sorted(tot):
        print(f"  {k:32s} {tot[k]:.4g}")
    g = lambda k: tot.get(k, 0.0)  # noqa: E731
    if g("SQ_INSTS_MFMA"):
        m = g("SQ_INSTS_MFMA")
        print(f"  per MFMA: VALU {g('SQ_INSTS_VALU') / m:.2f}  SALU {g('SQ_INSTS_SALU') / m:.2f}  LDS "
              f"{g('SQ_INSTS_LDS') / m:.2f}  VMEM {g('SQ_INSTS_VMEM') / m:.2f}")
    if g("SQ_WAVE_CYCLES"):
        w = g("SQ_WAVE_CYCLES")
        print(f"  wave-cycle fractions: wait_any {g('SQ_WAIT_ANY') / w:.3f}  wait_inst {g('SQ_WAIT_INST_ANY') / w:.3f}  "
              f"active {g('SQ_ACTIVE_INST_ANY') / w:.3f}  active_valu {g('SQ_ACTIVE_INST_VALU') / w:.3f}")
    if g("GRBM_GUI_ACTIVE") and g("SQ_VALU_MFMA_BUSY_CYCLES"):
        print(f"  mfma busy {g('SQ_VALU_MFMA_BUSY_CYCLES') / (1024 * g('GRBM_GUI_ACTIVE') / 8):.3f}")


if __name__ == "__main__":
    main()
