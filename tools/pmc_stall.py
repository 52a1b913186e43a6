"""Wave-state breakdown per kernel from a rocprofv3 PMC pass (tools/gpu_pmc_stall.sh): the share of wave cycles
parked on s_waitcnt / barriers (SQ_WAIT_ANY), stalled at issue (SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY);
VMEM-read and LDS instructions per wave.

usage: python tools/pmc_stall.py <pmc_dir> > profiles/<name>_stall.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(lambda: defaultdict(int))
    for fn in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                m = re.search(r"(k_\w+(?:<[^>]*>)?)", r.get("Kernel_Name", ""))
                if m:
                    acc[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
                    n[m.group(1)][r["Counter_Name"]] += 1
    out = {}
    for k, c in acc.items():
        v = {q: c[q] / max(1, n[k][q]) for q in c}
        cyc = v.get("SQ_WAVE_CYCLES", 0.0)
        waves = v.get("SQ_WAVES", 0.0)
        if cyc <= 0 or waves <= 0:
            continue
        out[k] = {"wave_cycles": cyc, "waves": waves,
                  "wait_any": v.get("SQ_WAIT_ANY", 0.0) / cyc, "wait_inst": v.get("SQ_WAIT_INST_ANY", 0.0) / cyc,
                  "active_inst": v.get("SQ_ACTIVE_INST_ANY", 0.0) / cyc,
                  "vmem_rd_per_wave": v.get("SQ_INSTS_VMEM_RD", 0.0) / waves,
                  "lds_per_wave": v.get("SQ_INSTS_LDS", 0.0) / waves}
    print(json.dumps(dict(sorted(out.items(), key=lambda kv: -kv[1]["wave_cycles"])), indent=1))


if __name__ == "__main__":
    main()
