"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs as
MI355X_MICROARCH.md §rocprofv3 PMC slots requires) -> profiles/<name>.json used by bench.py.

FETCH_SIZE and WRITE_SIZE are in KB per dispatch. On gfx950 FETCH_SIZE under-reads wide streaming
loads (cdna_hip_programming.md §7), so the read side is calibrated on a kernel with a known byte count
in the same access pattern: k_dot (FGMRES's |b|^2, one coalesced 8-B-per-lane stream of N*nVar
doubles). hbm_bytes = FETCH_SIZE*1024*factor + WRITE_SIZE*1024.

python tools/pmc_summary.py <fetch_dir> <write_dir> <workload_key> <n_rhs_doubles> > profiles/r01_pmc.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def read_counters(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: [0.0, 0])
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", "")
                m = re.search(r"::(k_\w+)", name) or re.search(r"(k_\w+)", name)
                key = m.group(1) if m else name
                acc[(key, r["Counter_Name"])][0] += float(r["Counter_Value"])
                acc[(key, r["Counter_Name"])][1] += 1
    return {k: v[0] / v[1] for k, v in acc.items()}


def main():
    fetch_dir, write_dir, wkey, n_rhs = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    fe = read_counters(fetch_dir)
    wr = read_counters(write_dir)
    known = 8.0 * n_rhs
    cal_kb = fe.get(("k_dot", "FETCH_SIZE"))
    factor = known / (cal_kb * 1024.0) if cal_kb else 1.0
    out = {"workload": wkey,
           "calibration": {"kernel": "k_dot", "known_bytes": known, "fetch_kb": cal_kb, "factor": factor},
           "kernels": {}}
    names = sorted({k for (k, c) in fe} | {k for (k, c) in wr})
    for k in names:
        f = fe.get((k, "FETCH_SIZE"))
        w = wr.get((k, "WRITE_SIZE"))
        if f is None or w is None:
            continue
        out["kernels"][k] = {"fetch_kb": f, "write_kb": w, "hbm_bytes": f * 1024.0 * factor + w * 1024.0}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
