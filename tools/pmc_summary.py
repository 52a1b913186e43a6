"""Per-kernel HBM traffic from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs as
MI355X_MICROARCH.md §rocprofv3 PMC slots requires) -> profiles/<name>.json used by bench.py.

FETCH_SIZE and WRITE_SIZE are in KB per dispatch. On gfx950 FETCH_SIZE reports exactly 1/2 of the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md §HBM), so the guide's correction is applied:
    hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.
For comparison the file also carries a self-calibrated figure (hbm_bytes_calibrated): FETCH scaled so that
k_fg_spmv<nVar> reads exactly its BSR matrix stream (nnzb * nVar^2 * 8 bytes); that calibration is circular for that
kernel and is not what bench.py reports. Kernels are keyed by name with template arguments (k_fg_spmv<11>, ...),
non-template kernels by name. The workload key must be bench.py's (`<workload> <dims> ns<Ns> parts<P>`).

python tools/pmc_summary.py <fetch_dir> <write_dir> "<workload key>" <nVar> <nnzb> > profiles/r03_pmc_<wl>.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def read_counters(d, peak=False):
    """Mean (or, peak=True, max) counter value per dispatch of each kernel."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: [0.0, 0])
    mx = defaultdict(float)
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", "")
                m = re.search(r"(k_\w+(?:<[^>]*>)?)", name)
                key = m.group(1) if m else name
                acc[(key, r["Counter_Name"])][0] += float(r["Counter_Value"])
                acc[(key, r["Counter_Name"])][1] += 1
                mx[(key, r["Counter_Name"])] = max(mx[(key, r["Counter_Name"])], float(r["Counter_Value"]))
    return dict(mx) if peak else {k: v[0] / v[1] for k, v in acc.items()}


def main():
    fetch_dir, write_dir, wkey, nv, nnzb = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    fe = read_counters(fetch_dir)
    wr = read_counters(write_dir)
    known = 8.0 * nnzb * nv * nv
    # the FGMRES SpMV (k_fg_spmv before round 3, k_fg_spmv_full since, k_fg_spmv_stage since round 5), else the plain
    # SpMV
    cal = [k for k in (f"k_fg_spmv<{nv}>", f"k_fg_spmv_stage<{nv}>", f"k_fg_spmv_full<{nv}>", f"k_spmv<{nv}>")
           if (k, "FETCH_SIZE") in fe][:1]
    cal_kb = fe.get((cal[0], "FETCH_SIZE")) if cal else None
    factor = known / (cal_kb * 1024.0) if cal_kb else 1.0
    out = {"workload": wkey, "fetch_factor": 2.0,
           "calibration": {"kernel": cal[0] if cal else None, "known_bytes": known, "fetch_kb": cal_kb, "factor": factor},
           "kernels": {}}
    names = sorted({k for (k, c) in fe} | {k for (k, c) in wr})
    for k in names:
        f = fe.get((k, "FETCH_SIZE"))
        w = wr.get((k, "WRITE_SIZE"))
        if f is None or w is None:
            continue
        out["kernels"][k] = {"fetch_kb": f, "write_kb": w, "hbm_bytes": 2.0 * f * 1024.0 + w * 1024.0,
                             "hbm_bytes_calibrated": f * 1024.0 * factor + w * 1024.0}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
