"""FP64 work per kernel from a rocprofv3 PMC pass of SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64, SQ_INSTS_VALU, SQ_WAVES
(tools/gpu_pmc_extra.sh): wavefront instructions per dispatch, the FP64 share of VALU instructions, and FP64 FLOP
per dispatch counted as 64 lanes x (ADD + MUL + 2 FMA + TRANS) (an upper bound: inactive lanes of partial
waves count too). Durations are the dispatches' own start/end stamps in the same pass. Peak: 78.6 TFLOP/s FP64
vector (MI355X spec).

usage: python tools/pmc_fp64.py <pmc_dir> "<bench workload key>" > profiles/<name>_fp64.json
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

PEAK = 78.6e12


def main():
    d = sys.argv[1]
    workload = sys.argv[2] if len(sys.argv) > 2 else None
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    dur = defaultdict(dict)
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                m = re.search(r"(k_\w+(?:<[^>]*>)?)", r.get("Kernel_Name", ""))
                if not m:
                    continue
                k = m.group(1)
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[k][r["Counter_Name"]] += 1
                dur[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    out = {"workload": workload, "peak_fp64_tflops": PEAK / 1e12, "kernels": {}}
    for k in acc:
        c = {q: acc[k][q] / max(1, cnt[k][q]) for q in acc[k]}
        add, mul, fma, trans = (c.get("SQ_INSTS_VALU_%s_F64" % x, 0.0) for x in ("ADD", "MUL", "FMA", "TRANS"))
        valu = c.get("SQ_INSTS_VALU", 0.0)
        flop = 64.0 * (add + mul + 2.0 * fma + trans)
        t = sum(dur[k].values()) / max(1, len(dur[k]))
        out["kernels"][k] = {
            "valu_insts": valu, "f64_insts": add + mul + fma + trans, "f64_share_of_valu": (add + mul + fma + trans) / valu if valu else 0.0,
            "fp64_flop": flop, "avg_us_under_pmc": t * 1e6, "fp64_tflops": flop / t / 1e12 if t else 0.0,
            "frac_of_fp64_peak": flop / t / PEAK if t else 0.0, "waves": c.get("SQ_WAVES", 0.0)}
    out["kernels"] = dict(sorted(out["kernels"].items(), key=lambda kv: -kv[1]["fp64_flop"]))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
