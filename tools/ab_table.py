"""Same-box A/B summary of bench lines: python tools/ab_table.py <label>=<bench log> ... > profiles/<name>.txt
(value, ms per step, FGMRES iterations and the phases above 0.3 ms per step, one line per run)."""
import json
import sys

for arg in sys.argv[1:]:
    label, fn = arg.split("=", 1)
    lines = [x for x in open(fn) if x.startswith("{")]
    if not lines:
        print(f"{label:10s} (no bench line: {fn})")
        continue
    d = json.loads(lines[-1])
    p = d["phase_ms_per_step"]
    ph = " ".join(f"{k}={p[k]:.2f}" for k in sorted(p, key=lambda k: -p[k]) if p[k] > 0.3)
    print(f"{label:10s} {d['value']:8.3f} Mcells*iters/s {d['ms_per_step']:7.3f} ms/step  {ph}")
