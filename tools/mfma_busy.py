"""MFMA-busy fraction per kernel from a rocprofv3 --pmc pass with
SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (tools/r02_probe.sh).

  python tools/mfma_busy.py <run_counter_collection.csv> [--json out.json]

SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe busy cycles summed over every SIMD
(MI355X_MICROARCH.md: = 32 x N_mfma for 32x32x16 bf16); GRBM_GUI_ACTIVE is the
dispatch's GPU-active cycles summed over the 8 XCDs.  busy fraction =
MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs).  Rows of one dispatch are summed
per counter first (rocprofv3 emits one row per counter instance).  The effective clock
is GRBM_GUI_ACTIVE / 8 / the dispatch's wall time (MI355X_MICROARCH.md, DVFS
give-back), and busy x clock (GHz) is the kernel's MFMA rate in units of one SIMD's
16x16x32 issue at 1 GHz: the product the DVFS argument of DESIGN.md rests on."""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.pmc_traffic import label  # noqa: E402

SIMDS = 256 * 4
XCDS = 8


def main():
    path = sys.argv[1]
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # dispatch -> counter -> value
    names = {}
    wall = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
        if "End_Timestamp" in r:
            wall[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for d, c in per.items():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in c or "GRBM_GUI_ACTIVE" not in c:
            continue
        a = agg[label(names[d])]
        a[0] += 1
        a[1] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        a[2] += c["GRBM_GUI_ACTIVE"]
        a[3] += wall.get(d, 0.0)
    tot_b = sum(v[1] for v in agg.values())
    tot_g = sum(v[2] for v in agg.values())
    out = {}
    for k, (n, b, g, t) in sorted(agg.items(), key=lambda kv: -kv[1][2]):
        if b == 0:
            continue
        frac = b / (g / XCDS * SIMDS)
        ghz = g / XCDS / t / 1e9 if t > 0 else None
        out[k] = {"dispatches": n, "mfma_busy_frac": round(frac, 4), "gpu_active_cycles_per_xcd": g / XCDS / n,
                  "avg_ms": round(t / n * 1e3, 4), "eff_clock_ghz": round(ghz, 3) if ghz else None,
                  "busy_x_clock": round(frac * ghz, 3) if ghz else None}
        print(f"{k:60s} n={n:4d}  mfma_busy {frac:6.1%}  clock {ghz or 0:5.2f} GHz  busy*clock {frac * (ghz or 0):5.3f}"
              f"  share of active {g / tot_g:6.1%}")
    whole = tot_b / (tot_g / XCDS * SIMDS)
    print(f"{'ALL dispatches':60s}         mfma_busy {whole:6.1%}")
    out["ALL"] = {"mfma_busy_frac": round(whole, 4)}
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
