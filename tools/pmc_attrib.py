"""Issue/wait attribution of a kernel's wave cycles from tools/pmc_attrib.sh's four passes.

    python tools/pmc_attrib.py gpurun_out/attrib_<tag> [kernel-label filter] [--json out.json] [--steps N]

--steps N: the profiled program ran N identical steps (tools/recipe.sh benchattrib): the launches
of one label are told apart by their position in the step (label#k = the k-th launch of that
kernel in a step), so that one kernel's layers get a row each.

Per kernel label (tools/pmc_traffic.label), summed over its dispatches in each pass:
  * SQ_WAVE_CYCLES = SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY (disjoint,
    MI355X_MICROARCH.md rocprofv3 section; all three in quad-cycles): parked at s_waitcnt /
    s_barrier, stalled at issue (MFMA dependency / pipe busy; SQ_WAIT_INST_LDS = the LDS
    issue part of it), and issuing;
  * SQ_ACTIVE_INST_{VALU,LDS,SCA,VMEM,MISC,FLAT}: quad-cycles each instruction class is
    being issued (classes overlap the MFMA pipe);
  * SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over SIMDs) against GRBM_GUI_ACTIVE / 8 x 1024
    SIMDs: the MFMA-busy fraction; instruction counts per wave from pass 3.
Passes are separate runs of the same launches: ratios are taken within a pass, and
across passes only per dispatch-normalised counts are combined.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.pmc_traffic import label  # noqa: E402

SIMDS, XCDS = 256 * 4, 8


def load(d, steps=0):
    """label -> counter -> (sum over dispatches, dispatches); wall seconds per label."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names, wall = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = (f, int(r["Dispatch_Id"]))
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            names[key] = label(r["Kernel_Name"])
            if "End_Timestamp" in r:
                wall[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    if steps:  # label#k: the k-th launch of the label within a step (per pass file)
        byf = collections.defaultdict(list)
        for key in names:
            byf[(key[0], names[key])].append(key)
        for (_, lab), keys in byf.items():
            keys.sort(key=lambda k: k[1])
            per_step = max(1, len(keys) // steps)
            for i, key in enumerate(keys):
                names[key] = f"{lab}#{i % per_step}"
    agg = collections.defaultdict(lambda: collections.defaultdict(lambda: [0.0, 0]))
    tw = collections.defaultdict(lambda: [0.0, 0])
    for key, c in per.items():
        for k, v in c.items():
            a = agg[names[key]][k]
            a[0] += v
            a[1] += 1
        if "SQ_WAVE_CYCLES" in c:
            tw[names[key]][0] += wall.get(key, 0.0)
            tw[names[key]][1] += 1
    return agg, tw


def main():
    d = sys.argv[1]
    skip = {i + 1 for i, a in enumerate(sys.argv) if a in ("--steps", "--json")}
    filt = [a for i, a in enumerate(sys.argv[2:], 2) if not a.startswith("--") and i not in skip]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 0
    agg, tw = load(d, steps)
    out = {}
    for lab, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", [0])[0]):
        if filt and not any(f in lab for f in filt):
            continue
        if "SQ_WAVE_CYCLES" not in c:
            continue

        def m(k):  # mean per dispatch
            v = c.get(k)
            return v[0] / v[1] if v and v[1] else float("nan")
        wc = m("SQ_WAVE_CYCLES")
        row = {"dispatches": int(c["SQ_WAVE_CYCLES"][1]), "wave_cycles_per_dispatch": wc}
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            row[k + "/WAVE"] = m(k) / wc
        mb = m("SQ_VALU_MFMA_BUSY_CYCLES")
        if not mb or mb != mb:
            continue  # (no matrix work: not a conv kernel)
        busy = mb / (m("GRBM_GUI_ACTIVE") / XCDS * SIMDS)
        row["mfma_busy_frac"] = busy
        row["coexec/mfma_busy"] = m("SQ_VALU_MFMA_COEXEC_CYCLES") / mb
        # pass 2 is another run of the same launches: normalise by its own GRBM cycles
        g2 = None
        for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM",
                  "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_FLAT", "SQ_INST_CYCLES_SALU", "SQ_INST_CYCLES_VMEM_RD",
                  "SQ_INST_CYCLES_VMEM_WR", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_DATA_FIFO_FULL",
                  "SQ_LDS_CMD_FIFO_FULL", "SQ_INST_LEVEL_LDS", "SQ_INST_LEVEL_VMEM", "SQ_LDS_UNALIGNED_STALL"):
            row[k + "/dispatch"] = m(k)
        waves = m("SQ_WAVES")
        for k in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM",
                  "SQ_INSTS_BRANCH"):
            row[k + "/wave"] = m(k) / waves if waves == waves and waves else float("nan")
        t, n = tw.get(lab, [0.0, 0])
        row["avg_ms_pass1"] = t / n * 1e3 if n else None
        row["eff_clock_ghz"] = m("GRBM_GUI_ACTIVE") / XCDS / (t / n) / 1e9 if n and t else None
        out[lab] = row
        print(f"== {lab}  ({row['dispatches']} dispatches, {row['avg_ms_pass1']:.3f} ms, "
              f"{row['eff_clock_ghz'] or 0:.2f} GHz)")
        print(f"   mfma busy {busy:6.1%}   WAIT_ANY {row['SQ_WAIT_ANY/WAVE']:6.1%}   WAIT_INST_ANY "
              f"{row['SQ_WAIT_INST_ANY/WAVE']:6.1%} (LDS {row['SQ_WAIT_INST_LDS/WAVE']:6.1%})   ACTIVE_INST_ANY "
              f"{row['SQ_ACTIVE_INST_ANY/WAVE']:6.1%}   coexec/mfma {row['coexec/mfma_busy']:.3f}")
        print("   per wave: " + "  ".join(f"{k[9:]}={row[k + '/wave']:.0f}" for k in
                                         ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU",
                                          "SQ_INSTS_VMEM", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH")))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
