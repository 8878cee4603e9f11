"""Join the PMC passes of tools/pmc_layers.sh per conv dispatch and print derived
metrics (fractions of SQ_WAVE_CYCLES, MFMA busy, HBM bytes, L2 hit rate).

    python tools/pmc_summary.py gpurun_out/<tag> [labels...]

The k-th conv-kernel dispatch of every pass is the same launch (each pass runs
the same program).  Optional labels name the dispatches in order (bench_layers
runs each op twice: warmup, timed).  gfx950 corrections (MI355X_MICROARCH.md):
FETCH_SIZE counts wide reads at half their bytes (doubled here); sizes in KiB.
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.pmc_traffic import label  # noqa: E402

KEYS = ("halo", "wgrad", "tconv", "igemm", "conv_c3")


def load(path):
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        if d not in per:
            per[d] = [r["Kernel_Name"], collections.defaultdict(float),
                      (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6]
        per[d][1][r["Counter_Name"]] += float(r["Counter_Value"])
    return [v for v in per.values() if any(k in v[0] for k in KEYS)]


def main():
    d = sys.argv[1]
    labels = sys.argv[2:]
    passes = [load(f) for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")))]
    n = min(len(p) for p in passes)
    for i in range(n):
        name = label(passes[0][i][0])
        c = {}
        for p in passes:
            c.update(p[i][1])
        ms = passes[0][i][2]
        lab = labels[i] if i < len(labels) else str(i)
        out = [f"{lab:14s} {name:34s} {ms:7.3f} ms"]
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            out.append("wait_any %.2f wait_inst %.2f active %.2f" % (
                c["SQ_WAIT_ANY"] / wc, c["SQ_WAIT_INST_ANY"] / wc, c["SQ_ACTIVE_INST_ANY"] / wc))
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
            out.append("mfma %.2f clk %.2fGHz" % (c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024),
                                                 c["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3) / 1e9))
        if c.get("SQ_LDS_IDX_ACTIVE"):
            out.append("ldsconf %.3f" % (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]))
        if "FETCH_SIZE" in c:
            out.append("rd %.2f GB" % (2 * c["FETCH_SIZE"] * 1024 / 1e9))
        if "WRITE_SIZE" in c:
            out.append("wr %.2f GB" % (c["WRITE_SIZE"] * 1024 / 1e9))
        if "TCC_HIT_sum" in c:
            out.append("L2hit %.2f" % (c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])))
        print("  ".join(out))


if __name__ == "__main__":
    main()
