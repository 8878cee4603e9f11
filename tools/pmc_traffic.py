"""HBM bytes per launch per kernel from the rocprofv3 --pmc passes of
tools/pmc_traffic.sh (two per workload shape) -> profiles/pmc_traffic.json (read by
bench.py's roofline, which uses it only for the same library build and shape).

    python tools/pmc_traffic.py gpurun_out profiles/pmc_traffic.json

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 128-B
requests at 64 B, i.e. half the bytes of wide coalesced reads -> doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.  Both are reported in KiB.
Keys are the kernel labels bench.py uses (cnnitmo_*_kernel_name)."""
import collections
import csv
import json
import re
import subprocess
import sys

CXXFILT = "c++filt"


def demangle(names):
    try:
        out = subprocess.run([CXXFILT], input="\n".join(names), capture_output=True, text=True, check=True).stdout
        return out.splitlines()
    except Exception:
        return names


def unmangle(n):
    """Itanium-mangled template kernels with a bf16 (DF16b) / float first argument,
    e.g. _Z17igemm_fwd2_kernelIDF16bLi256ELi128ELi4ELi2ELi3EEv7FwdArgs (c++filt
    here does not know DF16b)."""
    m = re.match(r"_Z(?:N12_GLOBAL__N_1)?\d+([A-Za-z_0-9]+?)I((?:L[ib]\d+E|DF16b|f)+)E", n)
    if not m:
        return n
    args = []
    for tok in re.findall(r"L[ib]\d+E|DF16b|f", m.group(2)):
        if tok == "DF16b":
            args.append("__bf16")
        elif tok == "f":
            args.append("float")
        elif tok[1] == "b":
            args.append("true" if tok[2:-1] == "1" else "false")
        else:
            args.append(tok[2:-1])
    return "%s<%s>" % (m.group(1), ",".join(args))


def label(name):
    n = unmangle(name.replace(" ", "")).replace("(anonymousnamespace)::", "")
    m = re.search(r"halo_conv_kernel<(?:(__bf16|float),)?(\d+),(\d+)(?:,(true|false))?(?:,(true|false))?(?:,(\d+))?(?:,(?:true|false))?>", n)
    if m:
        pool = "" if m.group(5) != "true" else (",route" if m.group(3) == "2" else ",pool")
        return "halo_conv_kernel<%s%s,%s%s%s>" % ("f32," if m.group(1) == "float" else "", m.group(2), m.group(3),
                                                 ",wres" if m.group(4) == "true" else "", pool)
    m = re.search(r"halo_gemm_kernel<(\d+),(\d+),(\d+),(\d+),\d+(?:,(\d+))?>", n)
    if m:
        return "halo_gemm_kernel<%s,%s,%s,%s%s>" % (m.groups()[:4] + (",bnb" if m.group(5) not in (None, "0") else "",))
    m = re.search(r"tconv_stream_kernel<(\d+),(\d+),\d+,(true|false)>", n)
    if m:
        return "tconv_stream_kernel<%s,%s%s>" % (m.group(1), m.group(2), ",bnb" if m.group(3) == "true" else "")
    m = re.search(r"tconv_ws_kernel<(\d+),(\d+)(?:,\d+)*(?:,(__bf16|float))?>", n)
    if m:
        return "tconv_ws_kernel<%s%s,%s>" % ("f32," if m.group(3) == "float" else "", m.group(1), m.group(2))
    m = re.search(r"wgrad_halo_kernel<(\d+),(\d+),(\d+),", n)
    if m:
        return "wgrad_halo_kernel<%s,%s,%s>" % m.groups()
    m = re.search(r"igemm_fwd2p_kernel<(\d+),(\d+),", n)
    if m:
        return "igemm_fwd2p_kernel<bf16,%sx%s>" % m.groups()
    m = re.search(r"igemm_fwd2_kernel<__bf16,(\d+),(\d+),", n) or re.search(r"igemm_fwd2_kernel<[^,]*,(\d+),(\d+),", n)
    if m:
        t = "bf16" if "bf16" in n else "f32"
        return "igemm_fwd2_kernel<%s,%sx%s>" % (t, m.group(1), m.group(2))
    m = re.search(r"igemm_fwd_kernel<[^,]*,(\d+),(\d+),", n)
    if m:
        t = "bf16" if "bf16" in n else "f32"
        return "igemm_fwd_kernel<%s,%sx%s>" % (t, m.group(1), m.group(2))
    m = re.search(r"igemm_wgrad2_kernel<(\d+),(\d+),\d+,\d+,(\d+),", n)
    if m:
        return "igemm_wgrad2_kernel<%s,%s,tpb%s>" % m.groups()
    m = re.search(r"igemm_wgrad_kernel<[^,]*,(\d+),(\d+),", n)
    if m:
        t = "bf16" if "bf16" in n else "f32"
        return "igemm_wgrad_kernel<%s,%s,%s>" % (t, m.group(1), m.group(2))
    m = re.match(r"(?:void)?([A-Za-z_0-9:]+?)(?:<|\()", n)
    return (m.group(1).split("::")[-1] if m else n)[:80]


def load(path):
    rows = list(csv.DictReader(open(path)))
    names = sorted({r["Kernel_Name"] for r in rows})
    dm = dict(zip(names, demangle(names)))
    per = collections.defaultdict(float)
    kern = {}
    for r in rows:
        per[r["Dispatch_Id"]] += float(r["Counter_Value"])
        kern[r["Dispatch_Id"]] = label(dm[r["Kernel_Name"]])
    return per, kern


def table(fetch_csv, write_csv):
    f, kf = load(fetch_csv)
    w, kw = load(write_csv)
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for d, v in f.items():
        agg[kf[d]][0] += 1
        agg[kf[d]][1] += 2.0 * v * 1024.0  # gfx950: FETCH_SIZE reads half of wide loads
    for d, v in w.items():
        agg[kw[d]][2] += v * 1024.0
    res = {}
    for k, (n, rd, wr) in sorted(agg.items(), key=lambda kv: -(kv[1][1] + kv[1][2])):
        res[k] = {"launches": n, "read_bytes_per_launch": rd / n, "write_bytes_per_launch": wr / max(n, 1),
                  "bytes_per_launch": (rd + wr) / n}
    return res


def main(outdir, out_json):
    """outdir: gpurun_out/ of a tools/pmc_traffic.sh run (pmc_<SHAPE_TAG>_<COUNTER>/ + lib_sha.txt)."""
    import glob
    import os
    shapes = {}
    for tag_file in sorted(glob.glob(os.path.join(outdir, "pmc_*_FETCH_SIZE.shape"))):
        tag = os.path.basename(tag_file)[len("pmc_"):-len("_FETCH_SIZE.shape")]
        shape = open(tag_file).read().strip()
        fc = glob.glob(os.path.join(outdir, f"pmc_{tag}_FETCH_SIZE", "**", "*counter_collection.csv"), recursive=True)
        wc = glob.glob(os.path.join(outdir, f"pmc_{tag}_WRITE_SIZE", "**", "*counter_collection.csv"), recursive=True)
        shapes[shape] = table(fc[0], wc[0])
        print(shape)
        for k, v in list(shapes[shape].items())[:12]:
            print(f"  {k:45s} {v['launches']:4d} {v['bytes_per_launch'] / 1e9:8.3f} GB/launch")
    meta = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), one bench.py step per shape "
                      "(tools/pmc_traffic.sh)",
            "correction": "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B); KiB -> bytes",
            "lib_sha256": open(os.path.join(outdir, "pmc_lib_sha.txt")).read().strip(),
            "shapes": sorted(shapes)}
    json.dump({"_meta": meta, "per_shape": shapes}, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:3])
