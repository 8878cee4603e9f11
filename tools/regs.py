"""Per-kernel register / LDS / spill table of one csrc/*.hip file (CPU side, hipcc remarks).

    python tools/regs.py conv_halo.hip [name-filter] [-D...]

Compiles the file for gfx950 with -Rpass-analysis=kernel-resource-usage into /tmp and prints
one line per kernel: VGPRs, AGPRs, spills, LDS bytes, occupancy.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1]
    if not os.path.exists(src):
        src = os.path.join(ROOT, "cnn_itmo_amd", "csrc", src)
    filt = [a for a in sys.argv[2:] if not a.startswith("-")]
    defs = [a for a in sys.argv[2:] if a.startswith("-")]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
           f"-I{os.path.join(ROOT, 'include')}", "-Rpass-analysis=kernel-resource-usage",
           "-c", src, "-o", "/tmp/_regs.o"] + defs
    r = subprocess.run(cmd, capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(r.returncode)
    for c in rows:
        if filt and not any(f in c["name"] for f in filt):
            continue
        print(f"{c.get('VGPRs', '?'):>4} v {c.get('AGPRs', '?'):>3} a  spill v{c.get('VGPRs Spill', '?')}"
              f" s{c.get('SGPRs Spill', '?')}  lds {c.get('LDS Size [bytes/block]', '?'):>6}"
              f"  occ {c.get('Occupancy [waves/SIMD]', '?')}  {c['name']}")


if __name__ == "__main__":
    main()
