"""HBM streaming ceilings on the GPU box (copy, pure read, the BN-apply shape).
    CPU:  python tools/hbm_probe.py --build   (-> cnn_itmo_amd/lib/variants/libhbmprobe.so)
    GPU:  python tools/hbm_probe.py
Prints TB/s per (kind, vectors per lane, grid, prefetch) on 8.5 GB streams, the size of
the level-1 activations of the bench (32 x 1088 x 1920 x 64 bf16)."""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "cnn_itmo_amd", "lib", "variants", "libhbmprobe.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           os.path.join(ROOT, "tools", "hbm_probe.hip"), "-o", SO])
    print(SO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--gb", type=float, default=8.5)
    ap.add_argument("--part", action="store_true", help="partial-line reads (FETCH_SIZE calibration)")
    ap.add_argument("--copy-policies", action="store_true",
                    help="copy with nt / sc1 cache policies (the guide's 6.29 TB/s float4 copy vs this box's plain copy)")
    a = ap.parse_args()
    if a.build:
        return build()
    import torch
    lib = ctypes.CDLL(SO)
    lib.hbm_probe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                              ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_void_p]
    nvec = int(a.gb * 1e9 / 16)
    A = torch.ones(nvec * 4, dtype=torch.int32, device="cuda")
    B = torch.ones(nvec * 4, dtype=torch.int32, device="cuda")
    O = torch.empty(nvec * 4, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def run(kind, u, pf, grid, nuse=None):
        nv = nuse or nvec
        f = lambda: lib.hbm_probe(kind, u, pf, A.data_ptr(), B.data_ptr(), O.data_ptr(), nv, grid, st)
        assert f() == 0
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        t = sorted(ts)[2]
        nbytes = nv * 16 * (2 if kind == 0 or kind >= 16 else 3 if kind == 2 else 1)
        name = ['copy', 'read', 'apply'][kind] if kind < 4 else (
            ["copy ntld+ntst", "copy ntst", "copy ntld", "copy sc1st"][kind - 16] if kind >= 16 else f"part{kind * 16}")
        print(f"{name:8s} U={u} pf={pf} grid={grid:5d}  {t:7.3f} ms  {nbytes / t / 1e9:5.2f} TB/s useful "
              f"({nbytes / 1e9:.2f} GB)", flush=True)

    if a.copy_policies:
        for kind in (0, 16, 17, 18, 19):
            for u in (1, 4, 8):
                for grid in (512, 1024, 2048):
                    run(kind, u, 0, grid)
        return
    if a.part:  # useful 64 B per pixel of ps*16 bytes; nvec/3 useful vectors (fits the 8.5 GB buffer at ps 12)
        for ps in (4, 8, 12):
            run(ps, 8, 0, 2048, nuse=nvec // 3)
        return
    for kind in (0, 1, 2):
        for u in (1, 2, 4, 8):
            for grid in (1024, 2048, 4096):
                for pf in ((0, 1) if kind == 2 else (0,)):
                    run(kind, u, pf, grid)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    O.copy_(A)
    t1.record()
    torch.cuda.synchronize()
    print(f"torch copy            {t0.elapsed_time(t1):7.3f} ms  {2 * nvec * 16 / t0.elapsed_time(t1) / 1e9:5.2f} TB/s")


if __name__ == "__main__":
    sys.exit(main())
