"""Calibration only (not the product path): what the vendor GEMM (torch.mm ->
hipBLASLt) reaches on the transposed-conv GEMM shapes of the bench, bf16.
    python tools/gemm_probe.py"""
import torch

SHAPES = [  # name, M (input pixels), N (4*cout or cin), K
    ("up6 fwd", 32 * 68 * 120, 2048, 512), ("up7 fwd", 32 * 136 * 240, 1024, 512),
    ("up8 fwd", 32 * 272 * 480, 512, 256), ("up7 dgrad", 32 * 136 * 240, 512, 1024),
    ("up6 dgrad", 32 * 68 * 120, 512, 2048),
]
for name, m, n, k in SHAPES:
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(k, n, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        c = a @ b
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = sorted(ts)[5]
    print(f"{name:10s} M={m} N={n} K={k}: {ms:.3f} ms  {2 * m * n * k / ms / 1e9:.1f} TFLOP/s")
    del a, b, c
