import sys, os, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from cnn_itmo_amd import ops
dt, T = ops.DTYPES["bfloat16"]
B, hi, wi, cin, cout = 32, 272, 480, 256, 128
x = ops.new_view(B, hi, wi, cin, T)
dy = torch.empty(B * 2 * hi * 2 * wi * cout, dtype=T, device="cuda")
dk = torch.empty(4 * cout * cin, device="cuda")
kT = (torch.randn(4 * cout * cin, device="cuda") * 0.05).to(T)
dx = torch.empty(B * hi * wi * cin, dtype=T, device="cuda")
def run(label, fill, inter):
    fill()
    ts = []
    for it in range(6):
        if inter:
            ops.tconv_dgrad(dt, dy, B, hi, wi, cout, kT, cin, dx)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); ops.tconv_wgrad(dt, x, dy, cout, dk); e1.record()
        torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    print(label, "inter" if inter else "alone", " ".join("%.3f" % t for t in ts[1:]), flush=True)
def f_uniform():
    x.buf.uniform_(-1, 1); dy.uniform_(-1, 1)
def f_zero():
    x.buf.zero_(); dy.zero_()
def f_relu():
    x.buf.normal_().clamp_(min=0); dy.normal_().mul_(1e-3)
for lab, f in (("zero", f_zero), ("uniform", f_uniform), ("relu", f_relu)):
    run(lab, f, False); run(lab, f, True)
