"""Run-to-run determinism of the training step at the benchmarked frame size.

Every reduction in the library is fixed-order (slab reductions, partial-sum rows, fp64 folds),
so three identical steps (same frames, same dropout seed, apply=False) must give bit-identical
loss, gradients and moving statistics.  A difference names a kernel that reads something it
did not write, or a race -- e.g. a register that a buffer store still reads being overwritten
by a later load's return, the failure an interleaved fused-dgrad epilogue showed in round 6
("Overlapping the fused dgrad's epilogue").  The 32x32 fp32 case is in
test_gpu_model.py::test_unet_two_steps_and_determinism; this one runs the bench's planner and
kernels at 1088 x 1920 (bf16: split level-0 concat, fused/deferred BN backwards, persistent
transposed convs; fp32: the fp32 halo/wgrad kernels)."""
import contextlib
import io

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dtype,n", [("bfloat16", 4), ("float32", 2)])
def test_train_step_bitwise_deterministic_1080p(dtype, n):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import cnn_itmo_amd as C
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(1080, 1920, 3), pad=True, dtype=dtype, seed=3, verbose=False)
    e = m._engine()
    rng = np.random.default_rng(6)
    x = torch.tensor(rng.random((n, 1080, 1920, 3), dtype=np.float32)).cuda()
    t = torch.tensor(rng.random((n, 1080, 1920, 3), dtype=np.float32)).cuda()
    runs = []
    b0 = e.bufs.clone()  # the moving statistics: each step updates them, so every run starts from b0
    for _ in range(3):
        e.bufs.copy_(b0)
        la = e.train_step(x, t, seed=11, apply=False)
        torch.cuda.synchronize()
        runs.append((la.cpu().numpy(), e.grads.clone(), e.bufs.clone()))
    C.clear_session()
    l0, g0, m0 = runs[0]
    assert np.isfinite(l0).all()
    for la, g, mv in runs[1:]:
        assert np.array_equal(la, l0), (la, l0)
        bad = []
        for name, (off, shp) in e.pslices.items():
            k = int(np.prod(shp))
            d = (g[off:off + k] - g0[off:off + k]).abs().max().item()
            if d != 0.0:
                bad.append((name, d))
        assert not bad, bad[:10]
        assert torch.equal(mv, m0)
    assert not torch.equal(m0, b0)  # (the step did update them)
