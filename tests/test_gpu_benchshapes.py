"""Parity at the benchmarked shapes (BASELINE configs[1], [2], [4]): the real
engine runs one step of each benchmarked workload -- the same model, dtype,
batch and frame as bench.py -- with EVERY launch checked the moment it returns
against an fp64 restatement of its contract over its whole output
(tests/launch_check.py for the convolutions, tests/launch_check_elem.py for
pooling, BatchNormalization, Dropout, the head, RMSprop, weight preparation and
BN folding).  Library calls outside a checked entry point fail the test.  This
pins the persistent grids, 960-column partial strips, 2-GB buffer-descriptor
rebasing and 2^31 guards that only exist at these sizes.

  configs[2]  1920x1080 (padded 1088), batch 32, bf16 training step
  configs[1]  1920x1080 (padded 1088), batch 8, fp32 inference (BN moving stats)
  north star  1920x1080 (padded 1088), batch 32, fp32 inference: the conv2d-forward
              point of BASELINE.json's target (fp32 buffers of 6.4 G elements)
  configs[4]  3840x2160, batch 8 per GPU, bf16 training step (no padding)
"""
import contextlib
import io

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from launch_check import LaunchChecker  # noqa: E402


def _run(h, w, batch, dtype, train, expect):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.backends.cuda.matmul.allow_tf32 = False
    import cnn_itmo_amd as C
    from cnn_itmo_amd import _lib as L
    from cnn_itmo_amd import ops
    C.clear_session()
    with contextlib.redirect_stdout(io.StringIO()):
        m = C.U_net(input_size=(h, w, 3), pad=True, dtype=dtype, seed=0, verbose=False)
    if not train:  # non-trivial moving statistics
        rng = np.random.default_rng(5)
        upd = {}
        for k, v in m.named_weights().items():
            if k.endswith("/moving_mean"):
                upd[k] = rng.uniform(0.0, 0.5, v.shape).astype(np.float32)
            elif k.endswith("/moving_variance"):
                upd[k] = rng.uniform(0.5, 2.0, v.shape).astype(np.float32)
        m.set_named_weights(upd)
    eng = m._engine()
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    x = torch.randint(0, 256, (batch, h, w, 3), generator=g, device="cuda", dtype=torch.uint8).float() / 255.0
    chk = LaunchChecker(ops, L.BF16 if dtype == "bfloat16" else L.F32)
    try:
        if train:
            t = torch.randint(0, 256, (batch, h, w, 3), generator=g, device="cuda", dtype=torch.uint8).float() / 255.0
            la = eng.train_step(x, t, seed=3).cpu().numpy()
            assert np.isfinite(la).all()
        else:
            y = eng.predict(x)
            assert bool(torch.isfinite(y).all())
    finally:
        chk.restore()
        del eng, m
        torch.cuda.empty_cache()
    summ = chk.summary()
    for (lab, met), v in sorted(summ.items()):
        print(f"{lab:60s} {met:14s} {v:.3e}")
    print("checked launches per entry point:", dict(sorted(chk.calls.items())))
    assert not chk.unchecked, f"library calls outside a checked entry point: {chk.unchecked}"
    missing = set(expect) - set(chk.calls)
    assert not missing, f"entry points never launched/checked: {missing}"


# MaxPooling2D at levels 0-2 rides on its producer's epilogue (conv3x3_fwd_pool, its BN-backward
# sums from the pooled r: pool_bnsums_pooled), and its backward on the deferred skip-path dgrad
# of the concat consumer (conv3x3_dgrad_bn_pooled); pool4 reads the Dropout output: maxpool_fwd
TRAIN = ["conv_c3_fwd", "conv3x3_fwd", "conv3x3_fwd_pool", "conv3x3_fwd_cat", "conv_wgrad_cat", "tconv_fwd",
         "conv3x3_dgrad", "conv3x3_dgrad_bn", "conv3x3_dgrad_bn_pooled", "tconv_dgrad", "tconv_dgrad_bn", "conv_wgrad", "tconv_wgrad",
         "conv_c3_wgrad", "maxpool_fwd", "maxpool_bwd", "pool_bnsums_pooled", "bn_fwd_finalize", "bn_apply", "bn_bwd_reduce",
         "bn_bwd_finalize", "bn_bwd_apply", "bn_bwd_apply_g3", "bn_consumer_sums", "colsum",
         "border_sums", "head_fwd_bwd_g3", "head_finalize", "rmsprop", "prep_conv3x3", "prep_tconv", "prep_c3",
         "fold_conv3x3", "fold_tconv"]
# predict(): conv9 (model.py:261) computes the sigmoid head (model.py:276) in its epilogue (conv3x3_fwd_head)
INFER_F32 = ["prep_conv3x3", "prep_tconv", "prep_c3", "conv_c3_fwd", "conv3x3_fwd", "conv3x3_fwd_pool", "tconv_fwd",
             "maxpool_fwd", "bn_infer_coeffs", "conv3x3_fwd_head"]


def test_config2_train_1080p_b32_bf16():
    _run(1080, 1920, 32, "bfloat16", True, TRAIN)


def test_config1_infer_1080p_b8_f32():
    _run(1080, 1920, 8, "float32", False, INFER_F32)


@pytest.mark.timeout(900)
def test_northstar_infer_1080p_b32_f32():
    """BASELINE.json's north-star point: fp32 conv2d forward at 1080p batch 32."""
    _run(1080, 1920, 32, "float32", False, INFER_F32)


def test_config4_train_4k_b8_bf16():
    _run(2160, 3840, 8, "bfloat16", True, TRAIN)


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_small_frame_all_launch_kinds(dtype):
    """The same per-launch checks on a small ragged frame (quick; every kind)."""
    # fp32 training: the transposed conv's BN backward unfused (its fused kernel is bf16) and
    # one level-0 concat buffer (the split members are a bf16 line-alignment fix)
    exp = TRAIN if dtype == "bfloat16" else [k for k in TRAIN if k != "tconv_dgrad_bn" and "_cat" not in k]
    _run(72, 112, 2, dtype, True, exp)
