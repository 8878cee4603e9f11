"""CPU checks of the boundary and host logic: every symbol declared in
include/cnn_itmo.h is exported by libcnnitmo.so and bound by _lib; the Keras-
compatible front end reproduces the reference's layers.txt; graph compilation,
parameter layout and error behaviour work without a GPU."""
import contextlib
import io
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cnn_itmo.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(cnnitmo_\w+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from cnn_itmo_amd import _lib, build
    if not os.path.exists(_lib.LIB_PATH):
        build.build()
    return _lib.load()


def test_header_exports_and_bindings(lib):
    from cnn_itmo_amd import _lib
    syms = header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in cnn_itmo.h but not exported"
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)
    assert lib.cnnitmo_version() == 2
    assert lib.cnnitmo_consumer_rows() == _lib.CONSUMER_ROWS == 64


def test_queries_without_gpu(lib):
    # pure host-side queries (no device calls)
    # one row of partial sums per 256-pixel (v2) or 128-pixel (v1, N=32) tile
    assert lib.cnnitmo_fwd_stat_rows(1, 66846720, 64) == 66846720 // 256
    assert lib.cnnitmo_fwd_stat_rows(1, 1000, 512) == 4
    assert lib.cnnitmo_fwd_stat_rows(1, 1000, 32) in (4, 8)
    assert lib.cnnitmo_border_rows(32) == 32 * 16
    # conv3x3 (bf16, halo kernel): one row per (stream, wave); without a device the
    # launcher assumes 256 CUs (one workgroup each); 512 columns = 8 blocks of 64 ->
    # 32 streams, 768 = 12 blocks -> 21 streams, 8 waves each
    lib.cnnitmo_conv3x3_stat_rows.restype = __import__("ctypes").c_long
    assert lib.cnnitmo_conv3x3_stat_rows(1, 32, 136, 240, 768, 512) == 32 * 8
    assert lib.cnnitmo_conv3x3_stat_rows(1, 32, 136, 240, 512, 768) == 21 * 8
    assert lib.cnnitmo_conv3x3_stat_rows(1, 32, 1088, 1920, 96, 64) == 256 * 8
    assert lib.cnnitmo_wgrad_workspace_bytes(1, 32, 1088, 1920, 96, 64, 9) > 0
    assert lib.cnnitmo_bn_bwd_rows(1000, 64) >= 1


def test_invalid_shape_errors(lib):
    from cnn_itmo_amd import _lib
    # channels not a multiple of 32 -> EINVAL with a message, before any launch
    rc = lib.cnnitmo_conv3x3_fwd(1, None, 8, 0, 1, 4, 4, 8, None, None, 20, None, 20, 0, 0, None, None, None, None, None)
    assert rc == _lib.C.c_int(-1).value or rc < 0
    assert b"multiple" in lib.cnnitmo_last_error()


def test_summary_matches_layers_txt():
    import cnn_itmo_amd as C
    C.clear_session()
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        m = C.U_net()
    lines = [l.rstrip() for l in buf.getvalue().splitlines()]
    ref = os.path.join("/root/reference", "layers.txt")
    if os.path.exists(ref):
        want = [l.rstrip() for l in open(ref).read().splitlines()]
        assert lines[:len(want)] == want
    assert "Total params: 11,166,819" in lines
    assert "Trainable params: 11,159,011" in lines
    assert "Non-trainable params: 7,808" in lines
    assert m.count_params() == 11_166_819


def test_keras_errors_and_padding():
    import cnn_itmo_amd as C
    C.clear_session()
    with pytest.raises(ValueError):
        C.U_net(input_size=(1080, 1920, 3), verbose=False)  # Keras fails at the concat
    m = C.U_net(input_size=(1080, 1920, 3), pad=True, verbose=False)
    assert m.input_shape == (None, 1088, 1920, 3)
    x = C.Input((8, 8, 3))
    with pytest.raises(ValueError):
        C.concatenate([C.Conv2D(4, 3, padding="same")(x), C.MaxPooling2D(2)(x)])


def test_graph_compile_and_layout():
    import cnn_itmo_amd as C
    from cnn_itmo_amd.engine import BlockStage, ConcatStage, HeadStage, PoolStage, compile_graph, layout_params
    C.clear_session()
    m = C.U_net(input_size=(64, 64, 3), verbose=False)
    st = compile_graph(m)
    kinds = [type(s).__name__ for s in st]
    assert kinds.count("BlockStage") == 18 and kinds.count("PoolStage") == 4
    assert kinds.count("ConcatStage") == 4 and isinstance(st[-1], HeadStage)
    assert st[0].kind == "c3in" and sum(s.kind == "t2" for s in st if isinstance(s, BlockStage)) == 4
    drops = [s.drop_id for s in st if isinstance(s, BlockStage) and s.drop is not None]
    assert drops == [1, 2]
    # zero-copy concat placement: [skip, up] order (model.py:246)
    cat = [s for s in st if isinstance(s, ConcatStage)][0]
    assert [v.place[1] for v in cat.vins] == [0, 256]
    ps, bs, goff, n, nb = layout_params(st)
    total = sum(int(np.prod(s)) for _, s in ps.values())
    assert total == 11_159_011 and nb == 7_808
    # backward order == ascending offsets (head first)
    assert goff[-1][0] == 0
    nonempty = [g for g in goff[::-1] if g[1] > g[0]]
    assert all(a[1] <= b[0] for a, b in zip(nonempty, nonempty[1:]))


def test_unsupported_graph_raises():
    import cnn_itmo_amd as C
    from cnn_itmo_amd.engine import compile_graph
    C.clear_session()
    x = C.Input((16, 16, 3))
    y = C.Conv2D(8, 3, padding="same")(x)  # no ReLU: not on the path
    out = C.Conv2D(3, 1, activation="sigmoid")(y)
    with pytest.raises(NotImplementedError):
        compile_graph(C.Model(inputs=x, outputs=out))


def test_engine_refuses_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import cnn_itmo_amd as C
    from cnn_itmo_amd._lib import CnnItmoError
    C.clear_session()
    m = C.TinyNet()
    with pytest.raises(CnnItmoError):
        m.predict(np.zeros((1, 64, 64, 3)))


def test_keras_weight_layout_roundtrip():
    import cnn_itmo_amd as C
    C.clear_session()
    m = C.U_net(input_size=(32, 32, 3), verbose=False)
    ws = m.get_weights()
    assert ws[0].shape == (3, 3, 3, 32)       # Keras HWIO conv kernel
    k = [w for w in ws if w.shape == (2, 2, 512, 512)]
    assert len(k) == 1                         # Conv2DTranspose (2,2,Cout,Cin)
    named = m.named_weights()
    assert named["conv2d_1/kernel"].shape == (32, 3, 3, 3)  # engine OHWI
    m.set_weights(ws)
    for a, b in zip(ws, m.get_weights()):
        assert np.array_equal(a, b)


def test_lds_swizzles_conflict_free():
    """The halo kernels' XOR swizzles are bank-conflict-free for windows at any row."""
    import tools.check_swizzle as cs
    assert cs.check_b128()
    for R in (32, 64, 96, 128):
        assert cs.check_tr(R), R


def test_fused_head_size_fallback():
    """predict's fused conv9 + head (cnnitmo_conv3x3_fwd_head) addresses yhat with 32-bit
    offsets: batches whose fp32 yhat reaches 2 GiB take the unfused conv + head_fwd path
    (BlockStage._head_fits), e.g. fp32 4K at Model.predict's default batch of 32."""
    from types import SimpleNamespace
    from cnn_itmo_amd.engine import BlockStage
    st = SimpleNamespace(eng=SimpleNamespace(h_valid=2160), vout=SimpleNamespace(w=3840))
    assert BlockStage._head_fits(st, 21)          # 21 * 2160 * 3840 * 12 B < 2^31
    assert not BlockStage._head_fits(st, 22)
    assert not BlockStage._head_fits(st, 32)
    st = SimpleNamespace(eng=SimpleNamespace(h_valid=1080), vout=SimpleNamespace(w=1920))
    assert BlockStage._head_fits(st, 86) and not BlockStage._head_fits(st, 87)


def test_tconv_planner_choices(lib):
    """The Conv2DTranspose planners (host logic, no GPU work): up6-up8 run the persistent
    kernels in bf16 with one BN partial-sum row per (XCD, slot / column blocks, wave row), up9 the
    streamed kernels; the row count depends only on the sizes, so the engine's query matches the
    launch whatever epilogue flags it carries."""
    import ctypes
    rows = lib.cnnitmo_tconv2x2_stat_rows
    rows.restype = ctypes.c_long
    name = lib.cnnitmo_tconv2x2_kernel_name
    name.restype = ctypes.c_char_p
    cus = 256  # (no device here: the planners assume MI355X's 256 CUs)
    for (h, w, cin, cout) in [(272, 480, 256, 128), (136, 240, 512, 256), (68, 120, 512, 512)]:
        nblocks = 4 * cout // 256
        assert rows(1, 32, h, w, cin, cout) == 8 * (cus // 8 // nblocks) * 2
        assert name(1, 32, h, w, cin, cout, 0) == b"tconv_fwd2p_kernel<bf16,256x256>"
        assert name(1, 32, h, w, cin, cout, 1) == b"igemm_fwd2p_kernel<bf16,256x256>"
    assert name(1, 32, 544, 960, 128, 64, 0).startswith(b"tconv_stream_kernel")
    assert name(0, 8, 272, 480, 256, 128, 0).startswith(b"tconv_ws_kernel<f32")  # fp32: unchanged


def test_halo_global_accesses_inside_their_tensors():
    """tools/check_halo_bounds.py: every in-range raw-buffer access of the shipped halo conv
    (patch and weight pieces, epilogue stores, the fused BN backward's r loads and pool route) of
    every bench launch shape lies inside the tensor it addresses; the full-line (8 rows x 128 B)
    patch shape of the round-5 variant that faulted reads past the row (the checker has teeth)."""
    import tools.check_halo_bounds as hb
    bad, n = hb.run()
    assert n > 50 and not bad, bad[:5]
    bad_line, _ = hb.run(line=128)
    assert bad_line
