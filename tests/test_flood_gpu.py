"""HIP min-sum / BP decoder vs the oracle and the reference's golden fixtures (GPU).

Bar: min-sum decisions bit-exact (integer-like work: the reference's float32 operation sequence
is reproduced); BP decisions within a stated tolerance (the reference's torch-CPU tanh/atanh are
SLEEF approximations, not correctly rounded -- see DESIGN.md "Parity")."""
import os

import numpy as np
import pytest
import torch

from conftest import code_path, golden

from ldpc_neural_decoder import _native as N
from ldpc_neural_decoder.models import BeliefPropagationDecoder, MinSumScaledDecoder
from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu
SNRS = [-1.0, 0.0, 2.0, 4.0, 6.0]


def H_of(z):
    return expand_base_matrix(load_base_matrix(code_path(z)), z)


@pytest.fixture(scope="module")
def H4():
    return H_of(4)


@pytest.fixture(scope="module")
def H32():
    return H_of(32)


def test_lifting_detected(cuda, H4, H32):
    for H, z, fixed in ((H4, 4, 1), (H32, 32, 2)):
        dec = MinSumScaledDecoder(H, max_iterations=5)
        g = dec.graph(cuda)
        assert g.Z == z and g.E == 788 * z // 4 and g.max_dc == 10 and g.max_dv == 23
        assert g.set_variant(0) == fixed  # the reference's codes get the compile-time schedule


@pytest.mark.parametrize("algo", ["minsum", "bp"])
@pytest.mark.parametrize("es", [False, True, "frame"])
def test_fixed_and_table_driven_agree(cuda, H32, algo, es):
    """The compile-time-schedule kernel and the table-driven kernel are bit-identical."""
    llr = torch.from_numpy(golden("trad_z32_low.npz")["llrs"].reshape(-1, 1664)).to(cuda)
    mk = (lambda: MinSumScaledDecoder(H32, 7, 0.75, early_stopping=es)) if algo == "minsum" \
        else (lambda: BeliefPropagationDecoder(H32, 7, early_stopping=es))
    d_fix, d_tab = mk(), mk()
    assert d_tab.graph(cuda).set_variant(1) == 0
    b1, i1, f1 = d_fix.decode(llr, return_frame_iters=True)
    b2, i2, f2 = d_tab.decode(llr, return_frame_iters=True)
    assert torch.equal(b1, b2) and i1 == i2 and torch.equal(f1, f2)


@pytest.mark.parametrize("alpha,key", [(0.75, "ms_a0.75"), (0.8, "ms_a0.8")])
@pytest.mark.parametrize("es", [False, True])
def test_minsum_z4_golden_bitexact(cuda, H4, alpha, key, es):
    t, ch = golden("trad_z4.npz"), golden("channel_z4.npz")
    dec = MinSumScaledDecoder(H4, max_iterations=5, scaling_factor=alpha, early_stopping=es)
    for k in range(len(SNRS)):
        bits, it = dec.decode(torch.from_numpy(ch["llrs"][k]).to(cuda))
        assert bits.dtype == torch.float32 and bits.shape == (64, 208)
        assert np.array_equal(bits.cpu().numpy().astype(np.uint8), t[f"{key}_es{int(es)}_bits"][k])
        assert it == t[f"{key}_es{int(es)}_iters"][k]


@pytest.mark.parametrize("es", [False, True])
def test_minsum_z32_golden_bitexact(cuda, H32, es):
    dec = MinSumScaledDecoder(H32, max_iterations=10, scaling_factor=0.75, early_stopping=es)
    for name in ("trad_z32.npz", "trad_z32_low.npz"):
        t = golden(name)
        llrs = golden("channel_z32.npz")["llrs"] if name == "trad_z32.npz" else t["llrs"]
        for k in range(llrs.shape[0]):
            bits, it = dec.decode(torch.from_numpy(llrs[k]).to(cuda))
            assert np.array_equal(bits.cpu().numpy().astype(np.uint8),
                                  t[f"ms_a0.75_es{int(es)}_bits"][k]), (name, k)
            assert it == t[f"ms_a0.75_es{int(es)}_iters"][k]


@pytest.mark.parametrize("es", [False, True])
def test_bp_z4_golden(cuda, H4, es):
    """Decisions within tolerance: at most 0.1 % of bits may differ from the reference
    (tanh/atanh rounding); iteration counts must agree."""
    t, ch = golden("trad_z4.npz"), golden("channel_z4.npz")
    dec = BeliefPropagationDecoder(H4, max_iterations=5, early_stopping=es)
    total = diff = 0
    for k in range(len(SNRS)):
        bits, it = dec.decode(torch.from_numpy(ch["llrs"][k]).to(cuda))
        ref = t[f"bp_es{int(es)}_bits"][k]
        diff += int((bits.cpu().numpy().astype(np.uint8) != ref).sum())
        total += ref.size
        assert it == t[f"bp_es{int(es)}_iters"][k]
    assert diff <= 1e-3 * total, diff


@pytest.mark.parametrize("es", [False, True])
def test_bp_z32_golden(cuda, H32, es):
    """BP at Z=32 against the reference's own decisions (bp_z32.npz: B=8, 10 iterations, -6/-4/-2/0
    dB, where frames keep errors): iteration counts equal, at most 0.1 % of bits differ (the BP bar,
    as at Z=4)."""
    t = golden("bp_z32.npz")
    dec = BeliefPropagationDecoder(H32, max_iterations=10, early_stopping=es)
    total = diff = 0
    for k in range(len(t["snrs"])):
        bits, it = dec.decode(torch.from_numpy(t["llrs"][k]).to(cuda))
        ref = t[f"bp_es{int(es)}_bits"][k]
        diff += int((bits.cpu().numpy().astype(np.uint8) != ref).sum())
        total += ref.size
        assert it == t[f"bp_es{int(es)}_iters"][k]
    print(f"bp z32 es={es}: {diff} of {total} bits differ from the reference")
    assert diff <= 1e-3 * total, diff


@pytest.mark.parametrize("z,iters", [(4, 5), (32, 10)])
@pytest.mark.parametrize("algo", ["minsum", "bp"])
def test_vs_oracle_random_batches(cuda, oracle_mod, z, iters, algo):
    """Odd batch sizes (tail workgroups), low and high SNR; min-sum exact, BP exact vs the
    oracle (both evaluate tanh/atanh in double and round)."""
    H = H_of(z)
    g = oracle_mod.Graph(H.numpy())
    rng = np.random.default_rng(z * 7 + iters)
    for B, snr in ((1, -3.0), (37, 0.0), (129 if z == 4 else 19, 2.0)):
        llr = (rng.normal(1.0, 1.0, size=(B, H.shape[1])) * (2 * 10 ** (snr / 10))).astype(np.float32)
        if algo == "minsum":
            dec = MinSumScaledDecoder(H, max_iterations=iters, early_stopping=False)
        else:
            dec = BeliefPropagationDecoder(H, max_iterations=iters, early_stopping=False)
        bits, _ = dec.decode(torch.from_numpy(llr).to(cuda))
        ref, _, _, _ = oracle_mod.flood_decode(g, llr, algo, iters, 0.75, 0)
        got = bits.cpu().numpy().astype(np.uint8)
        if algo == "minsum":
            assert np.array_equal(got, ref), (B, snr)
        else:
            assert (got != ref).mean() <= 1e-4, (B, snr)


def test_per_frame_early_stop(cuda, oracle_mod, H4):
    llr = golden("channel_z4.npz")["llrs"][3]
    g = oracle_mod.Graph(H4.numpy())
    dec = MinSumScaledDecoder(H4, max_iterations=8, early_stopping="frame")
    bits, it, fi = dec.decode(torch.from_numpy(llr).to(cuda), return_frame_iters=True)
    rb, _, _, ri = oracle_mod.flood_decode(g, llr, "minsum", 8, 0.75, 2)
    assert np.array_equal(bits.cpu().numpy().astype(np.uint8), rb)
    assert np.array_equal(fi.cpu().numpy(), ri)
    assert it == ri.max()


def test_counters_and_u8_output(cuda, H32):
    llr = torch.from_numpy(golden("trad_z32_low.npz")["llrs"][0]).to(cuda)
    dec = MinSumScaledDecoder(H32, max_iterations=10, early_stopping=False)
    cnt = torch.zeros(4, dtype=torch.int64, device=cuda)
    b8, _ = dec.decode(llr, out_dtype=torch.uint8, counters=cnt)
    bf, _ = dec.decode(llr)
    assert b8.dtype == torch.uint8 and torch.equal(b8.float(), bf)
    be = int(bf.sum().item())
    fe = int((bf.sum(1) > 0).sum().item())
    assert cnt.tolist() == [be, fe, llr.shape[0], 10 * llr.shape[0]]


def test_generic_code_z1(cuda, oracle_mod):
    """A non-QC parity-check matrix (lifting Z = 1): Hamming(7,4) and a random sparse code."""
    Hh = torch.tensor([[1, 1, 0, 1, 1, 0, 0], [1, 0, 1, 1, 0, 1, 0], [0, 1, 1, 1, 0, 0, 1]],
                      dtype=torch.float32)
    rng = np.random.default_rng(5)
    Hr = np.zeros((30, 60), dtype=np.float32)
    for j in range(60):
        Hr[rng.choice(30, size=3, replace=False), j] = 1
    for H in (Hh, torch.from_numpy(Hr)):
        dec = MinSumScaledDecoder(H, max_iterations=6, early_stopping=False)
        assert dec.graph(cuda).Z == 1
        llr = rng.normal(1.5, 2.0, size=(70, H.shape[1])).astype(np.float32)
        bits, _ = dec.decode(torch.from_numpy(llr).to(cuda))
        ref, _, _, _ = oracle_mod.flood_decode(oracle_mod.Graph(H.numpy()), llr, "minsum", 6, 0.75, 0)
        assert np.array_equal(bits.cpu().numpy().astype(np.uint8), ref)


def test_special_values(cuda, oracle_mod, H4):
    """Zeros (torch.sign(0) = 0), infinities and NaN follow the reference's float semantics."""
    rng = np.random.default_rng(3)
    llr = rng.normal(0.5, 1.0, size=(16, 208)).astype(np.float32)
    llr[0, :40] = 0.0
    llr[1, 5] = np.inf
    llr[2, 9] = -np.inf
    llr[3, 11] = np.nan
    g = oracle_mod.Graph(H4.numpy())
    dec = MinSumScaledDecoder(H4, max_iterations=4, early_stopping=False)
    bits, _ = dec.decode(torch.from_numpy(llr).to(cuda))
    ref, _, _, _ = oracle_mod.flood_decode(g, llr, "minsum", 4, 0.75, 0)
    assert np.array_equal(bits.cpu().numpy().astype(np.uint8), ref)


def test_cpu_input_roundtrip_and_errors(cuda, H4):
    dec = MinSumScaledDecoder(H4, max_iterations=3, early_stopping=False)
    llr = torch.randn(5, 208) + 2
    bits, it = dec.decode(llr)
    assert bits.device.type == "cpu" and it == 3
    with pytest.raises(ValueError):
        dec.decode(torch.randn(5, 207))
    with pytest.raises(UnboundLocalError):
        MinSumScaledDecoder(H4, max_iterations=0).decode(llr)
    empty, _ = dec.decode(torch.zeros(0, 208))
    assert empty.shape == (0, 208)


def test_large_batch_properties(cuda, H32):
    """Full-size batch (B = 65536, cfg3): at 6 dB every frame decodes to the all-zero codeword
    (and the counters say so); the decision is independent of the batch it rides in."""
    from ldpc_neural_decoder.utils import awgn_llr
    B = 65536
    llr = awgn_llr(B, 1664, 6.0, seed=11, device=cuda)
    dec = MinSumScaledDecoder(H32, max_iterations=10, early_stopping=False)
    cnt = torch.zeros(4, dtype=torch.int64, device=cuda)
    bits, _ = dec.decode(llr, out_dtype=torch.uint8, counters=cnt)
    assert cnt.tolist()[:3] == [0, 0, B]
    low = awgn_llr(B, 1664, -4.0, seed=12, device=cuda)
    full, _ = dec.decode(low, out_dtype=torch.uint8)
    part, _ = dec.decode(low[1000:1037].contiguous(), out_dtype=torch.uint8)
    assert torch.equal(full[1000:1037], part)
    assert full.sum() > 0


@pytest.mark.parametrize("z", [4, 32])
def test_graph_create_qc_equals_edge_list_graph(cuda, z):
    """ldpc_graph_create_qc (base graph + Z: load_base_matrix + expand_base_matrix, LU:97-147)
    builds the same graph as ldpc_graph_create on the lifted H's edge list: same info, same
    check-major edges, same decisions."""
    import ctypes
    base = load_base_matrix(code_path(z))
    H = expand_base_matrix(base, z)
    b = np.ascontiguousarray(base.numpy().astype(np.int32))
    h = ctypes.c_void_p()
    with torch.cuda.device(cuda):
        N.check(N.lib().ldpc_graph_create_qc(b.ctypes.data_as(ctypes.c_void_p), b.shape[0], b.shape[1], z,
                                             ctypes.byref(h)))
    try:
        dec = MinSumScaledDecoder(H, max_iterations=6, early_stopping=False)
        g = dec.graph(cuda)
        vals = [ctypes.c_int(), ctypes.c_int(), ctypes.c_int64(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()]
        N.check(N.lib().ldpc_graph_info(h, *[ctypes.byref(v) for v in vals]))
        assert [v.value for v in vals] == [g.M, g.N, g.E, g.Z, g.max_dc, g.max_dv]
        e1c, e1v = np.empty(g.E, np.int32), np.empty(g.E, np.int32)
        e2c, e2v = np.empty(g.E, np.int32), np.empty(g.E, np.int32)
        N.check(N.lib().ldpc_graph_edges(h, e1c.ctypes.data_as(ctypes.c_void_p), e1v.ctypes.data_as(ctypes.c_void_p)))
        N.check(N.lib().ldpc_graph_edges(g.handle, e2c.ctypes.data_as(ctypes.c_void_p),
                                         e2v.ctypes.data_as(ctypes.c_void_p)))
        assert np.array_equal(e1c, e2c) and np.array_equal(e1v, e2v)
        rows, cols = np.nonzero(H.numpy())
        assert np.array_equal(e1c, rows) and np.array_equal(e1v, cols)  # check-major, ascending
        llr = torch.from_numpy(golden(f"channel_z{z}.npz")["llrs"].reshape(-1, H.shape[1])).to(cuda)
        out = [torch.empty(llr.shape, dtype=torch.uint8, device=cuda) for _ in range(2)]
        for handle, o in zip((h, g.handle), out):
            N.check(N.lib().ldpc_flood_decode(handle, N.LDPC_ALGO_MINSUM, N.ptr(llr), llr.shape[0], 6, 0.75,
                                              N.LDPC_ES_OFF, N.LDPC_OUT_U8, N.ptr(o), None, None, None, None, 0,
                                              N.stream_ptr(cuda)))
        assert torch.equal(out[0], out[1])
    finally:
        N.lib().ldpc_graph_destroy(h)


def _validity_by_iteration(oracle_mod, g, x, K):
    val = np.zeros((x.shape[0], K), bool)
    for t in range(1, K + 1):
        val[:, t - 1] = oracle_mod.syndrome_valid(g, oracle_mod.flood_decode(g, x, "minsum", t, 0.75, 0)[0])
    return val


def test_batch_early_stop_fallback_path(cuda, oracle_mod, H4, monkeypatch):
    """The batch-global rule (traditional_decoders.py:104-107) when the T-search passes are not
    enough: a frame that is valid at iteration 5, invalid at 6 and valid again from 7 shares the
    batch with a frame first valid at 6.  Every workgroup is all-valid at some t_wg (5 and 6), T = 6,
    but the batch is first all-valid at 7, so the exhaustive fallback must run and return the
    oracle's batch-global result.  The forced-fallback knob must not change any result."""
    g = oracle_mod.Graph(H4.numpy())
    rng = np.random.default_rng(1)
    s = 10 ** 0.0
    x = (2 * s * (1 / np.sqrt(2) + rng.normal(0, np.sqrt(1 / (2 * s)), size=(2000, g.N)))).astype(np.float32)
    K = 12
    val = _validity_by_iteration(oracle_mod, g, x, K)
    flip = [i for i in range(len(x)) if val[i, 4] and not val[i, 5] and val[i, 6:].all()]
    late = [i for i in range(len(x)) if not val[i, :5].any() and val[i, 5:].all()]
    assert flip and late, "fixture search: no suitable frames"
    easy = np.full((1, g.N), 8.0, np.float32)          # the all-zero codeword, valid from iteration 1
    fg = 16                                            # frames per workgroup at Z = 4
    batch = np.concatenate([x[flip[:1]], np.repeat(easy, fg - 1, 0), x[late[:1]], np.repeat(easy, fg - 1, 0)])
    ref_bits, _, ref_it, _ = oracle_mod.flood_decode(g, batch, "minsum", 20, 0.75, 1)
    assert ref_it == 7
    dec = MinSumScaledDecoder(H4, max_iterations=20, scaling_factor=0.75, early_stopping=True)
    llr = torch.from_numpy(batch).to(cuda)
    bits, it, fr = dec.decode(llr, return_frame_iters=True)
    assert it == 7 and torch.equal(fr.cpu(), torch.full((batch.shape[0],), 7, dtype=torch.int32))
    assert np.array_equal(bits.cpu().numpy().astype(np.uint8), ref_bits)
    # forced fallback on an ordinary batch: same decisions and iteration count as the fast passes
    llr2 = torch.from_numpy(x[:300]).to(cuda)
    b_fast, i_fast = dec.decode(llr2)
    monkeypatch.setenv("LDPC_FLOOD_ES_FALLBACK", "1")
    b_fb, i_fb = dec.decode(llr2)
    b_fb2, i_fb2 = dec.decode(llr)
    assert i_fast == i_fb and torch.equal(b_fast, b_fb)
    assert i_fb2 == 7 and torch.equal(b_fb2, bits)


@pytest.mark.parametrize("algo", ["minsum", "bp"])
@pytest.mark.parametrize("es", [False, True, "frame"])
def test_streaming_kernels_match_lds_kernels(cuda, H32, monkeypatch, algo, es):
    """The streaming decoder (messages in HBM, any graph) against the LDS-resident one on the
    reference's code: identical decisions, iteration counts and counters (min-sum and BP share
    the float32 operation sequence)."""
    llr = torch.from_numpy(golden("trad_z32_low.npz")["llrs"].reshape(-1, 1664)).to(cuda)
    llr = torch.cat([llr, torch.from_numpy(golden("channel_z32.npz")["llrs"].reshape(-1, 1664)).to(cuda)])
    mk = (lambda: MinSumScaledDecoder(H32, 9, 0.75, early_stopping=es)) if algo == "minsum" \
        else (lambda: BeliefPropagationDecoder(H32, 9, early_stopping=es))
    c1 = torch.zeros(4, dtype=torch.int64, device=cuda)
    c2 = torch.zeros(4, dtype=torch.int64, device=cuda)
    b1, i1, f1 = mk().decode(llr, return_frame_iters=True)
    mk().decode(llr, counters=c1)
    monkeypatch.setenv("LDPC_FLOOD_STREAM", "1")
    b2, i2, f2 = mk().decode(llr, return_frame_iters=True)
    mk().decode(llr, counters=c2)
    assert torch.equal(b1, b2) and i1 == i2 and torch.equal(f1, f2)
    assert torch.equal(c1, c2)


@pytest.mark.parametrize("z,B", [(12, 40), (96, 9), (384, 3)])
@pytest.mark.parametrize("es", [0, 1, 2])
def test_lifting_sizes_beyond_lds(cuda, oracle_mod, z, B, es):
    """expand_base_matrix lifts any Z (ldpc_utils.py:97-125).  Z = 12 and 96 do not divide 64 and
    Z = 384 (the 5G maximum) is far beyond a CU's LDS: these decode on the streaming kernels.
    Min-sum decisions and iteration counts are bit-exact to the oracle in every stopping mode."""
    base = load_base_matrix(code_path(32))
    H = expand_base_matrix(base, z)
    g = oracle_mod.Graph(H.numpy())
    rng = np.random.default_rng(z)
    s = 10 ** (0.5 / 10)
    x = (2 * s * (1 / np.sqrt(2) + rng.normal(0, np.sqrt(1 / (2 * s)), size=(B, g.N)))).astype(np.float32)
    ref_bits, _, ref_it, ref_frame_it = oracle_mod.flood_decode(g, x, "minsum", 8, 0.75, es)
    dec = MinSumScaledDecoder(H, 8, 0.75, early_stopping={0: False, 1: True, 2: "frame"}[es])
    bits, it, fr = dec.decode(torch.from_numpy(x).to(cuda), return_frame_iters=True)
    assert np.array_equal(bits.cpu().numpy().astype(np.uint8), ref_bits)
    # frame mode: the batch-level count is the largest per-frame count
    assert it == (8 if es == 0 else (ref_it if es == 1 else int(ref_frame_it.max())))
    if es == 2:
        assert np.array_equal(fr.cpu().numpy(), ref_frame_it)


def test_streaming_large_sparse_code_chunked_grid(cuda, oracle_mod):
    """A non-QC (3, 6)-regular code with 70 000 checks and 140 000 variables: beyond any LDS
    schedule, and more nodes of one degree than a launch's grid.y (65 535), so the streaming
    kernels' per-degree launches are chunked.  Decisions bit-exact to the oracle, on the C ABI
    with the graph built from the edge list (ldpc_graph_create)."""
    M, Nv, dv, dc = 70000, 140000, 3, 6
    rng = np.random.default_rng(11)
    sockets = np.repeat(np.arange(Nv, dtype=np.int64), dv)
    rng.shuffle(sockets)
    chk = np.repeat(np.arange(M, dtype=np.int64), dc)
    pairs = np.unique(chk * Nv + sockets)  # drop repeated (check, var) pairs; sorted check-major
    ec, ev = (pairs // Nv).astype(np.int32), (pairs % Nv).astype(np.int32)
    g = N.NativeGraph(ec, ev, M, Nv, cuda)
    assert g.Z == 1 and g.E == len(ec)
    B, iters = 6, 4
    x = rng.normal(1.0, 2.0, size=(B, Nv)).astype(np.float32)
    bits = torch.empty((B, Nv), dtype=torch.uint8, device=cuda)
    wsb = N.check(N.lib().ldpc_flood_workspace_size(g.handle, B, iters, N.LDPC_ES_OFF))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=cuda)
    xt = torch.from_numpy(x).to(cuda)
    N.check(N.lib().ldpc_flood_decode(g.handle, N.LDPC_ALGO_MINSUM, N.ptr(xt), B, iters, 0.75, N.LDPC_ES_OFF,
                                      N.LDPC_OUT_U8, N.ptr(bits), None, None, None, N.ptr(ws), ws.numel(), None))
    torch.cuda.synchronize()
    og = object.__new__(oracle_mod.Graph)  # the oracle's graph from the same edge list
    og.M, og.N, og.E = M, Nv, len(ec)
    og.edge_chk, og.edge_var = ec, ev
    og.chk_ptr = np.zeros(M + 1, dtype=np.int32)
    np.cumsum(np.bincount(ec, minlength=M), out=og.chk_ptr[1:])
    og.var_edge = np.lexsort((ec, ev)).astype(np.int32)
    og.var_ptr = np.zeros(Nv + 1, dtype=np.int32)
    np.cumsum(np.bincount(ev, minlength=Nv), out=og.var_ptr[1:])
    ref, _, _, _ = oracle_mod.flood_decode(og, x, "minsum", iters, 0.75, 0)
    assert np.array_equal(bits.cpu().numpy(), ref)


def test_cfg3_full_batch_spot_frames_vs_oracle(cuda, oracle_mod, H32):
    """cfg3 exactly as benched (BG2 Z=32, min-sum alpha 0.75, 10 iterations, B = 65 536 frames of
    the on-device channel at 2 dB, bench.py's seed): four spot frames spread over the batch (first,
    last, and two in between) are bit-exact to the oracle decoding the same LLR rows, and the
    counters equal the decisions' own error counts."""
    from ldpc_neural_decoder.utils import awgn_llr
    B = 65536
    llr = awgn_llr(B, 1664, 2.0, seed=20251015, frame_offset=0, device=cuda)
    dec = MinSumScaledDecoder(H32, max_iterations=10, scaling_factor=0.75, early_stopping=False)
    cnt = torch.zeros(4, dtype=torch.int64, device=cuda)
    bits, _ = dec.decode(llr, out_dtype=torch.uint8, counters=cnt)
    spots = [0, 12345, 40001, B - 1]
    x = llr[spots].cpu().numpy()
    ref, _, _, _ = oracle_mod.flood_decode(oracle_mod.Graph(H32.numpy()), x, "minsum", 10, 0.75, 0)
    assert np.array_equal(bits[spots].cpu().numpy(), ref)
    be = int(bits.sum().item())
    fe = int((bits.sum(1) > 0).sum().item())
    assert cnt.tolist() == [be, fe, B, 10 * B]


@pytest.mark.parametrize("algo", ["minsum", "bp"])
def test_cfg3_full_batch_with_errors_every_frame_vs_oracle(cuda, oracle_mod, H32, algo):
    """cfg3's full per-GPU batch (B = 65 536, BG2 Z=32, 10 iterations) at -4 dB, where most frames
    still carry errors after the decode, compared with the oracle (traditional_decoders.py:42-109,
    :177-260) on EVERY frame, so that a workgroup-indexing or batch-tail fault with non-trivial
    decisions cannot hide.  Min-sum: bit-exact.  BP: the oracle bar
    (<= 1e-4 of bits; measured 0).  The oracle runs its OpenMP frame loop on the host's share."""
    from ldpc_neural_decoder.utils import awgn_llr
    B = 65536
    llr = awgn_llr(B, 1664, -4.0, seed=424242, frame_offset=0, device=cuda)
    if algo == "minsum":
        dec = MinSumScaledDecoder(H32, max_iterations=10, scaling_factor=0.75, early_stopping=False)
    else:
        dec = BeliefPropagationDecoder(H32, max_iterations=10, early_stopping=False)
    cnt = torch.zeros(4, dtype=torch.int64, device=cuda)
    bits, _ = dec.decode(llr, out_dtype=torch.uint8, counters=cnt)
    got = bits.cpu().numpy()
    x = llr.cpu().numpy()
    del llr
    oracle_mod.set_threads(min(16, os.cpu_count() or 1))
    ref, _, _, _ = oracle_mod.flood_decode(oracle_mod.Graph(H32.numpy()), x, algo, 10, 0.75, 0)
    frame_err = int((ref.sum(1) > 0).sum())
    assert frame_err > B // 4, f"-4 dB should leave many frames in error (got {frame_err})"
    if algo == "minsum":
        bad = np.nonzero((got != ref).any(1))[0]
        assert bad.size == 0, f"{bad.size} frames differ, first {bad[:8].tolist()}"
    else:
        assert (got != ref).mean() <= 1e-4, int((got != ref).sum())
    assert cnt.tolist() == [int(got.sum()), int((got.sum(1) > 0).sum()), B, 10 * B]
