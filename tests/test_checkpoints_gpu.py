"""The shipped trained checkpoints, on the paths the bench lines use them on (GPU).

checkpoints/gnn_bg2_z32_i15_h64.pt  cfg5: 15 layers, bf16 features + bf16 MFMA, per-frame early
                                    termination (a frame stops after the first layer whose decision
                                    through the last layer's output_projection is a codeword)
checkpoints/gnn_bg2_z32_i10_h64.pt  cfg4: 10 layers, fp32

Both are trained with tools/train_gnn_checkpoint.py (Adam, grad clip 1.0) and load with
torch.load(weights_only=True) into the reference's state_dict schema
(message_gnn_decoder.py:162-188, run_comparison_all.py:124-143).

Bars (stated):
  * bf16 vs the fp32 oracle at a frame's stop layer l: oracle.gnn_forward(..., all_layers=True)[l - 1]
    (the same decision the syndrome check reads, message_gnn_decoder.py:270, :298-307): mean
    |dp| <= 5e-3 and >= 99.5 % of the confident oracle decisions (|p - 0.5| > 0.05) equal -- the bar of
    test_gnn_gpu.py::test_bf16_path_within_tolerance, now on trained weights;
  * the oracle's own decision at a stop layer l < 15 satisfies every parity check (the bf16 path
    stopped on a codeword that the fp32 arithmetic also reaches);
  * early termination on vs off at 0 dB (bit errors present; at 1 dB the checkpoint decodes 8192
    codewords without one): >= 99.9 % of decisions equal ("check vs no-ET run
    statistically");
  * chunking is exact: a frame's result depends on that frame alone, also while frames terminate;
  * fp32 cfg4 checkpoint vs the oracle: |dp| <= 2e-5 (the bar of test_gnn_depth_gpu.py).
"""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, code_path

from ldpc_neural_decoder.models import create_message_gnn_decoder
from ldpc_neural_decoder.utils import awgn_llr, expand_base_matrix, load_base_matrix
from ldpc_neural_decoder.utils.encoding import SystematicEncoder

pytestmark = pytest.mark.gpu
CFG_BATCH = 32768


def _load(layers, cuda, precision):
    path = os.path.join(ROOT, "checkpoints", f"gnn_bg2_z32_i{layers}_h64.pt")
    ck = torch.load(path, map_location="cpu", weights_only=True)
    assert ck["num_iterations"] == layers and ck["hidden_dim"] == 64
    base = load_base_matrix(code_path(32))
    H = expand_base_matrix(base, 32)
    dec, conv = create_message_gnn_decoder(H, num_iterations=layers, hidden_dim=64, base_graph=base, Z=32)
    dec.load_state_dict(ck["model_state_dict"])
    dec = dec.to(cuda)
    dec.precision = precision
    types = conv.get_message_types(base, 32)
    return H, dec, conv, types


def _codewords(H, B, snr, seed, cuda):
    gen = torch.Generator(device=cuda)
    gen.manual_seed(seed)
    bits = SystematicEncoder(H, cuda).random(B, generator=gen).to(torch.uint8)
    return bits, awgn_llr(B, H.shape[1], snr, seed=seed, bits=bits, device=cuda)


def _native(dec, conv, types, llr, cuda, chunk=None):
    io = conv.message_to_var_index().to(cuda).to(torch.int32)
    t = types.to(cuda).to(torch.int32)
    with torch.no_grad():
        return dec.native_forward(llr, io, t, conv.var_groups, conv.check_groups, chunk=chunk)


def _oracle_layers(oracle_mod, dec, conv, H, types, llr):
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    return oracle_mod.gnn_forward(sd, llr.cpu(), conv.edge_var, conv.edge_var, conv.edge_chk,
                                  H.shape[1], H.shape[0], types, all_layers=True).numpy()


@pytest.fixture(scope="module")
def cfg5(cuda):
    H, dec, conv, types = _load(15, cuda, "bf16")
    dec.early_termination = True
    bits, llr = _codewords(H, CFG_BATCH, 2.0, 20251015, cuda)
    p = _native(dec, conv, types, llr, cuda)
    it = dec.last_iterations.clone()
    return H, dec, conv, types, bits, llr, p, it


def test_cfg5_terminates_at_full_batch(cfg5):
    H, dec, conv, types, bits, llr, p, it = cfg5
    avg = float(it.double().mean())
    hist = torch.bincount(it.cpu().long(), minlength=16)[1:].tolist()
    print(f"cfg5 trained checkpoint, {CFG_BATCH} random codewords at 2 dB: avg layers {avg:.3f}, "
          f"stop-layer histogram {hist}")
    assert bool(((it >= 1) & (it <= 15)).all())
    assert avg < 15.0
    assert int((it < 15).sum()) > CFG_BATCH // 2  # termination fires for most frames
    assert bool(torch.isfinite(p).all())
    # decisions of the terminated frames are codewords (the syndrome check's own definition)
    enc = SystematicEncoder(H, p.device)
    hard = (p > 0.5).float()
    stopped = it < 15
    assert bool(enc.syndrome_ok(hard[stopped]).all())


def test_cfg5_spot_frames_vs_oracle_at_stop_layer(cfg5, oracle_mod):
    H, dec, conv, types, bits, llr, p, it = cfg5
    itc = it.cpu().numpy()
    # 8 frames spread over the stop layers that occur (earliest, latest, and in between)
    order = np.argsort(itc, kind="stable")
    pick = np.unique(order[np.linspace(0, CFG_BATCH - 1, 8).astype(int)])
    idx = torch.from_numpy(pick).to(llr.device)
    ref_all = _oracle_layers(oracle_mod, dec, conv, H, types, llr[idx])  # (15, 8, N)
    graph = oracle_mod.Graph(H.numpy())
    pn = p[idx].cpu().numpy()
    for r, f in enumerate(pick):
        stop = int(itc[f])
        ref = ref_all[stop - 1, r]
        d = np.abs(pn[r] - ref)
        sure = np.abs(ref - 0.5) > 0.05
        agree = ((pn[r] > 0.5) == (ref > 0.5))[sure].mean()
        print(f"frame {f}: stop layer {stop}, mean |dp| {d.mean():.2e}, max {d.max():.2e}, agree {agree:.5f}")
        assert d.mean() <= 5e-3 and agree >= 0.995, (f, stop)
        if stop < 15:
            hard = (ref > 0.5).astype(np.uint8)[None]
            assert bool(oracle_mod.syndrome_valid(graph, hard)[0]), (f, stop)


def test_cfg5_chunked_equals_unchunked_while_terminating(cfg5, cuda):
    H, dec, conv, types, bits, llr, p, it = cfg5
    assert int((it < 15).sum()) > 0
    q = _native(dec, conv, types, llr, cuda, chunk=5000)
    assert torch.equal(p, q) and torch.equal(it, dec.last_iterations)
    sub = _native(dec, conv, types, llr[31000:31111].contiguous(), cuda)
    assert torch.equal(sub, p[31000:31111]) and torch.equal(dec.last_iterations, it[31000:31111])


def test_cfg5_et_on_vs_off_at_0db(cuda):
    H, dec, conv, types = _load(15, cuda, "bf16")
    bits, llr = _codewords(H, 16384, 0.0, 777, cuda)
    dec.early_termination = True
    p_on = _native(dec, conv, types, llr, cuda)
    it = dec.last_iterations.clone()
    dec.early_termination = False
    p_off = _native(dec, conv, types, llr, cuda)
    d_on, d_off = p_on > 0.5, p_off > 0.5
    err_on = int((d_on != bits.bool()).sum())
    err_off = int((d_off != bits.bool()).sum())
    agree = float((d_on == d_off).double().mean())
    print(f"0 dB, 16384 codewords: avg layers {float(it.double().mean()):.3f}, bit errors ET on {err_on} / "
          f"off {err_off}, decisions equal {agree:.6f}")
    assert err_off > 0  # the statistic is taken where decoding errors exist
    assert agree >= 0.999
    # frames that never terminated ran the same 15 layers: bitwise the ET-off outputs
    full = it == 15
    assert bool(full.any()) and torch.equal(p_on[full], p_off[full])


def test_cfg4_fp32_checkpoint_vs_oracle(cuda, oracle_mod):
    H, dec, conv, types = _load(10, cuda, "fp32")
    bits, llr = _codewords(H, 4096, 2.0, 4242, cuda)
    p = _native(dec, conv, types, llr, cuda)
    pick = torch.tensor([0, 1, 777, 1500, 2048, 3001, 4000, 4095], device=cuda)
    ref = _oracle_layers(oracle_mod, dec, conv, H, types, llr[pick])[-1]
    np.testing.assert_allclose(p[pick].cpu().numpy(), ref, atol=2e-5)
    ber = float(((p > 0.5) != bits.bool()).double().mean())
    print(f"cfg4 trained checkpoint, 4096 codewords at 2 dB: BER {ber:.2e}")
    assert ber < 1e-3


def _strata(B, chunk, E, H, extra=16, seed=5):
    """Frames where the fp32 forward's indexing changes regime: the first and last frame of every
    chunk (LDPC_GNN_WORKSPACE_BYTES), of every frame half (the two streams of gnn_fp32_forward), and
    either side of the frames whose (B, E, H) offsets cross 2^29 / 2^30 / 2^31 elements within a
    half, plus `extra` random frames."""
    picks = set()
    for s in range(0, B, chunk):
        n = min(chunk, B - s)
        halves = [(s, n)] if n < 128 else [(s, n // 2), (s + n // 2, n - n // 2)]
        for h0, hn in halves:
            picks.update({h0, h0 + 1, h0 + hn - 2, h0 + hn - 1})
            for k in (29, 30, 31):
                f = (1 << k) // (E * H)
                picks.update({h0 + f - 1, h0 + f, h0 + f + 1} if f + 1 < hn else set())
    rng = np.random.default_rng(seed)
    picks.update(rng.integers(0, B, extra).tolist())
    return sorted(p for p in picks if 0 <= p < B)


def test_cfg4_full_batch_stratified_vs_oracle(cuda, oracle_mod):
    """cfg4 at its full per-GPU batch (32768 frames, 10 layers, the trained checkpoint, random
    codewords at 0 dB: decoding errors present) against the oracle on >= 64 frames chosen where the
    indexing changes regime (_strata), at the fp32 bar (|dp| <= 2e-5)."""
    from ldpc_neural_decoder import _native as N
    H, dec, conv, types = _load(10, cuda, "fp32")
    bits, llr = _codewords(H, CFG_BATCH, 0.0, 6060, cuda)
    p = _native(dec, conv, types, llr, cuda)
    assert bool(torch.isfinite(p).all())
    # the chunk native_forward used (the same budget arithmetic)
    plan = dec._plan(conv.var_groups, conv.check_groups, cuda)
    ws = lambda b: N.check(N.lib().ldpc_gnn_workspace_size(plan.handle, 64, H.shape[1], b, 10, 0))
    budget = int(os.environ.get("LDPC_GNN_WORKSPACE_BYTES", 48 << 30))
    chunk = max(1, min(CFG_BATCH, (budget - ws(1)) // max(ws(2) - ws(1), 1)))
    E = len(conv.messages)
    pick = _strata(CFG_BATCH, chunk, E, 64)
    assert len(pick) >= 64, (len(pick), chunk)
    idx = torch.tensor(pick, device=cuda)
    ref = _oracle_layers(oracle_mod, dec, conv, H, types, llr[idx])[-1]
    got = p[idx].cpu().numpy()
    err = np.abs(got - ref).max(axis=1)
    print(f"cfg4 stratified: chunk {chunk}, {len(pick)} frames, max |dp| {err.max():.2e}, "
          f"BER {float(((p > 0.5) != bits.bool()).double().mean()):.2e}")
    bad = [(f, float(e)) for f, e in zip(pick, err) if e > 2e-5]
    assert not bad, bad[:8]
