"""Hybrid min-sum decoder (CustomMinSum*, message_gnn_decoder.py:966-1291): oracle and host logic (CPU).

The reference's decoder cannot run.  What pins this build's definition of it:
  * the check update: the reference's own CustomCheckMessageGNNLayer.check_layer_update, run on the
    per-message rows its loop reads (tests/golden/make_custom_golden.py -> custom_check_z4.npz);
    observed here through one iteration of the oracle, where v2c = llr and
    probs = sigmoid(llr + sum of that c2v);
  * the variable update and damping (MGD:650-663) cannot execute in the reference: the oracle's C
    restatement is the definition, cross-checked below against an independent numpy restatement;
  * the module's state_dict layout against the reference's constructor (fixture sd_keys)."""
import numpy as np
import pytest
import torch

from conftest import golden

from ldpc_neural_decoder.models import create_custom_minsum_message_gnn_decoder
from ldpc_neural_decoder.models.custom_decoders import _graph_from_index_tensors
from ldpc_neural_decoder.utils import edge_list

TOL = 2e-6  # float32 sigmoid: the C library's expf vs numpy's exp


def graph_of_messages(oracle, msg_chk, msg_var, n):
    H = np.zeros((int(msg_chk.max()) + 1, n), dtype=np.uint8)
    H[msg_chk, msg_var] = 1
    return oracle.Graph(H), H


def sigmoid32(x):
    x = x.astype(np.float32)
    return (np.float32(1.0) / (np.float32(1.0) + np.exp(-x))).astype(np.float32)


def test_check_update_pinned_by_reference(oracle_mod):
    d = golden("custom_check_z4.npz")
    llr, c2v, chk, var = d["llr"], d["c2v"], d["msg_chk"], d["msg_var"]
    g, _ = graph_of_messages(oracle_mod, chk, var, llr.shape[1])
    # S_v over v's messages in ascending message order (the fixture's messages are check-major)
    out = llr.copy()
    for v in range(llr.shape[1]):
        ms = np.nonzero(var == v)[0]
        if len(ms):
            s = c2v[:, ms[0]].copy()
            for m in ms[1:]:
                s = (s + c2v[:, m]).astype(np.float32)
            out[:, v] = (out[:, v] + s).astype(np.float32)
    probs = oracle_mod.custom_minsum(g, llr, 1)
    np.testing.assert_allclose(probs, sigmoid32(out), atol=TOL, rtol=0)
    assert (c2v[0] == 0).sum() > 0  # the zeros reached the checks (torch.sign(0) = 0)


def numpy_custom_minsum(H, llr, iters):
    """Independent restatement (per frame, python loops; see custom_decoders.py docstring)."""
    ec, ev = edge_list(H)
    E = len(ec)
    B, n = llr.shape
    out = np.zeros_like(llr)
    f32 = np.float32
    for b in range(B):
        c2v = np.zeros(E, dtype=np.float32)
        v2c = np.zeros(E, dtype=np.float32)
        for it in range(iters):
            for v in range(n):
                ms = np.nonzero(ev == v)[0]
                if not len(ms):
                    continue
                s = c2v[ms[0]]
                for m in ms[1:]:
                    s = f32(s + c2v[m])
                tot = f32(llr[b, v] + s)
                for m in ms:
                    x = f32(tot - c2v[m])
                    if it > 0:
                        x = f32(f32(f32(0.5) * x) + f32(f32(0.5) * c2v[m]))
                    v2c[m] = x
            new = np.zeros(E, dtype=np.float32)
            for c in range(H.shape[0]):
                ms = np.nonzero(ec == c)[0]
                for m in ms:
                    others = [o for o in ms if o != m]
                    if not others:
                        continue
                    sg = f32(1.0)
                    mn = f32(np.inf)
                    for o in others:
                        sg = f32(sg * np.sign(v2c[o]))
                        mn = min(mn, abs(v2c[o]))
                    new[m] = f32(sg * mn)
            c2v = new
        for v in range(n):
            ms = np.nonzero(ev == v)[0]
            o = llr[b, v]
            if len(ms):
                s = c2v[ms[0]]
                for m in ms[1:]:
                    s = f32(s + c2v[m])
                o = f32(o + s)
            out[b, v] = o
    return sigmoid32(out)


def test_oracle_matches_numpy_restatement(oracle_mod):
    rng = np.random.default_rng(7)
    H = (rng.random((9, 16)) < 0.3).astype(np.uint8)
    H[0, :] = 0
    H[0, 3] = 1                       # a degree-1 check: its edge gets 0
    H[:, 5] = 0                       # a variable with no edges: probs = sigmoid(llr)
    llr = rng.normal(0.5, 1.5, (5, 16)).astype(np.float32)
    llr[1, ::4] = 0.0
    g = oracle_mod.Graph(H)
    for iters in (1, 2, 4):
        np.testing.assert_allclose(oracle_mod.custom_minsum(g, llr, iters), numpy_custom_minsum(H, llr, iters),
                                   atol=TOL, rtol=0)
    np.testing.assert_allclose(oracle_mod.custom_minsum(g, llr, 0), sigmoid32(llr), atol=TOL, rtol=0)


def test_state_dict_layout_matches_reference():
    d = golden("custom_check_z4.npz")
    E = len(d["msg_chk"])
    H = np.zeros((int(d["msg_chk"].max()) + 1, d["llr"].shape[1]), dtype=np.float32)
    H[d["msg_chk"], d["msg_var"]] = 1
    dec, conv = create_custom_minsum_message_gnn_decoder(torch.from_numpy(H), num_iterations=3, hidden_dim=8)
    assert len(conv.messages) == E
    sd = dec.state_dict()
    assert sorted(sd) == list(d["sd_keys"])
    numel = [len(sd[k].shape) and sd[k].numel() for k in sorted(sd)]
    assert numel == list(d["sd_numel"])


def test_index_tensors_rebuild_the_graph():
    rng = np.random.default_rng(3)
    H = (rng.random((12, 20)) < 0.25).astype(np.float32)
    dec, conv = create_custom_minsum_message_gnn_decoder(torch.from_numpy(H), num_iterations=2)
    ec, ev = _graph_from_index_tensors(dec.check_index_tensor, dec.variable_index_tensor, 12, 20)
    rc, rv = edge_list(torch.from_numpy(H))
    assert np.array_equal(ec, rc) and np.array_equal(ev, rv)
    # the reference's message-id layout: check rows list the check's messages, ascending
    ci = dec.check_index_tensor
    for c in range(12):
        row = ci[c][ci[c] >= 0].tolist()
        assert row == conv.check_to_messages[c]


def test_variable_decoder_state_dict_layout_matches_reference():
    from ldpc_neural_decoder.models import CustomVariableMessageGNNDecoder
    d = golden("custom_check_z4.npz")
    dec = CustomVariableMessageGNNDecoder(len(d["msg_chk"]), 3, 64, 1, 3)
    sd = dec.state_dict()
    assert sorted(sd) == list(d["sdv_keys"])
    assert [len(sd[k].shape) and sd[k].numel() for k in sorted(sd)] == list(d["sdv_numel"])


def test_variable_decoder_hidden_dims():
    """The reference's constructor takes any hidden_dim (MGD:765): this build runs 1 .. 1024 (64 on the
    split-MFMA kernels, other widths on the tiled fp32 kernels) and refuses the rest when the decoder
    is constructed, with a message that says so (not at the first forward)."""
    from ldpc_neural_decoder.models import CustomVariableMessageGNNDecoder
    for h in (8, 32, 96, 1024):
        CustomVariableMessageGNNDecoder(40, 3, h, 1, 3)
    with pytest.raises(ValueError, match="hidden_dim 1 .. 1024"):
        CustomVariableMessageGNNDecoder(40, 3, 2048, 1, 3)
