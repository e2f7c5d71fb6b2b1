"""Pin the CPU oracle to the reference: every golden fixture made by importing the reference
(tests/golden/make_golden.py) must be reproduced by oracle/ (CPU, no GPU needed)."""
import numpy as np
import pytest
import torch

from conftest import code_path, golden

SNRS = [-1.0, 0.0, 2.0, 4.0, 6.0]


@pytest.mark.parametrize("z", [4, 32])
def test_expand_and_edge_order(oracle_mod, z):
    c = golden(f"codes_z{z}.npz")
    base = oracle_mod.load_base(code_path(z))
    assert np.array_equal(base.astype(np.int32), c["base"])
    H = oracle_mod.expand(base, z)
    assert H.shape == tuple(c["H_shape"]) and H.sum() == c["H_sum"]
    assert np.array_equal(np.nonzero(H)[0], c["H_rows"]) and np.array_equal(np.nonzero(H)[1], c["H_cols"])
    g = oracle_mod.Graph(H)
    assert np.array_equal(g.edge_var, c["messages"][:, 0])
    assert np.array_equal(g.edge_chk, c["messages"][:, 1])
    assert np.array_equal(oracle_mod.message_types(g, base, z), c["message_types"])


@pytest.mark.parametrize("z", [4, 32])
def test_normalized_adjacency_is_group_mean(z):
    """D^-1/2 (A+I) D^-1/2 of message_gnn_decoder.py:449-469 is a group mean: diag = 1/|group|,
    row sums = 1 (fixtures hold the reference matrix's diagonal and row sums)."""
    c = golden(f"codes_z{z}.npz")
    ev, ec = c["messages"][:, 0], c["messages"][:, 1]
    dv = np.bincount(ev)[ev].astype(np.float32)
    dc = np.bincount(ec)[ec].astype(np.float32)
    np.testing.assert_allclose(c["Av_diag"], 1.0 / dv, rtol=1e-6)
    np.testing.assert_allclose(c["Ac_diag"], 1.0 / dc, rtol=1e-6)
    np.testing.assert_allclose(c["Av_rowsum"], 1.0, rtol=1e-5)
    np.testing.assert_allclose(c["Ac_rowsum"], 1.0, rtol=1e-5)


def _graph(oracle_mod, z):
    return oracle_mod.Graph(oracle_mod.expand(oracle_mod.load_base(code_path(z)), z))


@pytest.mark.parametrize("key,algo,alpha", [("bp", "bp", 0.0), ("ms_a0.75", "minsum", 0.75),
                                            ("ms_a0.8", "minsum", 0.8)])
@pytest.mark.parametrize("es", [0, 1])
def test_flood_z4_matches_reference(oracle_mod, key, algo, alpha, es):
    g = _graph(oracle_mod, 4)
    ch, t = golden("channel_z4.npz"), golden("trad_z4.npz")
    for k in range(len(SNRS)):
        bits, _, it, _ = oracle_mod.flood_decode(g, ch["llrs"][k], algo, 5, alpha, es)
        assert np.array_equal(bits, t[f"{key}_es{es}_bits"][k]), (key, es, SNRS[k])
        assert it == t[f"{key}_es{es}_iters"][k]


@pytest.mark.parametrize("es", [0, 1])
def test_minsum_z32_matches_reference(oracle_mod, es):
    g = _graph(oracle_mod, 32)
    ch, t = golden("channel_z32.npz"), golden("trad_z32.npz")
    for k in range(len(SNRS)):
        bits, _, it, _ = oracle_mod.flood_decode(g, ch["llrs"][k], "minsum", 10, 0.75, es)
        assert np.array_equal(bits, t[f"ms_a0.75_es{es}_bits"][k]), (es, SNRS[k])
        assert it == t[f"ms_a0.75_es{es}_iters"][k]


@pytest.mark.parametrize("es", [0, 1])
def test_minsum_z32_low_snr_matches_reference(oracle_mod, es):
    """-6/-5/-4 dB: frames with hundreds of residual errors, decisions still bit-identical."""
    g = _graph(oracle_mod, 32)
    t = golden("trad_z32_low.npz")
    for k in range(len(t["snrs"])):
        bits, _, it, _ = oracle_mod.flood_decode(g, t["llrs"][k], "minsum", 10, 0.75, es)
        assert np.array_equal(bits, t[f"ms_a0.75_es{es}_bits"][k]), (es, t["snrs"][k])
        assert it == t[f"ms_a0.75_es{es}_iters"][k]


@pytest.mark.parametrize("es", [0, 1])
def test_bp_z32_matches_reference(oracle_mod, es):
    """BeliefPropagationDecoder (traditional_decoders.py:42-109) at Z=32, 10 iterations, -6..0 dB
    (bp_z32.npz, made by importing the reference): iteration counts equal, decisions within the BP
    bar (<= 0.1 % of bits: the reference's tanh/atanh are SLEEF approximations)."""
    g = _graph(oracle_mod, 32)
    t = golden("bp_z32.npz")
    diff = total = 0
    for k in range(len(t["snrs"])):
        bits, _, it, _ = oracle_mod.flood_decode(g, t["llrs"][k], "bp", 10, 0.0, es)
        ref = t[f"bp_es{es}_bits"][k]
        diff += int((bits != ref).sum())
        total += ref.size
        assert it == t[f"bp_es{es}_iters"][k], (es, t["snrs"][k])
    assert diff <= 1e-3 * total, diff


def test_fixtures_exercise_errors():
    """The low-SNR fixtures must contain decoding errors, or bit-equality would prove little."""
    t = golden("trad_z32_low.npz")
    assert t["ms_a0.75_es0_bits"][0].sum() > 100  # -6 dB
    t4 = golden("trad_z4.npz")
    assert t4["bp_es0_bits"][0].sum() > 50 and t4["ms_a0.75_es0_bits"][0].sum() > 50
    b32 = golden("bp_z32.npz")
    assert b32["bp_es0_bits"][0].sum() > 100  # -6 dB: BP leaves errors too


@pytest.mark.parametrize("z", [4, 32])
def test_gnn_oracle_matches_reference(oracle_mod, z):
    c, f = golden(f"codes_z{z}.npz"), golden(f"gnn_z{z}.npz")
    sd = {k[3:]: torch.from_numpy(f[k]) for k in f.files if k.startswith("w__")}
    ev, ec = c["messages"][:, 0], c["messages"][:, 1]
    Nv, M = int(c["H_shape"][1]), int(c["H_shape"][0])
    p = oracle_mod.gnn_forward(sd, f["llr"], ev, ev, ec, Nv, M, c["message_types"]).numpy()
    np.testing.assert_allclose(p, f["probs"], atol=2e-6)
    p = oracle_mod.gnn_forward(sd, f["llr"], ev, ev, ec, Nv, M, None).numpy()
    np.testing.assert_allclose(p, f["probs_no_types"], atol=2e-6)
    quirk = (ev == 0).astype(np.int64)  # column 0 of the (E, N) one-hot, .long()
    p = oracle_mod.gnn_forward(sd, f["llr"], quirk, ev, ec, Nv, M, c["message_types"]).numpy()
    np.testing.assert_allclose(p, f["probs_2d_quirk"], atol=2e-6)
    _, loss = oracle_mod.gnn_forward(sd, f["llr"], ev, ev, ec, Nv, M, c["message_types"],
                                     f["ground_truth"])
    assert abs(loss.item() - float(f["loss"])) < 1e-5


def test_philox_known_answers(oracle_mod):
    """Random123 Philox-4x32-10 known-answer vectors."""
    kat = [([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
           ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
           ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
            [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1])]
    for ctr, key, want in kat:
        assert oracle_mod.philox4x32_10(ctr, key)[0].tolist() == want


def test_oracle_per_frame_mode_is_consistent(oracle_mod):
    """Per-frame early stop: each frame's bits equal a fixed-iteration decode at its own
    iteration count, and that decision is a valid codeword when it stopped early."""
    g = _graph(oracle_mod, 4)
    llr = golden("channel_z4.npz")["llrs"][3]
    bits, _, _, iters = oracle_mod.flood_decode(g, llr, "minsum", 8, 0.75, 2)
    for b in range(0, 64, 7):
        ref, _, _, _ = oracle_mod.flood_decode(g, llr[b:b + 1], "minsum", int(iters[b]), 0.75, 0)
        assert np.array_equal(bits[b], ref[0])
        if iters[b] < 8:
            assert oracle_mod.syndrome_valid(g, bits[b:b + 1])[0]


def test_dense_gnn_oracle_matches_reference():
    """oracle.gnn_forward_dense (the reference's dense-bmm aggregation, used to pin the general-
    adjacency path) on the normalized clique adjacencies reproduces the reference's probs."""
    import oracle as oracle_py
    from ldpc_neural_decoder.models.message_gnn_decoder import TannerToMessageGraph
    from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix
    from conftest import code_path
    c, f = golden("codes_z4.npz"), golden("gnn_z4.npz")
    sd = {k[3:]: torch.from_numpy(f[k]) for k in f.files if k.startswith("w__")}
    H = expand_base_matrix(load_base_matrix(code_path(4)), 4)
    conv = TannerToMessageGraph(H)
    ev = c["messages"][:, 0]
    p = oracle_py.gnn_forward_dense(sd, f["llr"], ev, int(c["H_shape"][1]), conv.var_to_check_adjacency,
                                    conv.check_to_var_adjacency, c["message_types"]).numpy()
    np.testing.assert_allclose(p, f["probs"], atol=2e-6)
