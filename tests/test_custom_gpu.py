"""Hybrid min-sum decoder (CustomMinSum*, message_gnn_decoder.py:1137-1251) on the GPU vs the oracle.

Bar: probs within 2e-6 (absolute) of oracle/ldpc_oracle.c's ldpc_oracle_custom_minsum -- every
message update is the same float32 operation sequence; only the final sigmoid's expf may differ in
the last ulp.  The check update is pinned to the reference's own check_layer_update through
custom_check_z4.npz (tests/test_custom_host.py); the decoder as a whole cannot run in the reference,
so its end-to-end parity is against this build's stated definition ("parity unpinned" beyond the
check update)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import code_path, golden

from ldpc_neural_decoder import _native as N
from ldpc_neural_decoder.models import create_custom_minsum_message_gnn_decoder
from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu
TOL = 2e-6


def decoder_for(H, iters):
    dec, conv = create_custom_minsum_message_gnn_decoder(H, num_iterations=iters)
    return dec, conv


def run(dec, llr, cuda):
    with torch.no_grad():
        return dec(llr.to(cuda)).cpu().numpy()


@pytest.mark.parametrize("z,B,iters", [(4, 37, 5), (32, 64, 10), (12, 65, 6), (4, 7, 1), (4, 7, 0)])
def test_custom_minsum_vs_oracle(cuda, oracle_mod, z, B, iters):
    base_file = code_path(z if z in (4, 32) else 32)
    H = expand_base_matrix(load_base_matrix(base_file), z)
    dec, _ = decoder_for(H, iters)
    g = dec._graph(H.shape[1], cuda)
    assert g.N == H.shape[1]
    rng = np.random.default_rng(z)
    llr = rng.normal(1.0, 2.0, (B, H.shape[1])).astype(np.float32)
    llr[0, :40] = 0.0
    llr[1, :20] = -0.0  # the first variable phase turns -0 into +0 as (llr + 0) - 0 does
    got = run(dec, torch.from_numpy(llr), cuda)
    ref = oracle_mod.custom_minsum(oracle_mod.Graph(H.numpy().astype(np.uint8)), llr, iters)
    np.testing.assert_allclose(got, ref, atol=TOL, rtol=0)


def test_check_update_fixture_through_one_iteration(cuda, oracle_mod):
    d = golden("custom_check_z4.npz")
    llr, chk, var = d["llr"], d["msg_chk"], d["msg_var"]
    H = np.zeros((int(chk.max()) + 1, llr.shape[1]), dtype=np.float32)
    H[chk, var] = 1
    dec, _ = decoder_for(torch.from_numpy(H), 1)
    got = run(dec, torch.from_numpy(llr), cuda)
    c2v = d["c2v"]
    out = llr.copy()
    for v in range(llr.shape[1]):
        ms = np.nonzero(var == v)[0]
        s = c2v[:, ms[0]].copy()
        for m in ms[1:]:
            s = (s + c2v[:, m]).astype(np.float32)
        out[:, v] = (out[:, v] + s).astype(np.float32)
    want = (np.float32(1) / (np.float32(1) + np.exp(-out))).astype(np.float32)
    np.testing.assert_allclose(got, want, atol=TOL, rtol=0)


def test_forward_with_ground_truth_and_decode(cuda):
    H = expand_base_matrix(load_base_matrix(code_path(4)), 4)
    dec, _ = decoder_for(H, 4)
    llr = torch.randn(9, H.shape[1], device=cuda) + 2.0
    gt = torch.zeros_like(llr)
    probs, loss = dec(llr, None, None, None, None, ground_truth=gt)
    assert torch.allclose(loss, F.binary_cross_entropy(probs, gt))
    bits = dec.decode(llr)
    assert torch.equal(bits, (probs > 0.5).float())
    # sub-batch invariance: frames are independent
    assert torch.equal(dec(llr[3:7]), probs[3:7])
    assert dec(llr[:0]).shape == (0, H.shape[1])


def test_c_abi_arguments(cuda):
    H = expand_base_matrix(load_base_matrix(code_path(4)), 4)
    dec, _ = decoder_for(H, 2)
    g = dec._graph(H.shape[1], cuda)
    lib = N.lib()
    assert lib.ldpc_custom_minsum_decode(g.handle, None, 4, 2, None, None, 0, None) == N.LDPC_EINVAL
    x = torch.zeros(4, H.shape[1], device=cuda)
    p = torch.empty_like(x)
    assert lib.ldpc_custom_minsum_decode(g.handle, N.ptr(x), 4, 2, N.ptr(p), None, 0, N.stream_ptr(cuda)) == N.LDPC_EINVAL


def _fixture_rows(chk):
    """Row m = [check of m, the check's other messages ascending, m]: the rows
    tests/golden/make_custom_golden.py handed the reference's check_layer_update."""
    E = len(chk)
    ptr = np.concatenate([[0], np.cumsum(np.bincount(chk))])
    width = int((ptr[1:] - ptr[:-1]).max()) + 1
    rows = -np.ones((E, width), dtype=np.int64)
    for m in range(E):
        c = chk[m]
        others = [f for f in range(ptr[c], ptr[c + 1]) if f != m]
        rows[m, 0] = c
        rows[m, 1:1 + len(others)] = others
        rows[m, 1 + len(others)] = m
    return rows


def _literal_check_rows(x, rows):
    """Restatement of check_layer_update's loop (MGD:998-1038) per row: the last assignment
    excludes the last valid entry; torch.sign / prod / min semantics in numpy float32."""
    B = x.shape[0]
    out = np.zeros((B, rows.shape[0]), dtype=np.float32)
    for m, row in enumerate(rows):
        ids = [int(i) for i in row[1:] if i >= 0]
        if len(ids) < 2:
            continue
        others = ids[:-1]
        v = x[:, others]
        sg = np.prod(np.where(v > 0, 1.0, np.where(v < 0, -1.0, 0.0)).astype(np.float32), axis=1).astype(np.float32)
        a = np.abs(v)
        mn = np.where(np.isnan(a).any(axis=1), np.float32(np.nan), np.nanmin(np.where(np.isnan(a), np.inf, a), axis=1))
        out[:, m] = (sg * mn.astype(np.float32)).astype(np.float32)
    return out


def test_check_layer_update_pinned_by_reference(cuda):
    """CustomCheckMessageGNNLayer.check_layer_update on the fixture's rows reproduces the
    reference's own output bit for bit (zeros and their signs included)."""
    from ldpc_neural_decoder.models.custom_decoders import CustomCheckMessageGNNLayer
    d = golden("custom_check_z4.npz")
    llr, chk, var, ref = d["llr"], d["msg_chk"], d["msg_var"], d["c2v"]
    rows = torch.from_numpy(_fixture_rows(chk))
    v2c = torch.from_numpy(llr[:, var]).contiguous()
    layer = CustomCheckMessageGNNLayer(1, 8)
    got = layer.check_layer_update(v2c.to(cuda), torch.zeros(len(chk), dtype=torch.long), rows)
    assert got.device == torch.device(cuda) and got.shape == ref.shape
    g = got.cpu().numpy()
    assert np.array_equal(g.view(np.uint32), ref.view(np.uint32))
    # CPU tensors in, CPU tensor out (the computation still runs on the GPU)
    assert np.array_equal(layer.check_layer_update(v2c, None, rows).numpy().view(np.uint32), ref.view(np.uint32))


def test_check_layer_update_general_rows(cuda):
    """Rows with padding between ids, a repeated id, one or no valid id, NaN / zero inputs, against
    the loop's restatement."""
    from ldpc_neural_decoder.models.custom_decoders import CustomCheckMessageGNNLayer
    rng = np.random.default_rng(5)
    B, E = 9, 40
    x = rng.normal(0, 2, (B, E)).astype(np.float32)
    x[0, 3] = 0.0
    x[1, 7] = -0.0
    x[2, 11] = np.nan
    rows = -np.ones((E, 7), dtype=np.int64)
    for m in range(E):
        k = rng.integers(0, 6)
        ids = rng.choice(E, size=k, replace=True)
        pos = np.sort(rng.choice(np.arange(1, 7), size=k, replace=False))
        rows[m, 0] = rng.integers(0, 10)
        rows[m, pos] = ids
    rows[0, 1:] = [3, 7, 11, -1, 5, -1]
    rows[1, 1:] = [4, -2, 9, -7, 13, -2]  # any negative id is padding (the reference keeps ids >= 0, MGD:1004)
    got =CustomCheckMessageGNNLayer(1, 8).check_layer_update(torch.from_numpy(x).to(cuda), None,
                                                              torch.from_numpy(rows)).cpu().numpy()
    ref = _literal_check_rows(x, rows)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.array_equal(got[ok].view(np.uint32), ref[ok].view(np.uint32))
    with pytest.raises(IndexError):
        bad = rows.copy()
        bad[0, 1] = E
        CustomCheckMessageGNNLayer(1, 8).check_layer_update(torch.from_numpy(x).to(cuda), None, torch.from_numpy(bad))


@pytest.mark.parametrize("iteration", [0, 1])
def test_variable_layer_update(cuda, iteration):
    """CustomVariableMessageGNNLayer.variable_layer_update by its definition (MGD:611-670, per
    frame): (llr + ascending sum of the incoming c2v) - the last one; the LLR alone without ids;
    damping 0.5 / 0.5 with the message's own c2v from iteration 1 on."""
    from ldpc_neural_decoder.models.custom_decoders import CustomVariableMessageGNNLayer
    rng = np.random.default_rng(6 + iteration)
    B, Nv, E = 5, 12, 30
    llr = rng.normal(0, 2, (B, Nv)).astype(np.float32)
    c2v = rng.normal(0, 2, (B, E)).astype(np.float32)
    rows = -np.ones((E, 6), dtype=np.int64)
    for m in range(E):
        k = rng.integers(0, 6)
        rows[m, 0] = rng.integers(0, Nv)
        rows[m, 1:1 + k] = rng.choice(E, size=k, replace=False)
    got = CustomVariableMessageGNNLayer(1, 64).variable_layer_update(
        torch.from_numpy(llr).to(cuda), torch.from_numpy(c2v).to(cuda), torch.from_numpy(rows), iteration)
    f32 = np.float32
    ref = np.zeros((B, E), dtype=np.float32)
    for b in range(B):
        for m in range(E):
            ids = [int(i) for i in rows[m, 1:] if i >= 0]
            v = llr[b, rows[m, 0]]
            if ids:
                s = c2v[b, ids[0]]
                for i in ids[1:]:
                    s = f32(s + c2v[b, i])
                v = f32(f32(v + s) - c2v[b, ids[-1]])
            if iteration > 0:
                v = f32(f32(f32(0.5) * v) + f32(f32(0.5) * c2v[b, m]))
            ref[b, m] = v
    assert np.array_equal(got.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_hybrid_minsum_bench_size(cuda, oracle_mod):
    """The hybrid-minsum-z32 bench shape: B = 65 536 frames, BG2 Z = 32, 10 iterations.  Sub-batches
    decode identically to the same frames of the full batch and four spot frames match the C
    oracle."""
    from ldpc_neural_decoder.utils import awgn_llr
    H = expand_base_matrix(load_base_matrix(code_path(32)), 32)
    dec, _ = decoder_for(H, 10)
    B = 65536
    llr = awgn_llr(B, H.shape[1], 2.0, seed=20251015, device=cuda)
    with torch.no_grad():
        full = dec(llr)
        for s, e in ((0, 3), (40000, 40037), (B - 2, B)):
            assert torch.equal(dec(llr[s:e].contiguous()), full[s:e]), (s, e)
    spots = [0, 1, 40001, B - 1]
    ref = oracle_mod.custom_minsum(oracle_mod.Graph(H.numpy().astype(np.uint8)), llr[spots].cpu().numpy(), 10)
    np.testing.assert_allclose(full[spots].cpu().numpy(), ref, atol=TOL, rtol=0)
