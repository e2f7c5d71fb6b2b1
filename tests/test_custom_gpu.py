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
