"""On-device channel (Philox + QPSK/AWGN/demod) and BER/FER counters (GPU).

Parity with the reference channel (utils/channel.py:4-154) is statistical: the reference draws
from torch's CPU mt19937, this build from Philox-4x32-10.  Pinned here: the raw Philox stream
(bit-exact vs the oracle's Random123 restatement), the LLR distribution N(sqrt2*snr, 2*snr) of
the reference formula, determinism and shard-independence."""
import numpy as np
import pytest
import torch

from ldpc_neural_decoder import _native as N
from ldpc_neural_decoder.utils import awgn_llr, compute_ber_fer, count_errors, qpsk_demodulate, qpsk_modulate

pytestmark = pytest.mark.gpu


def test_philox_stream_bitexact(cuda, oracle_mod):
    n = 4096
    out = torch.empty(4 * n, dtype=torch.int32, device=cuda)
    seed = 0x1234_5678_9ABC_DEF0
    N.check(N.lib().ldpc_philox_raw(seed, 7, 9, n, N.ptr(out), N.stream_ptr(cuda)))
    ctr = np.stack([np.arange(n, dtype=np.uint32), np.zeros(n, np.uint32),
                    np.full(n, 7, np.uint32), np.full(n, 9, np.uint32)], 1)
    ref = oracle_mod.philox4x32_10(ctr, [seed & 0xFFFFFFFF, seed >> 32])
    assert np.array_equal(out.cpu().numpy().view(np.uint32).reshape(n, 4), ref)


@pytest.mark.parametrize("snr_db", [-2.0, 0.0, 3.0, 6.0])
def test_llr_statistics(cuda, snr_db):
    B, n = 4096, 1664
    llr = awgn_llr(B, n, snr_db, seed=99, device=cuda).double()
    s = 10 ** (snr_db / 10)
    mean, var = llr.mean().item(), llr.var().item()
    # LLR = 2 s (1/sqrt2 + n), n ~ N(0, 1/(2 s))  ->  mean sqrt2 s, var 2 s
    assert abs(mean - np.sqrt(2) * s) < 5e-3 * max(1.0, np.sqrt(2) * s)
    assert abs(var / (2 * s) - 1) < 5e-3
    # I and Q components are independent (correlation of adjacent bits ~ 0)
    x = llr.view(B, n // 2, 2)
    c = torch.corrcoef(torch.stack([x[..., 0].reshape(-1), x[..., 1].reshape(-1)]))[0, 1].item()
    assert abs(c) < 5e-3


def test_deterministic_and_shard_independent(cuda):
    a = awgn_llr(300, 208, 1.0, seed=5, device=cuda)
    b = awgn_llr(300, 208, 1.0, seed=5, device=cuda)
    assert torch.equal(a, b)
    part = awgn_llr(100, 208, 1.0, seed=5, frame_offset=150, device=cuda)
    assert torch.equal(a[150:250], part)
    c = awgn_llr(300, 208, 1.0, seed=6, device=cuda)
    assert not torch.equal(a, c)


def test_transmitted_bits_and_bpsk(cuda):
    bits = (torch.rand(64, 210, device=cuda) > 0.5).to(torch.uint8)
    llr = awgn_llr(64, 210, 30.0, seed=1, bits=bits)  # ~noise-free
    assert torch.equal((llr < 0).to(torch.uint8), bits)
    llr_b = awgn_llr(64, 210, 30.0, seed=1, bits=bits, bpsk=True)
    assert torch.equal((llr_b < 0).to(torch.uint8), bits)
    s = 10 ** 3.0
    np.testing.assert_allclose(llr_b.abs().mean().item(), 2 * s, rtol=1e-2)


def test_reference_api_functions(cuda):
    """qpsk_modulate / qpsk_demodulate keep the reference formulas (vectorised)."""
    bits = torch.tensor([[0, 1, 1, 0, 1]], dtype=torch.float32, device=cuda)
    sym = qpsk_modulate(bits)
    r2 = 1 / np.sqrt(2)
    want = torch.tensor([[complex(r2, -r2), complex(-r2, r2), complex(-r2, r2)]], dtype=torch.complex64)
    torch.testing.assert_close(sym.cpu(), want)
    llr = qpsk_demodulate(sym, 3.0)
    assert llr.shape == (1, 6)
    s = 10 ** 0.3
    torch.testing.assert_close(llr.cpu()[0, :2], torch.tensor([2 * r2 * s, -2 * r2 * s], dtype=torch.float32))


def test_count_errors_and_ber_fer(cuda):
    dec = torch.zeros(10, 50, device=cuda)
    dec[1, 3] = 1
    dec[4, :5] = 1
    c = count_errors(dec)
    assert c.tolist()[:3] == [6, 2, 10]
    tx = torch.zeros(10, 50)
    ber, fer = compute_ber_fer(tx, dec.cpu())
    assert abs(ber - 6 / 500) < 1e-12 and abs(fer - 0.2) < 1e-12
    ref = torch.ones(10, 50, dtype=torch.uint8, device=cuda)
    c2 = count_errors(dec.to(torch.uint8), ref=ref)
    assert c2.tolist()[:3] == [494, 10, 10]


@pytest.mark.parametrize("bpsk", [False, True])
def test_fused_channel_vs_restatement(cuda, oracle_mod, bpsk):
    """The fused kernel's Philox -> Box-Muller -> LLR arithmetic against oracle.awgn_llr (float64
    numpy on the same Philox words).  Tolerance (stated): the kernel uses float32 logf / sincosf /
    sqrtf and rounds every step to float32, so |d| <= 1e-5 |llr| + 2e-5 * 2 snr."""
    B, n, snr_db, seed, off = 7, 1666, 1.5, 0x0BAD_5EED_1234_5678, 123_456_789_012
    bits = (torch.rand(B, n, generator=torch.Generator().manual_seed(2)) > 0.5).to(torch.uint8)
    for tx in (None, bits):
        got = awgn_llr(B, n, snr_db, seed=seed, frame_offset=off, bits=None if tx is None else tx.to(cuda),
                       bpsk=bpsk, device=cuda).double().cpu().numpy()
        want = oracle_mod.awgn_llr(B, n, snr_db, seed, off, None if tx is None else tx.numpy(), bpsk)
        s = 10 ** (snr_db / 10)
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=2e-5 * 2 * s)
