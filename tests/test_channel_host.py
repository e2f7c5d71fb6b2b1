"""The reference-API channel functions on the CPU, pinned bit-exactly to the reference's own
seeded outputs (no GPU).

tests/golden/channel_z{4,32}.npz hold the LLRs that the reference's
qpsk_modulate -> awgn_channel -> qpsk_demodulate chain (utils/channel.py:4-154) produced under
torch.manual_seed(1000 + i) at SNR i (tests/golden/make_golden.py:53-58, :83-86).  This build's
functions keep the reference's float32 operation sequence and its noise draw order (real part,
then imaginary part, from torch.randn on the input's device), so on the CPU they must reproduce
those LLRs bit for bit.  Bar: exact equality (integer-like reproducibility of one RNG stream)."""
import numpy as np
import pytest
import torch

from conftest import golden

from ldpc_neural_decoder.utils import awgn_channel, qpsk_demodulate, qpsk_modulate


@pytest.mark.parametrize("z", [4, 32])
def test_reference_channel_chain_bitexact(z):
    f = golden(f"channel_z{z}.npz")
    snrs, seeds, want = f["snrs"], f["seeds"], f["llrs"]
    B, n = want.shape[1:]
    for i, (snr, seed) in enumerate(zip(snrs.tolist(), seeds.tolist())):
        torch.manual_seed(int(seed))
        bits = torch.zeros((B, n))
        llr = qpsk_demodulate(awgn_channel(qpsk_modulate(bits), snr), snr).view(B, -1)
        assert llr.dtype == torch.float32 and llr.shape == (B, n)
        assert np.array_equal(llr.numpy(), want[i]), f"z={z} snr={snr}: max |d| " \
            f"{np.abs(llr.numpy() - want[i]).max()}"


def test_reference_channel_unbatched_and_odd_length():
    """1-D inputs keep the reference's shape rules (channel.py:18-29, :55-58, :148-152) and an odd
    bit count gets the +1/sqrt2 pad symbol (channel.py:42-43)."""
    bits = torch.tensor([0.0, 1.0, 1.0])
    sym = qpsk_modulate(bits)
    r2 = np.float32(1 / np.sqrt(2))
    assert sym.shape == (2,)
    assert sym[1].real.item() == -r2 and sym[1].imag.item() == r2
    torch.manual_seed(3)
    rx = awgn_channel(sym, 2.0)
    llr = qpsk_demodulate(rx, 2.0)
    assert llr.shape == (4,)
    snr = 10 ** 0.2
    np.testing.assert_array_equal(llr[0::2].numpy(), (2 * rx.real / (1 / snr)).numpy())
