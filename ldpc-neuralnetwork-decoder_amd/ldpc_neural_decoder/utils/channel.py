"""Channel and error counting (drop-in for the reference's utils/channel.py).

Two layers:
  * ``awgn_llr`` / ``count_errors``: the on-device hot path (fused QPSK + AWGN + demod kernel with
    a Philox counter RNG; integer BER/FER counters), used by the SNR sweep so that frames never
    leave HBM.  They replace the reference's qpsk_modulate -> awgn_channel -> qpsk_demodulate
    chain (channel.py:4-154) and compute_ber_fer (channel.py:156-190).
  * ``qpsk_modulate``, ``awgn_channel``, ``qpsk_demodulate``, ``compute_ber_fer``,
    ``AWGNChannel``: the reference's functions with the same signatures and float32 arithmetic,
    vectorised over the batch (the reference loops over frames in Python) and running on the
    input's device.  They exist so reference call sites keep working; they are not the hot path.
"""
import numpy as np
import torch

from ldpc_neural_decoder import _native as N


# ----------------------------------------------------------------------- reference API
def qpsk_modulate(bits):
    """channel.py:4-60.  0 -> +1/sqrt2, 1 -> -1/sqrt2; I = even bits, Q = odd bits; an odd
    length is padded with +1/sqrt2."""
    is_batched = bits.dim() > 1
    b = bits.reshape(bits.shape[0], -1) if is_batched else bits.reshape(1, -1)
    symbols = 1 / np.sqrt(2) - b.float() * np.sqrt(2)
    if b.shape[1] % 2 == 1:
        pad = torch.full((b.shape[0], 1), 1 / np.sqrt(2), device=b.device, dtype=symbols.dtype)
        symbols = torch.cat([symbols, pad], dim=1)
    out = torch.complex(symbols[:, 0::2].contiguous(), symbols[:, 1::2].contiguous())
    return out if is_batched else out.squeeze(0)


def awgn_channel(symbols, snr_db):
    """channel.py:62-88.  Draws the real part, then the imaginary part, from torch.randn."""
    snr_linear = 10 ** (snr_db / 10)
    noise_power = 1 / snr_linear
    noise_real = torch.randn(symbols.size(), device=symbols.device) * np.sqrt(noise_power / 2)
    noise_imag = torch.randn(symbols.size(), device=symbols.device) * np.sqrt(noise_power / 2)
    return symbols + torch.complex(noise_real, noise_imag)


def qpsk_demodulate(received_symbols, snr_db):
    """channel.py:90-154.  LLR = 2 r / (1/snr) on I and Q, interleaved [I0, Q0, I1, Q1, ...]."""
    is_batched = received_symbols.dim() > 1
    r = received_symbols.reshape(received_symbols.shape[0], -1) if is_batched \
        else received_symbols.reshape(1, -1)
    snr_linear = 10 ** (snr_db / 10)
    noise_var = 1 / snr_linear
    llr_i = 2 * r.real / noise_var
    llr_q = 2 * r.imag / noise_var
    llrs = torch.stack([llr_i, llr_q], dim=2).reshape(r.shape[0], -1)
    return llrs if is_batched else llrs.squeeze(0)


def compute_ber_fer(transmitted_bits, decoded_bits):
    """channel.py:156-190 -> (BER, FER) as Python floats, counted on the GPU."""
    assert transmitted_bits.shape == decoded_bits.shape, \
        "Transmitted and decoded bits must have the same shape"
    tx = transmitted_bits if transmitted_bits.dim() > 1 else transmitted_bits.unsqueeze(0)
    dec = decoded_bits if decoded_bits.dim() > 1 else decoded_bits.unsqueeze(0)
    dev = N.device_of(dec)
    ref = (tx.to(dev) != 0).to(torch.uint8).contiguous()
    c = count_errors(dec.to(dev), ref=ref)
    bit_err, frame_err, frames = (int(x) for x in c.tolist()[:3])
    n = dec.shape[1]
    return bit_err / (frames * n), frame_err / frames


class AWGNChannel:
    """channel.py:193-232 (BPSK).  ``transmit`` keeps the reference's torch.randn semantics;
    ``transmit_device`` is the fused on-device equivalent (Philox)."""

    def __init__(self):
        pass

    def transmit(self, bits, snr_db):
        symbols = 1.0 - 2.0 * bits
        snr_linear = 10 ** (snr_db / 10)
        noise_std = 1.0 / np.sqrt(snr_linear)
        noise = torch.randn_like(symbols) * noise_std
        received_symbols = symbols + noise
        return 2.0 * received_symbols / (noise_std ** 2)

    def transmit_device(self, bits, snr_db, seed=0, frame_offset=0):
        return awgn_llr(bits.shape[0], bits.shape[1], snr_db, seed=seed, frame_offset=frame_offset,
                        bits=bits, bpsk=True)


# ----------------------------------------------------------------------- on-device hot path
def awgn_llr(batch, n, snr_db, seed=0, frame_offset=0, bits=None, bpsk=False, device=None, out=None):
    """Fused transmit -> AWGN -> LLR for `batch` frames of `n` coded bits on the GPU.

    bits=None transmits the all-zero codeword (every reference harness does, e.g.
    comparative_evaluation.py:133).  Frame b draws its noise from Philox(seed) at counter
    (frame_offset + b, symbol), so shards of one sweep use disjoint frame_offset ranges.
    Returns float32 (batch, n).
    """
    dev = N.device_of(bits if bits is not None else out) if device is None else torch.device(device)
    if dev.type != "cuda":
        raise N.NativeError(f"awgn_llr runs on a HIP device, not {dev} (no CPU path)")
    if out is None:
        out = torch.empty((batch, n), dtype=torch.float32, device=dev)
    assert out.shape == (batch, n) and out.dtype == torch.float32 and out.is_contiguous()
    tx = None
    if bits is not None:
        tx = (bits.to(dev) != 0).to(torch.uint8).contiguous()
    N.check(N.lib().ldpc_awgn_llr(int(seed) & 0xFFFFFFFFFFFFFFFF, int(frame_offset), float(snr_db),
                                  N.ptr(tx), int(batch), int(n), 1 if bpsk else 0, N.ptr(out),
                                  N.stream_ptr(dev)))
    return out


def count_errors(bits, ref=None, counters=None):
    """uint64 counters [bit errors, frame errors, frames] (+= if `counters` is given) of hard
    decisions `bits` (B, N) (uint8 or float32) against `ref` (None = all-zero codeword)."""
    dev = N.device_of(bits)
    bits = bits.to(dev)
    if counters is None:
        counters = torch.zeros(4, dtype=torch.int64, device=dev)
    if bits.dtype == torch.float32:
        kind = N.LDPC_OUT_F32
    elif bits.dtype == torch.uint8:
        kind = N.LDPC_OUT_U8
    else:
        bits = (bits != 0).to(torch.uint8)
        kind = N.LDPC_OUT_U8
    bits = bits.contiguous()
    if ref is not None:
        ref = (ref.to(dev) != 0).to(torch.uint8).contiguous()
    if counters.device != dev or counters.dtype != torch.int64 or not counters.is_contiguous():
        raise ValueError("counters must be a contiguous int64 tensor on the bits' HIP device")
    N.check(N.lib().ldpc_count_errors(N.ptr(bits), kind, N.ptr(ref), bits.shape[0], bits.shape[1],
                                      N.ptr(counters), N.stream_ptr(dev)))
    return counters
