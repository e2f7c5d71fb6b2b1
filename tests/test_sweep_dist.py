"""Sharded SNR sweep logic on CPU with the gloo backend (world_size 2), no GPU needed.

The decode and channel functions are CPU stand-ins (a hard decision on seeded noise); what is
tested is the harness: trial -> rank assignment, global frame offsets (so shards draw disjoint
channel streams), the single SUM all-reduce of the counter matrix, and that the sharded result
equals the single-process result exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ldpc_neural_decoder.sweep import rates, run_sweep

SNRS = [-2.0, 0.0, 2.0]
B, TRIALS, N_BITS = 8, 5, 64


def llr_fn(b, n, snr, offset):
    # frame f's noise depends only on its global index (offset + row), like the Philox channel
    rows = []
    for f in range(offset, offset + b):
        g = torch.Generator().manual_seed(1000003 * f + int((snr + 10) * 7))
        rows.append(2 * 10 ** (snr / 10) * (1 / np.sqrt(2) + torch.randn(n, generator=g) * np.sqrt(0.5 / 10 ** (snr / 10))))
    return torch.stack(rows).float()


def decode_fn(llr, counters):
    bits = (llr < 0).long()
    be = bits.sum()
    fe = (bits.sum(1) > 0).sum()
    it = torch.tensor(3 * llr.shape[0])  # pretend every frame ran 3 iterations
    counters += torch.stack([be, fe, torch.tensor(llr.shape[0]), it])


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seen = []

    def llr_spy(b, n, snr, off):
        seen.append(off)
        return llr_fn(b, n, snr, off)

    c = run_sweep(decode_fn, llr_spy, SNRS, B, TRIALS, N_BITS, rank, world, "cpu",
                  lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM))
    out[rank] = (c.numpy(), seen)
    dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_sweep_equals_single_process():
    single = run_sweep(decode_fn, llr_fn, SNRS, B, TRIALS, N_BITS).numpy()
    assert single[:, 2].tolist() == [B * TRIALS] * len(SNRS)
    assert single[0, 0] > 0  # -2 dB uncoded: errors present
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, free_port(), out), nprocs=2, join=True)
    for r in (0, 1):
        assert np.array_equal(out[r][0], single)
    # trials dealt round-robin: disjoint frame ranges covering everything
    offs = sorted(out[0][1] + out[1][1])
    assert offs == [(si * TRIALS + t) * B for si in range(len(SNRS)) for t in range(TRIALS)]
    assert not set(out[0][1]) & set(out[1][1])


def test_rates_match_reference_averaging():
    """Mean over trials of per-trial BER/FER == global mean when batches are equal
    (comparative_evaluation.py:157-159)."""
    c = run_sweep(decode_fn, llr_fn, SNRS, B, TRIALS, N_BITS)
    ber, fer, it = rates(c, N_BITS)
    for si, snr in enumerate(SNRS):
        per_trial = []
        for t in range(TRIALS):
            bits = (llr_fn(B, N_BITS, snr, (si * TRIALS + t) * B) < 0).float()
            per_trial.append((bits.mean().item(), (bits.sum(1) > 0).float().mean().item()))
        assert abs(ber[si] - np.mean([p[0] for p in per_trial])) < 1e-12
        assert abs(fer[si] - np.mean([p[1] for p in per_trial])) < 1e-12
        assert it[si] == 3.0
