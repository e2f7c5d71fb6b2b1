"""BP parity statistics for DESIGN.md: bits that differ between the HIP BP decoder and (a) the
reference's golden fixtures (Z=4, 5 iterations, 5 SNRs x 64 frames, early stop off/on), (b) the
C oracle (tanh/atanh in double) on seeded random batches at Z=4 and Z=32.  GPU only."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ldpc-neuralnetwork-decoder_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from ldpc_neural_decoder.models import BeliefPropagationDecoder  # noqa: E402
from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix  # noqa: E402

dev = torch.device("cuda", 0)
G = os.path.join(ROOT, "tests", "golden")
H4 = expand_base_matrix(load_base_matrix(os.path.join(ROOT, "codes", "NR_2_0_4.txt")), 4)
t, ch = np.load(os.path.join(G, "trad_z4.npz")), np.load(os.path.join(G, "channel_z4.npz"))
for es in (0, 1):
    dec = BeliefPropagationDecoder(H4, max_iterations=5, early_stopping=bool(es))
    diff = total = it_ok = 0
    for k in range(ch["llrs"].shape[0]):
        bits, it = dec.decode(torch.from_numpy(ch["llrs"][k]).to(dev))
        ref = t[f"bp_es{es}_bits"][k]
        diff += int((bits.cpu().numpy().astype(np.uint8) != ref).sum())
        total += ref.size
        it_ok += int(it == t[f"bp_es{es}_iters"][k])
    print(f"fixtures Z=4 es={es}: {diff} of {total} bits differ, iteration counts equal {it_ok}/5")
for z, iters in ((4, 5), (32, 10)):
    H = expand_base_matrix(load_base_matrix(os.path.join(ROOT, "codes", f"NR_2_0_{z}.txt")), z)
    g = oracle.Graph(H.numpy())
    rng = np.random.default_rng(11)
    diff = total = 0
    for snr in (-3.0, 0.0, 2.0, 4.0):
        B = 64 if z == 4 else 16
        llr = (rng.normal(1.0, 1.0, size=(B, H.shape[1])) * (2 * 10 ** (snr / 10))).astype(np.float32)
        bits, _ = BeliefPropagationDecoder(H, iters, early_stopping=False).decode(torch.from_numpy(llr).to(dev))
        ref, _, _, _ = oracle.flood_decode(g, llr, "bp", iters, 0.75, 0)
        diff += int((bits.cpu().numpy().astype(np.uint8) != ref).sum())
        total += ref.size
    print(f"oracle Z={z} {iters} it, SNR -3/0/2/4 dB: {diff} of {total} bits differ")
