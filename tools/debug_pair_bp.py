"""Where does the frame-pair kernel's BP first differ from the one-frame fixed kernel?  (debug)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ldpc-neuralnetwork-decoder_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from ldpc_neural_decoder.models import BeliefPropagationDecoder, MinSumScaledDecoder  # noqa: E402
from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix  # noqa: E402

dev = torch.device("cuda", 0)
H = expand_base_matrix(load_base_matrix(os.path.join(ROOT, "codes", "NR_2_0_32.txt")), 32)
d = np.load(os.path.join(ROOT, "tests", "golden", "trad_z32_low.npz"))
llr = torch.from_numpy(d["llrs"].reshape(-1, 1664)).to(dev)
print("llr", tuple(llr.shape), float(llr.abs().min()), float(llr.abs().max()))
for algo in ("bp", "minsum"):
    for it in range(1, 8):
        res = []
        for pair in ("1", "0"):
            os.environ["LDPC_FLOOD_PAIR"] = pair
            dec = BeliefPropagationDecoder(H, it, early_stopping=False) if algo == "bp" else \
                MinSumScaledDecoder(H, it, 0.75, early_stopping=False)
            b, _ = dec.decode(llr)
            res.append(b.cpu().numpy())
        diff = res[0] != res[1]
        fr = np.nonzero(diff.any(1))[0]
        print(algo, "iters", it, "differing bits", int(diff.sum()), "frames", fr[:10].tolist(),
              "cols", np.nonzero(diff.any(0))[0][:12].tolist())
