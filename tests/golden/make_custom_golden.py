"""Golden vectors for the hybrid min-sum decoder's check update (CustomMinSum*, MGD:966-1291).

Run ONCE in the build container, where the reference is importable:

    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_custom_golden.py

The reference's Custom* decoders cannot run end to end: their update loops index
per-node tensors as if they were per-message.  CustomCheckMessageGNNLayer.check_layer_update
(message_gnn_decoder.py:976-1044) does run, though, when it is handed the per-message rows its loop
reads -- row m = [check of m, the check's other messages ascending, m itself]: the loop overwrites
c2v[:, m] for every listed message and keeps the last one, which then excludes m's own input, i.e.
the extrinsic min-sum update this build defines for the decoder.  This script records that output
for seeded inputs (with exact zeros for torch.sign(0) = 0) on BG2 Z = 4, as plain arrays:

  custom_check_z4.npz   llr (B, N) f32; msg_chk, msg_var (E,) int32 check-major message list;
                        c2v (B, E) f32 = check_layer_update(llr[:, msg_var]) from the reference;
                        sd_keys / sd_numel: CustomMinSumMessageGNNDecoder(E, 3, 8, 1, 2, 0.0)'s
                        state_dict layout (numel, 0 for scalars; its constructor runs, its factory does not);
                        sdv_keys / sdv_numel: the same for CustomVariableMessageGNNDecoder(E, 3, 64, 1, 3).
"""
import contextlib
import io
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("LDPC_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

from ldpc_neural_decoder.utils.ldpc_utils import load_base_matrix, expand_base_matrix  # noqa: E402
from ldpc_neural_decoder.models.message_gnn_decoder import (  # noqa: E402
    CustomCheckMessageGNNLayer, CustomMinSumMessageGNNDecoder, CustomVariableMessageGNNDecoder)


def main():
    z = 4
    base = load_base_matrix(os.path.join(REF, "5G LDPC CODES", f"NR_2_0_{z}.txt"))
    H = expand_base_matrix(base, z).numpy().astype(np.uint8)
    M, N = H.shape
    msg_chk, msg_var = [], []
    for c in range(M):
        for v in np.nonzero(H[c])[0]:
            msg_chk.append(c)
            msg_var.append(int(v))
    msg_chk = np.array(msg_chk, dtype=np.int32)
    msg_var = np.array(msg_var, dtype=np.int32)
    E = len(msg_chk)
    ptr = np.zeros(M + 1, dtype=np.int64)
    np.add.at(ptr, msg_chk + 1, 1)
    ptr = np.cumsum(ptr)
    width = int((ptr[1:] - ptr[:-1]).max()) + 1
    rows = -np.ones((E, width), dtype=np.int64)
    for m in range(E):
        c = msg_chk[m]
        others = [f for f in range(ptr[c], ptr[c + 1]) if f != m]
        rows[m, 0] = c
        rows[m, 1:1 + len(others)] = others
        rows[m, 1 + len(others)] = m  # own message last: the loop keeps the last assignment

    torch.manual_seed(4242)
    B = 8
    llr = (torch.randn(B, N) * 2.0 + 1.0).float()
    llr[0, :5] = 0.0           # torch.sign(0) = 0 inside a check
    llr[1, 7] = -0.0
    llr[2, ::3] = 0.0
    layer = CustomCheckMessageGNNLayer(1, 8)
    v2c = llr[:, torch.from_numpy(msg_var).long()].contiguous()
    with contextlib.redirect_stdout(io.StringIO()):  # the reference prints per call
        c2v = layer.check_layer_update(v2c, torch.zeros(E, dtype=torch.long), torch.from_numpy(rows))
    sd = CustomMinSumMessageGNNDecoder(E, 3, 8, 1, 2, 0.0).state_dict()
    keys = sorted(sd)
    shapes = np.array([len(sd[k].shape) and int(np.prod(sd[k].shape)) for k in keys], dtype=np.int64)
    sdv = CustomVariableMessageGNNDecoder(E, 3, 64, 1, 3).state_dict()
    vkeys = sorted(sdv)
    vshapes = np.array([len(sdv[k].shape) and int(np.prod(sdv[k].shape)) for k in vkeys], dtype=np.int64)
    np.savez(os.path.join(HERE, "custom_check_z4.npz"), llr=llr.numpy(), msg_chk=msg_chk, msg_var=msg_var,
             c2v=c2v.detach().numpy().astype(np.float32), sd_keys=np.array(keys), sd_numel=shapes,
             sdv_keys=np.array(vkeys), sdv_numel=vshapes)
    print("custom_check_z4.npz", E, "messages", B, "frames")


if __name__ == "__main__":
    main()
