"""H-matrix loader and lifting (drop-in for utils/ldpc_utils.py:97-147 of the reference).

Setup-time helpers, not the hot path: the decoders turn H into a device-resident graph once
(libldpc_amd's ldpc_graph_create detects the lifting back from H).
"""
import numpy as np
import torch


def load_base_matrix(file_path):
    """utils/ldpc_utils.py:127-147: whitespace-separated numbers, one row per line -> float tensor."""
    with open(file_path, "r") as f:
        rows = [[float(x) for x in line.split()] for line in f.readlines()]
    return torch.tensor(rows)


def expand_base_matrix(base_matrix, Z):
    """utils/ldpc_utils.py:97-125: -1 -> Z x Z zero block, s -> roll(eye(Z), s, dims=1).

    Row k of block (i, j) has its 1 in column (k + s) mod Z.  Returns float32 (rows*Z, cols*Z).
    """
    base = np.asarray(torch.as_tensor(base_matrix).cpu(), dtype=np.float64)
    rows, cols = base.shape
    H = np.zeros((rows * Z, cols * Z), dtype=np.float32)
    r, c = np.nonzero(base != -1)
    k = np.arange(Z)
    for i, j in zip(r, c):
        s = int(base[i, j]) % Z  # torch.roll wraps the shift
        H[i * Z + k, j * Z + (k + s) % Z] = 1.0
    return torch.from_numpy(H)


def edge_list(H):
    """Check-major edge list of a dense H (checks ascending, vars ascending inside a check):
    the order of TannerToMessageGraph.messages (message_gnn_decoder.py:397-406)."""
    Ht = torch.as_tensor(H)
    nz = torch.nonzero(Ht == 1).cpu().numpy()
    return nz[:, 0].astype(np.int32), nz[:, 1].astype(np.int32)
