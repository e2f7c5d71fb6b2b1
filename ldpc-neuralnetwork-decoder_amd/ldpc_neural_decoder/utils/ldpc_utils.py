"""H-matrix loader, lifting and the var-major LLR mapping (drop-in for utils/ldpc_utils.py of the
reference: :5-95 and :97-147).

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


def get_LLR_indexes(H_to_LLR_mapping_T):
    """utils/ldpc_utils.py:5-60: for every LLR index, the other LLR indices of its check (rows of
    the (checks, vars) mapping) and of its variable (columns), in ascending order, -1 padded to
    the longest list.  Vectorised: one stable sort per side instead of Python dict loops."""
    m = np.asarray(torch.as_tensor(H_to_LLR_mapping_T).cpu(), dtype=np.int64)
    E = int((m >= 0).sum())

    def side(mat):
        r, c = np.nonzero(mat >= 0)            # row-major: groups in order, members ascending by column
        ids = mat[r, c]
        groups = np.split(ids, np.cumsum(np.bincount(r, minlength=mat.shape[0]))[:-1])
        K = max((len(gid) - 1 for gid in groups if len(gid)), default=0)
        out = np.full((E, max(K, 0)), -1, dtype=np.int64)
        for gid in groups:
            for a in range(len(gid)):
                nb = np.delete(gid, a)
                out[gid[a], :len(nb)] = nb
        return torch.from_numpy(out)

    return side(m), side(m.T)


def create_LLR_mapping(H_T):
    """utils/ldpc_utils.py:62-95: LLR index i = the i-th nonzero of H_T (variables outer, checks
    inner).  Returns (H_to_LLR_mapping_T (checks, vars) long, check_LLR_matrix, var_LLR_matrix,
    output_index_tensor (1, E) = the variable of every LLR index)."""
    HT = torch.as_tensor(H_T)
    rows, cols = (HT == 1).nonzero(as_tuple=True)
    mapping = torch.full(HT.shape, -1, dtype=torch.long, device=HT.device)
    mapping[rows, cols] = torch.arange(rows.numel(), device=HT.device)
    mapping_T = mapping.T
    check_LLR, var_LLR = get_LLR_indexes(mapping_T)
    return mapping_T, check_LLR, var_LLR, rows.unsqueeze(0)
