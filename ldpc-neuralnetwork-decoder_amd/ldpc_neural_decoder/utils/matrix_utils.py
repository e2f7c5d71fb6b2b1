"""utils/matrix_utils.py of the reference (a duplicate of ldpc_utils' mapping helpers)."""
import torch

from ldpc_neural_decoder.utils.ldpc_utils import get_LLR_indexes  # matrix_utils.py:12-67 (identical)


def create_LLR_mapping(H_T):
    """matrix_utils.py:70-103.  The reference builds the output index with
    torch.tensor([row_indices]) (:101), which raises for any H with more than one nonzero; the
    same error is raised here so that callers see the reference's behaviour.  Use
    ldpc_utils.create_LLR_mapping (:62-95) for the working version."""
    rows = (torch.as_tensor(H_T) == 1).nonzero(as_tuple=True)[0]
    if rows.numel() != 1:
        raise TypeError("only integer tensors of a single element can be converted to an index")
    from ldpc_neural_decoder.utils.ldpc_utils import create_LLR_mapping as _ok
    m, c, v, _ = _ok(H_T)
    return m, c, v, torch.tensor([[int(rows[0])]], dtype=torch.int64)
