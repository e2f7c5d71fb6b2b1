"""ctypes binding of libldpc_amd.so (the C ABI declared in include/ldpc_amd.h).

This is the only door to the compute path.  There is no CPU fallback: if the library is missing
or no HIP device is visible, every decode raises.  Tensors cross the boundary as raw device
pointers (``tensor.data_ptr()``) plus the current HIP stream of torch.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LDPC_AMD_LIB", os.path.join(_HERE, "_lib", "libldpc_amd.so"))

LDPC_ALGO_MINSUM, LDPC_ALGO_BP = 0, 1
LDPC_ES_OFF, LDPC_ES_BATCH, LDPC_ES_FRAME = 0, 1, 2
LDPC_OUT_U8, LDPC_OUT_F32 = 0, 1
LDPC_GNN_EARLY_STOP = 1
LDPC_GNN_FP32_PRODUCTS = 2
LDPC_EINVAL, LDPC_EHIP, LDPC_EUNSUPPORTED, LDPC_ENOMEM = -1, -2, -3, -4

_P = ctypes.c_void_p
_I32, _I64, _U64, _F32 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float

# symbol -> (restype, argtypes); mirrors include/ldpc_amd.h exactly
SIGNATURES = {
    "ldpc_last_error": (ctypes.c_char_p, []),
    "ldpc_version": (ctypes.c_char_p, []),
    "ldpc_graph_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _I64, _P, _P, _P]),
    "ldpc_graph_create_qc": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P]),
    "ldpc_graph_destroy": (ctypes.c_int, [_P]),
    "ldpc_graph_info": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P]),
    "ldpc_graph_edges": (ctypes.c_int, [_P, _P, _P]),
    "ldpc_graph_set_variant": (ctypes.c_int, [_P, ctypes.c_int]),
    "ldpc_flood_workspace_size": (_I64, [_P, _I64, ctypes.c_int, ctypes.c_int]),
    "ldpc_custom_minsum_workspace_size": (_I64, [_P, _I64]),
    "ldpc_gnn_custom_var_workspace_size": (_I64, [_P, ctypes.c_int, ctypes.c_int, _I64, ctypes.c_int]),
    "ldpc_gnn_custom_var_forward": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P,
                                                   ctypes.c_int, _I64, _P, _P, _I64, _P]),
    "ldpc_custom_minsum_decode": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int, _P, _P, _I64, _P]),
    "ldpc_flood_decode": (ctypes.c_int, [_P, ctypes.c_int, _P, _I64, ctypes.c_int, _F32, ctypes.c_int,
                                         ctypes.c_int, _P, _P, _P, _P, _P, _I64, _P]),
    "ldpc_awgn_llr": (ctypes.c_int, [_U64, _U64, _F32, _P, _I64, ctypes.c_int, ctypes.c_int, _P, _P]),
    "ldpc_philox_raw": (ctypes.c_int, [_U64, ctypes.c_uint32, ctypes.c_uint32, _I64, _P, _P]),
    "ldpc_count_errors": (ctypes.c_int, [_P, ctypes.c_int, _P, _I64, ctypes.c_int, _P, _P]),
    "ldpc_gnn_plan_create": (ctypes.c_int, [_I64, ctypes.c_int, _P, ctypes.c_int, _P, _P]),
    "ldpc_gnn_plan_create_csr": (ctypes.c_int, [_I64, _P, _P, _P, _P, _P, _P, _P]),
    "ldpc_gnn_plan_destroy": (ctypes.c_int, [_P]),
    "ldpc_gnn_weights_size": (_I64, [ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "ldpc_gnn_workspace_size": (_I64, [_P, ctypes.c_int, ctypes.c_int, _I64, ctypes.c_int, ctypes.c_int]),
    "ldpc_gnn_forward": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P,
                                        ctypes.c_int, _I64, ctypes.c_int, _P, _P, _I64, _P]),
    "ldpc_gnn_forward_ex": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P,
                                           ctypes.c_int, _I64, ctypes.c_int, ctypes.c_int, _P, _P, _P, _I64, _P]),
    "ldpc_gather_minsum": (ctypes.c_int, [_P, _I64, ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, _P, _P, _P]),
    "ldpc_gather_minsum_backward": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, _P,
                                                   _P, _P]),
    "ldpc_check_groups_minsum": (ctypes.c_int, [_P, _I64, ctypes.c_int, _P, _P, ctypes.c_int, ctypes.c_int, _P, _P]),
    "ldpc_gather_sum": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, _P, _P]),
    "ldpc_var_groups_sum": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int, _P, ctypes.c_int, _P, _P]),
    "ldpc_gather_sum_backward": (ctypes.c_int, [_P, _I64, ctypes.c_int, _P, ctypes.c_int, ctypes.c_int, _P, _P]),
    "ldpc_residual": (ctypes.c_int, [_P, _P, _P, _P, _P, ctypes.c_int, _I64, ctypes.c_int, _P, _P]),
    "ldpc_residual_backward": (ctypes.c_int, [_P, _P, _P, _P, _P, ctypes.c_int, _I64, ctypes.c_int, _P, _P, _P, _P,
                                              _P]),
    "ldpc_output_layer": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int, _P, _P, _P, _P]),
    "ldpc_output_layer_backward": (ctypes.c_int, [_P, _P, _P, _P, _P, _I64, ctypes.c_int, _P, _P]),
    "ldpc_gnn_train_workspace_size": (_I64, [_P, ctypes.c_int, ctypes.c_int, _I64, ctypes.c_int]),
    "ldpc_gnn_forward_train": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P,
                                              ctypes.c_int, _I64, _P, _P, _P, _I64, _P]),
    "ldpc_index_rows_minsum": (ctypes.c_int, [_P, _I64, _I64, _P, _I64, ctypes.c_int, _P, _P]),
    "ldpc_index_rows_varsum": (ctypes.c_int, [_P, _I64, _I64, _P, _I64, _P, _I64, ctypes.c_int, ctypes.c_int, _P,
                                              _P]),
    "ldpc_gnn_backward": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P,
                                         ctypes.c_int, _I64, _P, _P, _P, _P, _P, _I64, _P]),
    "ldpc_gnn_layer_probs": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P,
                                            ctypes.c_int, _I64, _P, _P, _P, _I64, _P]),
    "ldpc_gnn_backward_ds": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P,
                                            ctypes.c_int, _I64, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "ldpc_gnn_train_proj_floats": (_I64, [_P, ctypes.c_int, _I64, ctypes.c_int]),
    "ldpc_gnn_forward_train_ex": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P,
                                                 ctypes.c_int, _I64, _P, _P, _P, _P, _I64, _P]),
    "ldpc_gnn_backward_ds_ex": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P, _P,
                                               ctypes.c_int, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
}

_lib = None
_lock = threading.Lock()


class NativeError(RuntimeError):
    pass


def lib():
    """Load libldpc_amd.so (once).  Raises if it was not built."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise NativeError(
                        f"libldpc_amd.so not found at {LIB_PATH}: build it with "
                        f"`make -C ldpc-neuralnetwork-decoder_amd` (or __graft_entry__.build())")
                handle = ctypes.CDLL(LIB_PATH)
                missing = []
                for name, (res, args) in SIGNATURES.items():
                    try:
                        fn = getattr(handle, name)
                    except AttributeError:
                        # an older build (A/B runs against a previous library): bind what it has,
                        # raise only when the absent entry point is actually called
                        missing.append(name)
                        continue
                    fn.restype = res
                    fn.argtypes = args
                _lib = _Lib(handle, missing)
    return _lib


class _Lib:
    """The loaded library.  Entry points declared in ``SIGNATURES`` that this build lacks raise
    ``NativeError`` when called (not at load time)."""

    def __init__(self, handle, missing):
        self._handle = handle
        self.missing = tuple(missing)
        for name in missing:
            setattr(self, name, _absent(name))

    def __getattr__(self, name):
        return getattr(self._handle, name)


def _absent(name):
    def fn(*_args, **_kw):
        raise NativeError(f"{LIB_PATH} does not export {name} (built from an older source tree?)")
    fn.__name__ = name
    return fn


def check(rc):
    if rc < 0:
        msg = lib().ldpc_last_error().decode(errors="replace")
        raise NativeError(f"libldpc_amd error {rc}: {msg}")
    return rc


def device_of(t=None):
    """The HIP device to run on: the tensor's if it is on one, else the current device."""
    if not torch.cuda.is_available():
        raise NativeError("libldpc_amd needs a HIP device (torch.cuda.is_available() is False); "
                          "there is no CPU fallback")
    if t is not None and t.is_cuda:
        return t.device
    return torch.device("cuda", torch.cuda.current_device())


def stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class NativeGraph:
    """An ldpc_graph* on one device, built from a check-major edge list."""

    def __init__(self, edge_chk, edge_var, M, N, device):
        import numpy as np
        ec = np.ascontiguousarray(edge_chk, dtype=np.int32)
        ev = np.ascontiguousarray(edge_var, dtype=np.int32)
        self.device = device
        self._h = ctypes.c_void_p()
        with torch.cuda.device(device):
            check(lib().ldpc_graph_create(int(M), int(N), len(ec), ec.ctypes.data_as(_P),
                                          ev.ctypes.data_as(_P), ctypes.byref(self._h)))
        vals = [ctypes.c_int(), ctypes.c_int(), ctypes.c_int64(), ctypes.c_int(), ctypes.c_int(),
                ctypes.c_int()]
        check(lib().ldpc_graph_info(self._h, *[ctypes.byref(v) for v in vals]))
        self.M, self.N, self.E, self.Z, self.max_dc, self.max_dv = [v.value for v in vals]

    @property
    def handle(self):
        return self._h

    def set_variant(self, variant):
        """0 = auto (compile-time schedule for the reference's codes), 1 = table-driven.
        Returns the kernel in use: 0 table-driven, 1 BG2 Z=4, 2 BG2 Z=32."""
        return check(lib().ldpc_graph_set_variant(self._h, int(variant)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            try:
                _lib.ldpc_graph_destroy(h)
            except Exception:
                pass


class NativeGnnPlan:
    """An ldpc_gnn_plan* on one device: the variable / check groupings of the E messages (group
    means), or -- ``NativeGnnPlan.csr`` -- two general (E, E) adjacencies in CSR form (weighted
    rows, fp32 forward only)."""

    weighted = False

    def __init__(self, vgroup, n_v, cgroup, n_c, device):
        import numpy as np
        vg = np.ascontiguousarray(vgroup, dtype=np.int32)
        cg = np.ascontiguousarray(cgroup, dtype=np.int32)
        self.E, self.n_v, self.n_c, self.device = len(vg), int(n_v), int(n_c), device
        self._h = ctypes.c_void_p()
        with torch.cuda.device(device):
            check(lib().ldpc_gnn_plan_create(self.E, self.n_v, vg.ctypes.data_as(_P), self.n_c,
                                             cg.ctypes.data_as(_P), ctypes.byref(self._h)))

    @classmethod
    def csr(cls, E, v_csr, c_csr, device):
        """v_csr / c_csr = (ptr (E+1,), col (nnz,), val (nnz,)) numpy arrays."""
        import numpy as np
        self = cls.__new__(cls)
        self.E, self.n_v, self.n_c, self.device, self.weighted = int(E), int(E), int(E), device, True
        arrs = []
        for ptr, col, val in (v_csr, c_csr):
            arrs += [np.ascontiguousarray(ptr, dtype=np.int32), np.ascontiguousarray(col, dtype=np.int32),
                     np.ascontiguousarray(val, dtype=np.float32)]
        self._keep = arrs
        self._h = ctypes.c_void_p()
        with torch.cuda.device(device):
            check(lib().ldpc_gnn_plan_create_csr(self.E, *[a.ctypes.data_as(_P) for a in arrs], ctypes.byref(self._h)))
        return self

    @property
    def handle(self):
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            try:
                _lib.ldpc_gnn_plan_destroy(h)
            except Exception:
                pass
