"""ctypes binding of librsk.so (include/rsk.h).

This is the only place Python touches the native library.  There is no CPU
fallback: if the library or a gfx950 device is missing, every call raises
:class:`RskError` (``HIP device required``) — the product path never degrades
to host code.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RSK_LIB", os.path.join(HERE, "librsk.so"))

RSK_OK, RSK_NO_CANDIDATE, RSK_EINVAL, RSK_EHIP, RSK_ERCCL = 0, 1, 2, 3, 4
RSK_F_DEVICE = 1
RSK_F_TILED = 4
TARGET_NONE, TARGET_NO_CANDIDATE, TARGET_NO_EVICT = -1, -2, -3

_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)
_f64p = C.POINTER(C.c_double)
_vp = C.c_void_p

# name -> (restype, argtypes); every array argument is passed as c_void_p so the
# same signature carries host (numpy) and device (HBM) pointers.
SIGNATURES = {
    "rsk_version": (C.c_int, []),
    "rsk_check_ws_layout": (C.c_int, [C.c_int32, C.c_int32, C.c_int32]),
    "rsk_last_error": (C.c_char_p, []),
    "rsk_ctx_create": (C.c_int, [C.c_int, C.POINTER(_vp)]),
    "rsk_ctx_destroy": (C.c_int, [_vp]),
    "rsk_ctx_set_stream": (C.c_int, [_vp, _vp]),
    "rsk_ctx_synchronize": (C.c_int, [_vp]),
    "rsk_ctx_set_profiling": (C.c_int, [_vp, C.c_int]),
    "rsk_ctx_kernel_time": (C.c_int, [_vp, C.c_char_p, _f64p, _i64p]),
    "rsk_ctx_reset_profiling": (C.c_int, [_vp]),
    "rsk_ctx_set_profile_only": (C.c_int, [_vp, C.c_char_p]),
    "rsk_car_plan_create": (C.c_int, [_vp, _vp, _vp, C.c_int32, _vp, C.c_int32, C.POINTER(_vp)]),
    "rsk_car_plan_destroy": (C.c_int, [_vp]),
    "rsk_car_plan_info": (C.c_int, [_vp, _vp, C.c_int]),
    "rsk_car_plan_execute": (C.c_int, [_vp, _vp, C.c_int32, _vp, _vp, _vp, C.c_int32, _vp, _vp, C.c_uint32]),
    "rsk_car_place": (C.c_int, [_vp, _vp, _vp, C.c_int32, _vp, C.c_int32, _vp, _vp, _vp, C.c_int32, _vp,
                                C.c_int32, _vp, _vp, C.c_uint32]),
    "rsk_spread_place": (C.c_int, [_vp, _vp, _vp, _vp, C.c_int32, C.c_int32, _vp, C.c_uint32]),
    "rsk_binpack_place": (C.c_int, [_vp, _vp, _vp, _vp, C.c_int32, C.c_int32, _vp, C.c_uint32]),
    "rsk_random_count": (C.c_int, [_vp, _vp, C.c_int32, C.c_int32, _vp, C.c_uint32]),
    "rsk_random_select": (C.c_int, [_vp, _vp, C.c_int32, C.c_int32, _vp, _vp, C.c_uint32]),
    "rsk_random_candidates": (C.c_int, [_vp, _vp, C.c_int32, _vp, _vp]),
    "rsk_random_place": (C.c_int, [_vp, _vp, C.c_int32, C.c_int32, _vp, _vp, C.c_uint32]),
    "rsk_py_randbelow": (C.c_int32, [C.c_uint64, C.c_int32]),
    "rsk_selftest_write_guard": (C.c_int, [_vp]),
    "rsk_node_reduce": (C.c_int, [_vp, _vp, C.c_int32, C.c_int32, _vp, _vp, C.c_int32, _vp, _vp, _vp, C.c_uint32]),
    "rsk_cpu_pct": (C.c_int, [_vp, _vp, _vp, C.c_int32, C.c_int32, _vp, C.c_uint32]),
    "rsk_detect": (C.c_int, [_vp, _vp, C.c_int32, C.c_int32, C.c_int32, _vp, _vp, C.c_uint32]),
    "rsk_load_std": (C.c_int, [_vp, _vp, _vp, C.c_int32, C.c_int32, _vp, C.c_uint32]),
    "rsk_cut_cost": (C.c_int, [_vp, _vp, _vp, C.c_int32, _vp, C.c_int32, _vp, _vp, C.c_uint32]),
    "rsk_rounds_create": (C.c_int, [_vp, _vp, _vp, C.c_int32, _vp, C.POINTER(_vp)]),
    "rsk_rounds_destroy": (C.c_int, [_vp]),
    "rsk_rounds_run": (C.c_int, [_vp, _vp, C.c_int32, _vp, _vp, C.c_int32, C.c_int32, C.c_int32, _vp, _vp,
                                 C.c_uint32]),
    "rsk_pick_max_pod": (C.c_int, [_vp, _vp, _vp, C.c_int32, C.c_int32, _vp, _vp, C.c_uint32]),
    "rsk_cut_cost_rows": (C.c_int, [_vp, _vp, _vp, C.c_int32, C.c_int32, C.c_int32, _vp, C.c_int32, _vp, _vp,
                                    C.c_uint32]),
    "rsk_rounds_place": (C.c_int, [_vp, _vp, C.c_int32, _vp, _vp, _vp, C.c_int32, _vp, _vp, C.c_uint32]),
    "rsk_car_row": (C.c_int, [_vp, _vp, C.c_int32, _vp, _vp, _vp, C.c_int32, _vp, _vp, C.c_uint32]),
    "rsk_rows_evict_key": (C.c_int, [_vp, _vp, C.c_int32, C.c_int32, _vp, _vp, C.c_uint32]),
    "rsk_rows_evict_decode": (C.c_int, [_vp, _vp, C.c_int32, C.c_int32, _vp, C.c_uint32]),
    "rsk_rows_apply": (C.c_int, [_vp, _vp, C.c_int32, _vp, _vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _vp, _vp,
                                 _vp, _vp, _vp, C.c_uint32]),
    "rsk_rows_cut_delta": (C.c_int, [_vp, _vp, _vp, _vp, _vp, C.c_int32, C.c_int32, C.c_int32, _vp, C.c_int32, _vp,
                                     _vp, C.c_int32, _vp, C.c_uint32]),
    "rsk_pick_max_pod16": (C.c_int, [_vp, _vp, _vp, C.c_int32, C.c_int32, _vp, _vp, C.c_uint32]),
    "rsk_rows_pick": (C.c_int, [_vp, _vp, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _vp, _vp, _vp, C.c_uint32]),
    "rsk_rows_place": (C.c_int, [_vp, _vp, C.c_int32, _vp, _vp, _vp, C.c_int32, C.c_int32, C.c_int32, _vp, _vp, _vp,
                                 _vp, _vp, _vp, C.c_uint32]),
    "rsk_rows_move": (C.c_int, [_vp, _vp, _vp, _vp, _vp, C.c_int32, C.c_int32, C.c_int32, _vp, C.c_int32, _vp, _vp,
                                C.c_int32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, C.c_int32, _vp, _vp, _vp, _vp, _vp,
                                C.c_uint32]),
    "rsk_rows_blk_bytes": (C.c_int64, [C.c_int32, C.c_int32]),
    "rsk_rows_detect_setup": (C.c_int, [_vp, _vp, _vp, C.c_int32, C.c_int32, C.c_int32, _vp, _vp, _vp, _vp, _vp,
                                        C.c_uint32]),
    "rsk_workmodel_parse": (C.c_int, [C.c_char_p, C.c_int64, C.POINTER(_vp)]),
    "rsk_workmodel_load": (C.c_int, [C.c_char_p, C.POINTER(_vp)]),
    "rsk_workmodel_sizes": (C.c_int, [_vp, _i32p, _i64p, _i64p]),
    "rsk_workmodel_csr": (C.c_int, [_vp, _vp, _vp]),
    "rsk_workmodel_names": (C.c_int, [_vp, _vp]),
    "rsk_workmodel_destroy": (C.c_int, [_vp]),
    "rsk_parse_quantities": (C.c_int, [_vp, _vp, C.c_int64, C.c_int32, _vp, _vp]),
}


class RskError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"librsk error {code}: {msg}")
        self.code = code


_lib = None
_lib_lock = threading.Lock()


def _prefer_torch_runtime():
    """Load PyTorch's HIP runtime before librsk.so when torch is installed.

    PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64.  If librsk.so were
    loaded first, the process would hold /opt/rocm's runtime too and torch would
    later report "No HIP GPUs are available".  Loading torch first makes librsk's
    libamdhip64.so.7 dependency resolve to the already-loaded runtime, so device
    pointers and streams are shared.  Set RSK_NO_TORCH=1 to skip (no torch in the
    process at all).
    """
    if os.environ.get("RSK_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load_library(path: Optional[str] = None):
    """Load librsk.so and declare every signature.  Loading needs no GPU."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        _prefer_torch_runtime()
        if not os.path.exists(p):
            raise RskError(RSK_EHIP, f"{p} not built (run python __graft_entry__.py build or make -C csrc)")
        lib = C.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib


def last_error() -> str:
    return (load_library().rsk_last_error() or b"").decode(errors="replace")


def check(rc: int, allow_no_candidate: bool = False) -> int:
    if rc == RSK_OK or (allow_no_candidate and rc == RSK_NO_CANDIDATE):
        return rc
    raise RskError(rc, last_error())


def ptr(a) -> Optional[int]:
    """Raw pointer of a numpy array / torch tensor / int (None passes through)."""
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if isinstance(a, np.ndarray):
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        if not a.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return a.data_ptr()
    raise TypeError(f"cannot take a pointer of {type(a).__name__}")


class Context:
    """One device + one stream (rsk_ctx).  Not shareable across threads."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = _vp()
        check(self.lib.rsk_ctx_create(device, C.byref(h)))
        self.handle = h
        self.device = device

    def close(self):
        if getattr(self, "handle", None):
            self.lib.rsk_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def set_stream(self, stream_handle: Optional[int]):
        check(self.lib.rsk_ctx_set_stream(self.handle, stream_handle))

    def synchronize(self):
        check(self.lib.rsk_ctx_synchronize(self.handle))

    def set_profiling(self, on: bool):
        check(self.lib.rsk_ctx_set_profiling(self.handle, int(on)))

    def set_profile_only(self, kernel: str | None):
        """Time only launches of `kernel` (None: every kernel)."""
        check(self.lib.rsk_ctx_set_profile_only(self.handle, kernel.encode() if kernel else None))

    def reset_profiling(self):
        check(self.lib.rsk_ctx_reset_profiling(self.handle))

    def kernel_time(self, name: str):
        ms, n = C.c_double(), C.c_int64()
        check(self.lib.rsk_ctx_kernel_time(self.handle, name.encode(), C.byref(ms), C.byref(n)))
        return ms.value, n.value


_default_ctx: Optional[Context] = None


def default_context() -> Context:
    """Process-wide context on device 0 (LOCAL_RANK under torch.distributed)."""
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(int(os.environ.get("LOCAL_RANK", "0")))
    return _default_ctx
