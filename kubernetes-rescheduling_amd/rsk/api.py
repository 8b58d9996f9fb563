"""Array-level API over librsk.so (numpy host arrays or device tensors).

Every function mirrors one entry point of include/rsk.h.  Host numpy arrays go
through the synchronous host-pointer path; pass ``device=True`` with device
tensors (anything exposing ``data_ptr()``) for the asynchronous HBM path on the
context's stream.  Layouts are the batched ABI's: per-scenario arrays are
scenario-minor, ``x[i*S + s]``.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ._lib import (RSK_F_DEVICE, RSK_F_TILED, Context, check, default_context, load_library, ptr)

_I32 = np.int32


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _flags(device: bool) -> int:
    return RSK_F_DEVICE if device else 0


class CarPlan:
    """A relation CSR uploaded once and binned by degree (rsk_car_plan_*).

    ``rows`` are the moving pods (default: every pod).  ``execute`` scores one
    batch of S scenarios; results are ``target[i*S + s]`` for ``rows[i]``.
    """

    def __init__(self, row_ptr, col_idx, rows=None, ctx: Optional[Context] = None):
        self.ctx = ctx or default_context()
        self.row_ptr = _c(row_ptr, _I32)
        self.col_idx = _c(col_idx, _I32) if len(col_idx) else np.zeros(1, _I32)
        self.P = int(self.row_ptr.shape[0] - 1)
        self.rows = None if rows is None else _c(rows, _I32)
        self.Q = self.P if rows is None else int(self.rows.shape[0])
        import ctypes as C
        h = C.c_void_p()
        check(self.ctx.lib.rsk_car_plan_create(self.ctx.handle, ptr(self.row_ptr), ptr(self.col_idx), self.P,
                                               ptr(self.rows), self.Q, C.byref(h)))
        self.handle = h

    INFO_FIELDS = ("tile_rows", "direct_rows", "mid_rows", "heavy_rows", "tiles", "tile_image_rows",
                   "tile_pods", "tile_bytes", "direct_bytes", "mid_bytes", "heavy_bytes", "max_degree",
                   "image_rows_total", "image_pods_distinct", "sorted_rows", "side_rows", "side_bytes",
                   "light_max", "tile_rows_lean", "tiles_lean", "fused_side_rows", "fused_nb_pods_distinct",
                   "nb_pods_distinct")

    def info(self) -> dict:
        """How the plan routed its rows (rsk_car_plan_info)."""
        out = np.zeros(len(self.INFO_FIELDS), np.int64)
        n = self.ctx.lib.rsk_car_plan_info(self.handle, ptr(out), len(out))
        return {k: int(v) for k, v in zip(self.INFO_FIELDS[:n], out[:n])}

    def close(self):
        if getattr(self, "handle", None):
            self.ctx.lib.rsk_car_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def execute(self, assign, S, cap_cpu, use_cpu, hazard, N, out_target=None, out_score=None,
                device: bool = False, want_score: bool = False, tiled: bool = False):
        """tiled: the tile / side kernels even for a small batch (RSK_F_TILED)."""
        fl = RSK_F_TILED if tiled else 0
        if device:
            check(self.ctx.lib.rsk_car_plan_execute(self.handle, ptr(assign), S, ptr(cap_cpu), ptr(use_cpu),
                                                    ptr(hazard), N, ptr(out_target), ptr(out_score),
                                                    RSK_F_DEVICE | fl))
            return out_target, out_score
        assign, cap_cpu, use_cpu = _c(assign, _I32), _c(cap_cpu, _I32), _c(use_cpu, _I32)
        hazard = _c(hazard, np.uint8)
        if assign.size != self.P * S or cap_cpu.size != N or use_cpu.size != N * S or hazard.size != N * S:
            raise ValueError("array sizes do not match P, N, S")
        tgt = np.empty(self.Q * S, _I32) if out_target is None else out_target
        sc = (np.empty(self.Q * S, _I32) if out_score is None else out_score) if (want_score or out_score is not None) else None
        check(self.ctx.lib.rsk_car_plan_execute(self.handle, ptr(assign), S, ptr(cap_cpu), ptr(use_cpu), ptr(hazard),
                                                N, ptr(tgt), ptr(sc), fl), allow_no_candidate=True)
        return tgt, sc


def car_place(row_ptr, col_idx, assign, S, cap_cpu, use_cpu, hazard, N, rows=None, ctx=None, want_score=False,
              tiled=False):
    """One-shot CAR scoring (host arrays): returns (target[Q*S], score or None)."""
    plan = CarPlan(row_ptr, col_idx, rows=rows, ctx=ctx)
    try:
        return plan.execute(assign, S, cap_cpu, use_cpu, hazard, N, want_score=want_score, tiled=tiled)
    finally:
        plan.close()


ROW_MAX_N = 32768


def car_row(node_of, cap_cpu, use_cpu, hazard, N, ctx=None):
    """One CAR placement (S = 1) from the related pods' nodes in one launch
    (rsk_car_row): returns (target, score); target -1 is None, and
    RSK_TARGET_NO_CANDIDATE when every node is hazard."""
    import ctypes as C
    ctx = ctx or default_context()
    nb = _c(node_of, _I32) if len(node_of) else np.zeros(1, _I32)
    cap, use, haz = _c(cap_cpu, _I32), _c(use_cpu, _I32), _c(hazard, np.uint8)
    t, sc = C.c_int32(), C.c_int32()
    check(ctx.lib.rsk_car_row(ctx.handle, ptr(nb), len(node_of), ptr(cap), ptr(use), ptr(haz), N, C.byref(t),
                              C.byref(sc), 0), allow_no_candidate=True)
    return t.value, sc.value


class Rounds:
    """The multi-round detect -> evict -> CAR -> update loop (rsk_rounds_*,
    SURVEY §8f item 1; main.py:55-110 per scenario, the pod's CPU moving with
    it).  ``run`` updates ``assign`` / ``use_cpu`` in place and returns
    (evict[R*S], target[R*S])."""

    def __init__(self, row_ptr, col_idx, pod_cpu, ctx: Optional[Context] = None):
        self.ctx = ctx or default_context()
        rp, pc = _c(row_ptr, _I32), _c(pod_cpu, _I32)
        ci = _c(col_idx, _I32) if len(col_idx) else np.zeros(1, _I32)
        self.P = int(rp.shape[0]) - 1
        if pc.size != self.P:
            raise ValueError("pod_cpu must have P entries")
        import ctypes as C
        h = C.c_void_p()
        check(self.ctx.lib.rsk_rounds_create(self.ctx.handle, ptr(rp), ptr(ci), self.P, ptr(pc), C.byref(h)))
        self.handle = h

    def run(self, assign, S, cap_cpu, use_cpu, N, R, threshold=30, out_evict=None, out_target=None,
            device: bool = False):
        if device:
            check(self.ctx.lib.rsk_rounds_run(self.handle, ptr(assign), S, ptr(cap_cpu), ptr(use_cpu), N, threshold,
                                              R, ptr(out_evict), ptr(out_target), RSK_F_DEVICE))
            return out_evict, out_target
        for a, dt in ((assign, _I32), (use_cpu, _I32)):
            if not (isinstance(a, np.ndarray) and a.dtype == dt and a.flags.c_contiguous):
                raise TypeError("assign and use_cpu are updated in place: pass contiguous int32 numpy arrays")
        cap = _c(cap_cpu, _I32)
        if assign.size != self.P * S or cap.size != N or use_cpu.size != N * S:
            raise ValueError("array sizes do not match P, N, S")
        ev, tg = np.empty(max(R * S, 1), _I32), np.empty(max(R * S, 1), _I32)
        check(self.ctx.lib.rsk_rounds_run(self.handle, ptr(assign), S, ptr(cap), ptr(use_cpu), N, threshold, R,
                                          ptr(ev), ptr(tg), 0))
        return ev[:R * S], tg[:R * S]

    def place(self, assign, S, cap_cpu, use_cpu, hazard, N, evict, out_target=None, device: bool = False):
        """One round's placement step alone (rsk_rounds_place): the CAR target of
        pod evict[s] per scenario, no state update; RSK_TARGET_NO_EVICT (-3)
        where evict[s] < 0."""
        if device:
            check(self.ctx.lib.rsk_rounds_place(self.handle, ptr(assign), S, ptr(cap_cpu), ptr(use_cpu), ptr(hazard), N,
                                                ptr(evict), ptr(out_target), RSK_F_DEVICE))
            return out_target
        a, c, u = _c(assign, _I32), _c(cap_cpu, _I32), _c(use_cpu, _I32)
        h, e = _c(hazard, np.uint8), _c(evict, _I32)
        if a.size != self.P * S or c.size != N or u.size != N * S or h.size != N * S or e.size != S:
            raise ValueError("array sizes do not match P, N, S")
        out = np.empty(S, _I32)
        check(self.ctx.lib.rsk_rounds_place(self.handle, ptr(a), S, ptr(c), ptr(u), ptr(h), N, ptr(e), ptr(out), 0))
        return out

    def close(self):
        if getattr(self, "handle", None):
            self.ctx.lib.rsk_rounds_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def spread_place(pod_count, name_rank, hazard, N, S, ctx=None, out=None, device=False):
    ctx = ctx or default_context()
    if device:
        check(ctx.lib.rsk_spread_place(ctx.handle, ptr(pod_count), ptr(name_rank), ptr(hazard), N, S, ptr(out),
                                       RSK_F_DEVICE))
        return out
    # converted arrays are held in locals: a pointer must not outlive its array
    v, r, h = _c(pod_count, _I32), _c(name_rank, _I32), _c(hazard, np.uint8)
    out = np.empty(S, _I32)
    check(ctx.lib.rsk_spread_place(ctx.handle, ptr(v), ptr(r), ptr(h), N, S, ptr(out), 0), allow_no_candidate=True)
    return out


def binpack_place(cpu_pct, name_rank, hazard, N, S, ctx=None, out=None, device=False):
    ctx = ctx or default_context()
    if device:
        check(ctx.lib.rsk_binpack_place(ctx.handle, ptr(cpu_pct), ptr(name_rank), ptr(hazard), N, S, ptr(out),
                                        RSK_F_DEVICE))
        return out
    v, r, h = _c(cpu_pct, _I32), _c(name_rank, _I32), _c(hazard, np.uint8)
    out = np.empty(S, _I32)
    check(ctx.lib.rsk_binpack_place(ctx.handle, ptr(v), ptr(r), ptr(h), N, S, ptr(out), 0), allow_no_candidate=True)
    return out


def random_candidates(hazard, N, ctx=None):
    """random's candidate list in one launch (rsk_random_candidates, S = 1):
    the non-hazard node indices in index order (rescheduling.py:149-150)."""
    import ctypes as C
    ctx = ctx or default_context()
    h = _c(hazard, np.uint8)
    out = np.empty(max(N, 1), _I32)
    cnt = C.c_int32(0)
    check(ctx.lib.rsk_random_candidates(ctx.handle, ptr(h), N, ptr(out), C.byref(cnt)))
    return out[:cnt.value]


def random_count(hazard, N, S, ctx=None):
    ctx = ctx or default_context()
    h = _c(hazard, np.uint8)
    out = np.empty(S, _I32)
    check(ctx.lib.rsk_random_count(ctx.handle, ptr(h), N, S, ptr(out), 0))
    return out


def random_select(hazard, N, S, r, ctx=None):
    ctx = ctx or default_context()
    h, rr = _c(hazard, np.uint8), _c(r, _I32)
    out = np.empty(S, _I32)
    check(ctx.lib.rsk_random_select(ctx.handle, ptr(h), N, S, ptr(rr), ptr(out), 0), allow_no_candidate=True)
    return out


def random_place(hazard, N, S, seeds, ctx=None):
    ctx = ctx or default_context()
    h, sd = _c(hazard, np.uint8), _c(seeds, np.uint64)
    out = np.empty(S, _I32)
    check(ctx.lib.rsk_random_place(ctx.handle, ptr(h), N, S, ptr(sd), ptr(out), 0), allow_no_candidate=True)
    return out


def py_randbelow(seed: int, n: int) -> int:
    """CPython ``random.Random(seed)._randbelow(n)`` from librsk's host MT19937 (no GPU)."""
    return int(load_library().rsk_py_randbelow(seed, n))


def node_reduce(assign, P, S, pod_cpu, pod_mem, N, ctx=None):
    ctx = ctx or default_context()
    a, c = _c(assign, _I32), _c(pod_cpu, _I32)
    m = None if pod_mem is None else _c(pod_mem, np.int64)
    cnt = np.empty(N * S, _I32)
    cpu = np.empty(N * S, np.int64)
    mem = np.empty(N * S, np.int64) if m is not None else None
    check(ctx.lib.rsk_node_reduce(ctx.handle, ptr(a), P, S, ptr(c), ptr(m), N, ptr(cnt), ptr(cpu), ptr(mem), 0))
    return cnt, cpu, mem


def cpu_pct(use_cpu, cap_cpu, N, S, ctx=None):
    ctx = ctx or default_context()
    u, c = _c(use_cpu, _I32), _c(cap_cpu, _I32)
    out = np.empty(N * S, _I32)
    check(ctx.lib.rsk_cpu_pct(ctx.handle, ptr(u), ptr(c), N, S, ptr(out), 0))
    return out


def detect(cpu_pct_arr, N, S, threshold=30, ctx=None):
    ctx = ctx or default_context()
    pc = _c(cpu_pct_arr, _I32)
    haz = np.empty(N * S, np.uint8)
    most = np.empty(S, _I32)
    check(ctx.lib.rsk_detect(ctx.handle, ptr(pc), N, S, threshold, ptr(haz), ptr(most), 0))
    return haz, most


def load_std(use_cpu, cap_cpu, N, S, ctx=None):
    ctx = ctx or default_context()
    u, c = _c(use_cpu, _I32), _c(cap_cpu, _I32)
    out = np.empty(S, np.float64)
    check(ctx.lib.rsk_load_std(ctx.handle, ptr(u), ptr(c), N, S, ptr(out), 0))
    return out


def cut_cost(row_ptr, col_idx, assign, P, S, missing=None, ctx=None):
    """Directed cut count per scenario (the reference reports it / 2)."""
    ctx = ctx or default_context()
    rp = _c(row_ptr, _I32)
    col = _c(col_idx, _I32) if len(col_idx) else np.zeros(1, _I32)
    a = _c(assign, _I32)
    m = None if missing is None else _c(missing, _I32)
    out = np.empty(S, np.int64)
    check(ctx.lib.rsk_cut_cost(ctx.handle, ptr(rp), ptr(col), P, ptr(a), S, ptr(m), ptr(out), 0))
    return out


def cut_cost_rows(row_ptr, col_idx, assign, P, S, r0, r1, missing=None, ctx=None):
    """Directed cut count per scenario over CSR rows [r0, r1) (one rank's
    partial under pod-row sharding); neighbours read from the full assign."""
    ctx = ctx or default_context()
    rp = _c(row_ptr, _I32)
    col = _c(col_idx, _I32) if len(col_idx) else np.zeros(1, _I32)
    a = _c(assign, _I32)
    m = None if missing is None else _c(missing, _I32)
    out = np.empty(S, np.int64)
    check(ctx.lib.rsk_cut_cost_rows(ctx.handle, ptr(rp), ptr(col), P, r0, r1, ptr(a), S, ptr(m), ptr(out), 0))
    return out


def pick_max_pod(assign, pod_cpu, P, S, most, ctx=None):
    ctx = ctx or default_context()
    a, c, m = _c(assign, _I32), _c(pod_cpu, _I32), _c(most, _I32)
    out = np.empty(S, _I32)
    check(ctx.lib.rsk_pick_max_pod(ctx.handle, ptr(a), ptr(c), P, S, ptr(m), ptr(out), 0))
    return out
