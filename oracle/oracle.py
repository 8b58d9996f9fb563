"""ctypes binding of the CPU oracle (liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It is the checker for librsk.so, never a fallback for it.  See
rsk_oracle.c for the reference line each function restates; the restatement is
pinned by tests/test_oracle_golden.py against fixtures produced by the reference
itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp, i32 = C.c_void_p, C.c_int32
        L.oracle_car.argtypes = [vp, vp, i32, vp, i32, vp, vp, vp, i32, vp, i32, vp, vp, C.c_int]
        L.oracle_car.restype = C.c_int
        L.oracle_car_sparse.argtypes = L.oracle_car.argtypes
        L.oracle_car_sparse.restype = C.c_int
        for f in (L.oracle_spread, L.oracle_binpack):
            f.argtypes = [vp, vp, vp, i32, i32, vp]
            f.restype = None
        L.oracle_py_randbelow.argtypes = [C.c_uint64, i32]
        L.oracle_py_randbelow.restype = i32
        L.oracle_random.argtypes = [vp, i32, i32, vp, vp, vp]
        L.oracle_random.restype = None
        L.oracle_cpu_pct.argtypes = [vp, vp, i32, i32, vp]
        L.oracle_cpu_pct.restype = None
        L.oracle_detect.argtypes = [vp, i32, i32, i32, vp, vp]
        L.oracle_detect.restype = None
        L.oracle_pick_max_pod.argtypes = [vp, vp, i32, i32, vp, vp]
        L.oracle_pick_max_pod.restype = None
        L.oracle_node_reduce.argtypes = [vp, i32, i32, vp, vp, i32, vp, vp, vp]
        L.oracle_node_reduce.restype = None
        L.oracle_load_std.argtypes = [vp, vp, i32, i32, vp]
        L.oracle_load_std.restype = None
        L.oracle_cut_cost.argtypes = [vp, vp, i32, vp, i32, vp, vp]
        L.oracle_cut_cost.restype = None
        L.oracle_rounds.argtypes = [vp, vp, i32, vp, vp, i32, vp, vp, i32, i32, i32, vp, vp]
        L.oracle_rounds.restype = None
        L.oracle_rounds_par.argtypes = L.oracle_rounds.argtypes + [C.c_int]
        L.oracle_rounds_par.restype = None
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def car(row_ptr, col_idx, assign, S, cap, use, hazard, N, rows=None, threads=1):
    """Literal CAR restatement; returns (target[Q*S], score[Q*S])."""
    row_ptr, col_idx = _c(row_ptr, np.int32), _c(col_idx if len(col_idx) else [0], np.int32)
    P = row_ptr.shape[0] - 1
    rows_a = None if rows is None else _c(rows, np.int32)
    Q = P if rows_a is None else rows_a.shape[0]
    tgt = np.empty(Q * S, np.int32)
    sc = np.empty(Q * S, np.int32)
    assign, cap, use, hazard = _c(assign, np.int32), _c(cap, np.int32), _c(use, np.int32), _c(hazard, np.uint8)
    lib().oracle_car(_p(row_ptr), _p(col_idx), P, _p(assign), S, _p(cap), _p(use), _p(hazard), N, _p(rows_a), Q,
                     _p(tgt), _p(sc), threads)
    return tgt, sc


def car_sparse(row_ptr, col_idx, assign, S, cap, use, hazard, N, rows=None, threads=1, want_score=True):
    """CAR by the sparse restatement (oracle_car_sparse: the row's entries plus a
    per-scenario zero case, the same decisions as `car`); (target[Q*S], score or None)."""
    row_ptr, col_idx = _c(row_ptr, np.int32), _c(col_idx if len(col_idx) else [0], np.int32)
    P = row_ptr.shape[0] - 1
    rows_a = None if rows is None else _c(rows, np.int32)
    Q = P if rows_a is None else rows_a.shape[0]
    tgt = np.empty(Q * S, np.int32)
    sc = np.empty(Q * S, np.int32) if want_score else None
    assign, cap, use, hazard = _c(assign, np.int32), _c(cap, np.int32), _c(use, np.int32), _c(hazard, np.uint8)
    lib().oracle_car_sparse(_p(row_ptr), _p(col_idx), P, _p(assign), S, _p(cap), _p(use), _p(hazard), N, _p(rows_a),
                            Q, _p(tgt), _p(sc), threads)
    return tgt, sc


def spread(pod_count, name_rank, hazard, N, S):
    out = np.empty(S, np.int32)
    a, r, h = _c(pod_count, np.int32), _c(name_rank, np.int32), _c(hazard, np.uint8)
    lib().oracle_spread(_p(a), _p(r), _p(h), N, S, _p(out))
    return out


def binpack(cpu_pct, name_rank, hazard, N, S):
    out = np.empty(S, np.int32)
    a, r, h = _c(cpu_pct, np.int32), _c(name_rank, np.int32), _c(hazard, np.uint8)
    lib().oracle_binpack(_p(a), _p(r), _p(h), N, S, _p(out))
    return out


def py_randbelow(seed, n):
    return int(lib().oracle_py_randbelow(seed, n))


def random(hazard, N, S, seeds):
    out = np.empty(S, np.int32)
    cnt = np.empty(S, np.int32)
    h, sd = _c(hazard, np.uint8), _c(seeds, np.uint64)
    lib().oracle_random(_p(h), N, S, _p(sd), _p(out), _p(cnt))
    return out, cnt


def cpu_pct(use, cap, N, S):
    out = np.empty(N * S, np.int32)
    u, c = _c(use, np.int32), _c(cap, np.int32)
    lib().oracle_cpu_pct(_p(u), _p(c), N, S, _p(out))
    return out


def detect(pct, N, S, threshold=30):
    haz = np.empty(N * S, np.uint8)
    most = np.empty(S, np.int32)
    pc = _c(pct, np.int32)
    lib().oracle_detect(_p(pc), N, S, threshold, _p(haz), _p(most))
    return haz, most


def pick_max_pod(assign, pod_cpu, P, S, most):
    out = np.empty(S, np.int32)
    a, c, m = _c(assign, np.int32), _c(pod_cpu, np.int32), _c(most, np.int32)
    lib().oracle_pick_max_pod(_p(a), _p(c), P, S, _p(m), _p(out))
    return out


def node_reduce(assign, P, S, pod_cpu, pod_mem, N):
    cnt = np.empty(N * S, np.int32)
    cpu = np.empty(N * S, np.int64)
    mem = np.empty(N * S, np.int64)
    a, c, m = _c(assign, np.int32), _c(pod_cpu, np.int32), _c(pod_mem, np.int64)
    lib().oracle_node_reduce(_p(a), P, S, _p(c), _p(m), N, _p(cnt), _p(cpu), _p(mem))
    return cnt, cpu, mem


def load_std(use, cap, N, S):
    out = np.empty(S, np.float64)
    u, c = _c(use, np.int32), _c(cap, np.int32)
    lib().oracle_load_std(_p(u), _p(c), N, S, _p(out))
    return out


def cut_cost(row_ptr, col_idx, assign, P, S, missing=None):
    out = np.empty(S, np.int64)
    rp, ci = _c(row_ptr, np.int32), _c(col_idx if len(col_idx) else [0], np.int32)
    a, m = _c(assign, np.int32), (None if missing is None else _c(missing, np.int32))
    lib().oracle_cut_cost(_p(rp), _p(ci), P, _p(a), S, _p(m), _p(out))
    return out


def dedup_csr(row_ptr, col_idx):
    """Rows as sets without the self edge (relation lists never double count,
    rescheduling.py:193; the evicted pod is off the cluster, main.py:73)."""
    rp, ci = [0], []
    for p in range(len(row_ptr) - 1):
        nb = sorted(set(int(q) for q in col_idx[row_ptr[p]:row_ptr[p + 1]]) - {p})
        ci += nb
        rp.append(len(ci))
    return np.array(rp, np.int32), np.array(ci if ci else [0], np.int32)


def dedup_csr_fast(row_ptr, col_idx):
    """dedup_csr in numpy (same rows: sorted, unique, no self edge), for graphs
    of 10^5-10^6 rows."""
    rp = np.asarray(row_ptr, np.int64)
    ci = np.asarray(col_idx[:rp[-1]], np.int64)
    P = len(rp) - 1
    row = np.repeat(np.arange(P, dtype=np.int64), np.diff(rp))
    key = np.unique(row * (P + 1) + ci)
    r, q = key // (P + 1), key % (P + 1)
    keep = r != q
    r, q = r[keep], q[keep]
    out_rp = np.zeros(P + 1, np.int32)
    np.cumsum(np.bincount(r, minlength=P), out=out_rp[1:])
    return out_rp, (q.astype(np.int32) if q.size else np.zeros(1, np.int32))


def rounds(row_ptr, col_idx, pod_cpu, assign, S, cap, use, N, R, threshold=30, threads=0):
    """The multi-round loop (oracle_rounds); returns (assign', use', evict[R*S], target[R*S]).
    threads > 0: oracle_rounds_par, the scenarios split over that many threads."""
    rp, ci = dedup_csr_fast(row_ptr, col_idx) if threads else dedup_csr(row_ptr, col_idx)
    P = len(rp) - 1
    a, u = np.array(assign, np.int32).copy(), np.array(use, np.int32).copy()
    pc, c = _c(pod_cpu, np.int32), _c(cap, np.int32)
    ev, tg = np.empty(max(R * S, 1), np.int32), np.empty(max(R * S, 1), np.int32)
    if threads:
        lib().oracle_rounds_par(_p(rp), _p(ci), P, _p(pc), _p(a), S, _p(c), _p(u), N, threshold, R, _p(ev), _p(tg),
                                threads)
    else:
        lib().oracle_rounds(_p(rp), _p(ci), P, _p(pc), _p(a), S, _p(c), _p(u), N, threshold, R, _p(ev), _p(tg))
    return a, u, ev[:R * S], tg[:R * S]
