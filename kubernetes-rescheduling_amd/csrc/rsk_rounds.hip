// Multi-round rescheduling loop on the device.
//
// The reference's control loop (main.py:55-110) runs, per round: monitor ->
// detection (harzard_detect.py:3-27) -> pod_delete / pick_max_pod
// (delete_replaced_pod.py:41-61) -> edit_cluster (main.py:10-19) -> the
// placement algorithm (here CAR, rescheduling.py:174-218).  It re-measures the
// live cluster every round, so what happens to the state after a move is
// build-defined: the pod's CPU moves with it.  This file runs R
// such rounds for S independent scenarios without a host round trip:
//
//   cpu_pct (a9) + detect (a8) in one pass -> pick_max_pod (a10)   [rsk_metrics.hip]
//   car_move_kernel: CAR of the one evicted pod per scenario (a1/a2), then the
//   update use[old] -= cpu, use[t] += cpu, assign[p] = t when t >= 0.
//
// car_move_kernel: one workgroup per scenario, lanes = the evicted pod's
// neighbours; their nodes counted in an LDS open-addressing hash (node+1
// keys), the max count and the best (rem, -node) reduced with LDS atomics.
// With no neighbour on a candidate node (max score 0) every non-hazard node
// ties: the workgroup scans the N nodes of its scenario.
#include <algorithm>
#include <climits>
#include <cstdio>
#include <vector>

#include "rsk_common.h"
#include "rsk_wave.h"

struct rsk_rounds {
    rsk_ctx *ctx = nullptr;
    int P = 0, dmax = 0;
    rsk::DevBuf row_ptr, col, pod_cpu;
    rsk::DevBuf haz, key_ws;
    rsk::DevBuf gtab;   // global hash work areas (rows whose distinct nodes overflow the LDS)
    // the eviction pick's pod lists (rsk_rounds_run): base node per pod, the
    // pods of each base node (CSR), per scenario the pods off their base node
    rsk::DevBuf lbase, loff, lpod, lcnt, llist;
    rsk::DevBuf blk;   // the persistent loop's per-(scenario, 64-node block) detect maxima
    ~rsk_rounds() {
        blk.release();
        lbase.release();
        loff.release();
        lpod.release();
        lcnt.release();
        llist.release();
        gtab.release();
        row_ptr.release();
        col.release();
        pod_cpu.release();
        haz.release();
        key_ws.release();
    }
};

namespace rsk {
namespace {

constexpr int kMoveThreads = 256;
constexpr int kNoEvict = -3;
constexpr size_t kPersistLdsCols = 39 * 1024;  // LDS per persistent workgroup with the columns (4 per CU)

__global__ __launch_bounds__(256) void fill_i32_kernel(int *__restrict__ out, size_t n, int v) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = v;
}

// Per-scenario lists of the pods off their base node (base = scenario 0's
// node), as entries (its current node; pod, its CPU) stored apart — lnode[],
// the 4-B words the pick scans, and lpc[] (int2), read only for the entries on
// the picked node (round 6: the scan reads 4 B per entry, not 16): every pod that has
// left its base node in scenario s has exactly one entry in list s, holding
// the node it is on now (the move kernel updates it in place, or appends the
// pod when it first leaves its base node).  In the persistent loop a
// workgroup's DevLists is its own scenario's: list = the scenario's entries,
// cnt / src = the list length and the entry the round's pick came from (-1:
// the base list), both in LDS.  cnt > cap: the list overflowed, the scenario
// is scanned in full from then on.
struct DevLists {
    const int *base = nullptr;
    int *cnt = nullptr, *src = nullptr;
    int *lnode = nullptr;   // [S][cap] the entry's current node
    int2 *lpc = nullptr;    // [S][cap] (pod, its CPU)
    int cap = 0;
};

// Per-phase wall clock of the persistent loop (profiling builds only: `make
// variant NAME=rprof DEFS=-DRSK_ROUNDS_PROF`; the product compiles the marks
// out).  Thread 0 of a workgroup reads the 100 MHz real-time counter at each
// phase boundary — after the barrier that ends the phase, so a phase includes
// waiting for the slowest wave — and accumulates the deltas in LDS; the host
// prints the sums per (scenario, round) after the call.
#ifdef RSK_ROUNDS_PROF
constexpr int kRProfPhases = 10;
struct PhaseClock {
    unsigned long long last, acc[kRProfPhases];
    __device__ __forceinline__ void start() { last = __builtin_amdgcn_s_memrealtime(); }
    __device__ __forceinline__ void mark(int k) {
        const unsigned long long n = __builtin_amdgcn_s_memrealtime();
        acc[k] += n - last;
        last = n;
    }
};
#define RPROF_MARK(pc, k) do { if ((pc) && threadIdx.x == 0) (pc)->mark(k); } while (0)
#else
struct PhaseClock {};
#define RPROF_MARK(pc, k) ((void)0)
#endif

__device__ __forceinline__ unsigned long long move_pack(int rem, int n) {  // (rem, -node), 0 = none
    return ((unsigned long long)((unsigned)rem ^ 0x80000000u) << 32) | (unsigned long long)(0x7fffffffu - (unsigned)n);
}

struct ScnState {  // the scenario's detect maxima (LDS)
    unsigned long long most, zkey;
    int zcnt;
};

// A scenario's node state as car_move_one and blk_update read and update it:
// the global [N][S] usage and hazard arrays at scenario s, or (the persistent
// loop) the scenario's own columns in LDS — usage as int[N], hazard as a
// bitset — so the round's dependent reads of a node's state are LDS round trips.
struct NodeGlobal {
    int *use;
    uint8_t *haz;
    int S, s;
    __device__ __forceinline__ int &u(int n) const { return use[(size_t)n * S + s]; }
    __device__ __forceinline__ bool h(int n) const { return haz[(size_t)n * S + s] != 0; }
    __device__ __forceinline__ void set_h(int n, bool v) const { haz[(size_t)n * S + s] = v; }
};
struct NodeCols {
    int *use;       // [N] (LDS)
    unsigned *hb;   // [ceil(N / 32)] hazard bits (LDS)
    __device__ __forceinline__ int &u(int n) const { return use[n]; }
    __device__ __forceinline__ bool h(int n) const { return (hb[n >> 5] >> (n & 31)) & 1u; }
    __device__ __forceinline__ void set_h(int n, bool v) const {
        if (v) atomicOr(&hb[n >> 5], 1u << (n & 31));
        else atomicAnd(&hb[n >> 5], ~(1u << (n & 31)));
    }
};

// One scenario s of car_move_kernel.  tab = the hash (keys[H] | cnts[H] | 8
// reduction words): the workgroup's LDS, or (kGlobal: rows whose distinct
// nodes overflow the LDS) its slot of a global work area, where every switch
// from writing to reading goes through an agent-scope fence (plain loads may
// hit stale L1 lines after atomics performed in L2).
template <bool kGlobal>
__device__ __forceinline__ void move_sync() {
    if (kGlobal) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
    __syncthreads();
}

template <bool kGlobal, class NS>
__device__ __forceinline__ int car_move_one(const int *__restrict__ row_ptr, const int *__restrict__ col,
                                             const int *__restrict__ pod_cpu, int *assign, const NS &ns,
                                             const int *__restrict__ cap,
                                             const int *__restrict__ evict, int s, int S, int N, int H, int update,
                                             int *__restrict__ out_target, unsigned short *__restrict__ asg16,
                                             unsigned *tab, unsigned long long *__restrict__ kpick,
                                             unsigned long long *__restrict__ kdet, int *__restrict__ ev_out,
                                             int *__restrict__ zc_cnt, unsigned long long *__restrict__ zc_key,
                                             int own0, int own1, DevLists dl, int p_direct = -1,
                                             int old_known = INT_MIN, int cpu_known = INT_MIN,
                                             PhaseClock *pc = nullptr, int zs_cnt = -1, unsigned long long zs_key = 0ull) {
    // returns the target to thread 0 (the persistent loop's wave 0 broadcasts it)
    // zs_cnt >= 0 (the persistent loop): the scenario's zero case (count, key)
    // from its LDS detect state instead of the global zc words
    unsigned *keys = tab, *cnts = tab + H;
    unsigned long long *red64 = reinterpret_cast<unsigned long long *>(tab + 2 * H);  // best
    unsigned *red = tab + 2 * H + 2;                                                   // M, n_at_M, n_free
    const int tid = threadIdx.x;
    int p;
    if (kpick) {  // the loop: the pick kernel's packed (cpu, ~pod) key, decoded here
        const unsigned long long k = kpick[s];
        p = k ? (int)(~(unsigned)(k & 0xffffffffull)) : -1;
    } else {
        p = evict ? evict[s] : p_direct;  // (the persistent loop: its pick, in registers)
    }
    if (kpick && tid == 0) ev_out[s] = p;
    if (p < own0 || p >= own1) {  // no eviction, or (row-sharded) another rank's pod
        if (tid == 0) {
            out_target[s] = kNoEvict;
            if (kpick) kpick[s] = kdet[s] = 0ull;  // zeroed for the next round's atomics
            if (zc_cnt) zc_cnt[s] = 0, zc_key[s] = 0ull;
        }
        return kNoEvict;
    }
    const int b = row_ptr[p], d = row_ptr[p + 1] - b;
    // the decision (thread 0): the target from the count of nodes at the max
    // score and the best (rem, -node) among them, then the update
    auto finish = [&](unsigned nbest, unsigned long long best) -> int {
        const int rem = (int)((unsigned)(best >> 32) ^ 0x80000000u);
        const int node = (int)(0x7fffffffu - (unsigned)(best & 0xffffffffu));
        int t;
        if (nbest == 0) t = RSK_TARGET_NO_CANDIDATE;  // max() of an empty sequence
        else if (nbest == 1) t = node;                // the single best, even if overloaded
        else t = rem >= 0 ? node : RSK_TARGET_NONE;   // largest remaining CPU, None if < 0
        out_target[s] = t;
        red[5] = (unsigned)t;  // for the workgroup (the persistent loop), after its next barrier
        red[4] = (unsigned)rem;  // the target's remaining CPU before the move (the loop's detect update)
        if (kpick) kpick[s] = kdet[s] = 0ull;  // every thread read p long before the last barrier
        if (zc_cnt) zc_cnt[s] = 0, zc_key[s] = 0ull;
        if (update && t >= 0) {  // build-defined update: the pod's CPU moves with it
            const size_t pc = (size_t)p * S + s;
            // (the persistent loop knows both: the hazard node and the pick key's CPU)
            const int old = old_known != INT_MIN ? old_known : assign[pc];
            const int c = cpu_known != INT_MIN ? cpu_known : pod_cpu[p];
            if ((unsigned)old < (unsigned)N) ns.u(old) -= c;
            ns.u(t) += c;
            assign[pc] = t;
            if (asg16) asg16[pc] = (unsigned short)t;
            if (dl.base) {  // the pod's entry follows it (one entry per pod off its base node)
                const int j = *dl.src, q = *dl.cnt;
                if (q <= dl.cap) {
                    if (j >= 0) {
                        dl.lnode[j] = t;
                    } else if (q < dl.cap) {
                        dl.lnode[q] = t;
                        dl.lpc[q] = make_int2(p, c);
                        *dl.cnt = q + 1;
                    } else {
                        *dl.cnt = dl.cap + 1;  // overflow: full scans from now on
                    }
                }
            }
        }
        return t;
    };
    const bool have_zc = zs_cnt >= 0 || zc_cnt;  // the zero case comes from detect state (no all-node scan)
    int tgt = kNoEvict;
    // Rows of at most 64 neighbours (a PA tree's pods mostly have 1-3): wave 0
    // alone, lane = neighbour, no hash and no workgroup barrier — each distinct
    // candidate node is counted by one ballot (a loop over the distinct nodes),
    // the max count, the nodes at it and their best (rem, -node) by wave
    // reductions.  Only a row with no neighbour on a candidate node and no
    // zero-case words (car_direct, car_move without the loop's detect state)
    // falls back to the workgroup's scan of every node.
    if (d <= 64) {  // uniform
        if (tid < 64) {
            int x = N;
            if (d > 0) x = assign[(size_t)col[b + min(tid, d - 1)] * S + s];
            const bool inN = (unsigned)x < (unsigned)N;
            const bool v = tid < d && inN && !ns.h(inN ? x : 0);
            int c = 0;
            unsigned long long live = __builtin_amdgcn_ballot_w64(v);
            while (live) {  // uniform: one pass per distinct candidate node
                const int l = __builtin_ctzll(live);
                const int xv = __builtin_amdgcn_readlane(x, l);
                const unsigned long long eq = __builtin_amdgcn_ballot_w64(v && x == xv);
                if (tid == l) c = __popcll(eq);
                live &= ~eq;
            }
            const int M = dpp_max(c);
            unsigned nb = 0;
            unsigned long long best = 0ull;
            if (M > 0) {
                const bool cand = c == M;
                nb = (unsigned)__popcll(__builtin_amdgcn_ballot_w64(cand));
                const int xc = cand ? x : 0;  // (clamped: an always-valid node for every lane's loads)
                const unsigned long long k = move_pack(cap[xc] - ns.u(xc), xc);
                best = dpp_max_u64(cand ? k : 0ull);
            } else if (have_zc) {  // max score 0: the detect state's zero case of the scenario
                const unsigned long long z = zs_cnt >= 0 ? zs_key : zc_key[s];
                nb = zs_cnt >= 0 ? (unsigned)zs_cnt : (unsigned)zc_cnt[s];
                best = nb ? move_pack((int)((unsigned)(z >> 32) ^ 0x80000000u), (int)~(unsigned)(z & 0xffffffffull)) : 0ull;
            }
            if (M > 0 || have_zc) {
                if (tid == 0) tgt = finish(nb, best);
            } else if (tid == 0) {  // the workgroup's scan below
                red[1] = 0u;
                *red64 = 0ull;
            }
            if (!have_zc && tid == 0) red[3] = M == 0;
        }
        if (have_zc) return tgt;  // uniform (the caller publishes red[5] and the update)
        move_sync<kGlobal>();
        if (red[3]) {  // uniform: max score 0 and no zero-case words: every non-hazard node ties
            unsigned long long best = 0;
            unsigned nb = 0;
            for (int n = tid; n < N; n += kMoveThreads) {
                if (ns.h(n)) continue;
                ++nb;
                best = max(best, move_pack(cap[n] - ns.u(n), n));
            }
            if (nb) {
                atomicAdd(&red[1], nb);
                atomicMax(red64, best);
            }
            move_sync<kGlobal>();
            if (tid == 0) tgt = finish(red[1], *red64);
        }
        return tgt;
    }
    for (int k = tid; k < 2 * H; k += kMoveThreads) tab[k] = 0u;
    if (tid < 8) tab[2 * H + tid] = 0u;
    move_sync<kGlobal>();
    RPROF_MARK(pc, 1);
    const unsigned mask = (unsigned)H - 1u;
    // A: count every neighbour on a non-hazard node (kU neighbours per thread
    // in flight: the col, assign and hazard loads of a batch issued together
    // from clamped, always-valid addresses)
    constexpr int kU = 4;
    for (int j0 = tid; j0 < d; j0 += kMoveThreads * kU) {
        int q[kU], x[kU];
        uint8_t hz[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) q[u] = col[b + min(j0 + u * kMoveThreads, d - 1)];
#pragma unroll
        for (int u = 0; u < kU; ++u) x[u] = assign[(size_t)q[u] * S + s];
#pragma unroll
        for (int u = 0; u < kU; ++u) hz[u] = ns.h((int)min((unsigned)x[u], (unsigned)N - 1u));
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (j0 + u * kMoveThreads >= d || (unsigned)x[u] >= (unsigned)N || hz[u]) continue;
            const unsigned k = (unsigned)x[u] + 1u;
            unsigned h = (k * 2654435761u) & mask;
            while (true) {
                const unsigned prev = atomicCAS(&keys[h], 0u, k);
                if (prev == 0u || prev == k) break;
                h = (h + 1u) & mask;
            }
            atomicAdd(&cnts[h], 1u);
        }
    }
    move_sync<kGlobal>();
    RPROF_MARK(pc, 2);
    // B: max count over the slots
    unsigned m = 0;
    for (int h = tid; h < H; h += kMoveThreads) m = max(m, cnts[h]);
    if (m) atomicMax(&red[0], m);
    move_sync<kGlobal>();
    RPROF_MARK(pc, 3);
    const unsigned M = red[0];
    if (M > 0) {  // C: nodes at the max count -> |best| and the best (rem, -node)
        unsigned long long best = 0;
        unsigned nb = 0;
        for (int h = tid; h < H; h += kMoveThreads) {
            if (cnts[h] != M) continue;
            const int n = (int)keys[h] - 1;
            ++nb;
            const unsigned long long k = move_pack(cap[n] - ns.u(n), n);
            best = k > best ? k : best;
        }
        if (nb) {
            atomicAdd(&red[1], nb);
            atomicMax(red64, best);
        }
    } else if (have_zc) {  // max score 0: the detect state's zero case of the scenario
        if (tid == 0) {
            const unsigned long long z = zs_cnt >= 0 ? zs_key : zc_key[s];
            red[1] = zs_cnt >= 0 ? (unsigned)zs_cnt : (unsigned)zc_cnt[s];
            *red64 = red[1] ? move_pack((int)((unsigned)(z >> 32) ^ 0x80000000u), (int)~(unsigned)(z & 0xffffffffull)) : 0ull;
        }
    } else {  // max score 0: every non-hazard node ties
        unsigned long long best = 0;
        unsigned nb = 0;
        for (int n = tid; n < N; n += kMoveThreads) {
            if (ns.h(n)) continue;
            ++nb;
            const unsigned long long k = move_pack(cap[n] - ns.u(n), n);
            best = k > best ? k : best;
        }
        if (nb) {
            atomicAdd(&red[1], nb);
            atomicMax(red64, best);
        }
    }
    move_sync<kGlobal>();
    RPROF_MARK(pc, 4);
    if (tid == 0) tgt = finish(red[1], *red64);
    return tgt;
}

// One workgroup per scenario (LDS hash), or kGlobal: a capped grid striding
// over the scenarios, each workgroup with its own global work area.
template <bool kGlobal>
__global__ __launch_bounds__(kMoveThreads) void car_move_kernel(const int *__restrict__ row_ptr,
                                                                const int *__restrict__ col,
                                                                const int *__restrict__ pod_cpu, int *assign,
                                                                int *use, const int *__restrict__ cap,
                                                                const uint8_t *__restrict__ haz,
                                                                const int *__restrict__ evict, int S, int N, int H,
                                                                int update, int *__restrict__ out_target,
                                                                unsigned short *__restrict__ asg16,
                                                                unsigned *__restrict__ gtab,
                                                                unsigned long long *__restrict__ kpick,
                                                                unsigned long long *__restrict__ kdet,
                                                                int *__restrict__ ev_out, int *__restrict__ zc_cnt,
                                                                unsigned long long *__restrict__ zc_key, int own0,
                                                                int own1, DevLists dl) {
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    unsigned *tab = kGlobal ? gtab + (size_t)blockIdx.x * (size_t)(2 * H + 8) : lds;
    for (int s = (int)blockIdx.x; s < S; s += (int)gridDim.x) {
        car_move_one<kGlobal>(row_ptr, col, pod_cpu, assign, NodeGlobal{use, const_cast<uint8_t *>(haz), S, s}, cap,
                              evict, s, S, N, H, update, out_target,
                              asg16, tab, kpick, kdet, ev_out, zc_cnt, zc_key, own0, own1, dl);
        if (kGlobal) move_sync<true>();  // the area is free before the next scenario clears it
    }
}

int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

// delete_replaced_pod.py:41-61 over the u16 shadow: thread = (chunk of ppt pods,
// 8 consecutive scenarios), one 16-B load per pod; the first max (cpu, -pod)
// among pods on most[s] with cpu > -1, packed as pick_pod_kernel packs it.  Half
// the bytes of the int32 scan (rsk_metrics.hip pick_pod_kernel).
__global__ __launch_bounds__(256) void pick16_kernel(const uint4 *__restrict__ asg, const int *__restrict__ pod_cpu,
                                                      int P, int S8, const int *__restrict__ most, int ppt,
                                                      unsigned total, unsigned long long *__restrict__ best) {
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (t >= total) return;
    const int s8 = (int)(t % (unsigned)S8);
    const int p0 = (int)(t / (unsigned)S8) * ppt, p1 = min(P, p0 + ppt);
    unsigned m[8];
    bool any = false;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int v = most[s8 * 8 + j];
        m[j] = v < 0 ? 0x10000u : (unsigned)v;  // no hazard node: matches nothing
        any |= v >= 0;
    }
    if (!any) return;
    unsigned long long b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int p = p0; p < p1; ++p) {
        const uint4 x = asg[(size_t)p * S8 + s8];
        const unsigned w[4] = {x.x, x.y, x.z, x.w};
        const int c = pod_cpu[p];
        const unsigned long long k = c >= 0 ? ((unsigned long long)((unsigned)c ^ 0x80000000u) << 32) | (unsigned long long)(~(unsigned)p)
                                            : 0ull;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned nd = (w[j >> 1] >> ((j & 1) * 16)) & 0xffffu;
            b[j] = (nd == m[j] && k > b[j]) ? k : b[j];
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (b[j]) atomicMax(&best[s8 * 8 + j], b[j]);
}

struct MoveGeom {
    int H;
    size_t lds;      // LDS bytes (0: the global work area)
    int grid;        // workgroups (kGlobal: capped, striding over the scenarios)
    int rc;
};

// The hash holds the distinct candidate nodes of one row: at most min(dmax, N)
// keys, load <= 1/2.  In the LDS while it fits (any degree when N <= ~10k);
// beyond, in global work areas of at most 256 MiB together.
MoveGeom move_geometry(rsk_rounds *r, int N, int S) {
    MoveGeom g;
    g.H = next_pow2(std::max(2, 2 * std::min(r->dmax, N)));
    const size_t bytes = move_tab_bytes(g.H);
    g.rc = RSK_OK;
    if (bytes <= 160 * 1024) {
        g.lds = bytes;
        g.grid = S;
        if (g.lds > 64 * 1024 &&
            hipFuncSetAttribute(reinterpret_cast<const void *>(&car_move_kernel<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)g.lds) != hipSuccess) {
            set_error("hipFuncSetAttribute failed");
            g.rc = RSK_EHIP;
        }
        return g;
    }
    g.lds = 0;
    g.grid = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)S, 1024, (int64_t)((256u << 20) / bytes)}));
    g.rc = r->gtab.reserve((size_t)g.grid * bytes);
    return g;
}

int launch_move(rsk_rounds *r, hipStream_t st, const MoveGeom &g, int *assign, int *use, const int *cap,
                const uint8_t *haz, const int *evict, int S, int N, int update, int *target, unsigned short *a16,
                unsigned long long *kpick = nullptr, unsigned long long *kdet = nullptr, int *ev_out = nullptr,
                int *zc_cnt = nullptr, unsigned long long *zc_key = nullptr, int own0 = 0, int own1 = INT_MAX,
                DevLists dl = DevLists()) {
    if (g.lds)
        car_move_kernel<false><<<dim3((unsigned)g.grid), dim3(kMoveThreads), g.lds, st>>>(
            r->row_ptr.as<int>(), r->col.as<int>(), r->pod_cpu.as<int>(), assign, use, cap, haz, evict, S, N, g.H,
            update, target, a16, nullptr, kpick, kdet, ev_out, zc_cnt, zc_key, own0, own1, dl);
    else
        car_move_kernel<true><<<dim3((unsigned)g.grid), dim3(kMoveThreads), 0, st>>>(
            r->row_ptr.as<int>(), r->col.as<int>(), r->pod_cpu.as<int>(), assign, use, cap, haz, evict, S, N, g.H,
            update, target, a16, r->gtab.as<unsigned>(), kpick, kdet, ev_out, zc_cnt, zc_key, own0, own1, dl);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

// ---- the eviction pick over pod lists (rsk_rounds_run) ----
// setup: base[p] = assign[p, 0] (clamped to N), the base nodes' pod counts
__global__ __launch_bounds__(256) void list_base_kernel(const int *__restrict__ assign, int P, int S, int N,
                                                        int *__restrict__ base, int *__restrict__ cnt) {
    const int p = (int)(blockIdx.x * 256 + threadIdx.x);
    if (p >= P) return;
    const int a = assign[(size_t)p * S];
    const int b = (unsigned)a < (unsigned)N ? a : N;
    base[p] = b;
    atomicAdd(&cnt[b], 1);
}

// exclusive scan of cnt[0..n] into off (one workgroup: setup only)
__global__ __launch_bounds__(1024) void list_scan_kernel(const int *__restrict__ cnt, int n, int *__restrict__ off) {
    __shared__ int part[1024];
    const int t = (int)threadIdx.x, per = (n + 1023) / 1024;
    const int i0 = min(n, t * per), i1 = min(n, i0 + per);
    int sum = 0;
    for (int i = i0; i < i1; ++i) sum += cnt[i];
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int x = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    int run = part[t] - sum;
    for (int i = i0; i < i1; ++i) {
        off[i] = run;
        run += cnt[i];
    }
    if (t == 1023) off[n] = part[1023];
}

// the base nodes' pod lists (cursor = a copy of off) and the scenarios' lists
// of pods off their base node.  Workgroup = (64-scenario chunk, kLF pods), lane
// = scenario, each wave a quarter of the pods: the lanes count their deviating
// pods, one atomic per scenario and workgroup reserves the list slots, then
// the pods (their rows now in L2) are walked again to write the entries.
constexpr int kLF = 1024;
__global__ __launch_bounds__(256) void list_fill_kernel(const int *__restrict__ assign, int P, int S, int N,
                                                        const int *__restrict__ base, int *__restrict__ cur,
                                                        int *__restrict__ pod, int *__restrict__ dcnt,
                                                        const int *__restrict__ pod_cpu, int *__restrict__ lnode,
                                                        int2 *__restrict__ lpc,
                                                        int cap, unsigned *__restrict__ err) {
    constexpr int kK = 16;  // deviations kept per (wave, lane) in LDS; more: the rows are walked again
    __shared__ int wc[4][64];
    __shared__ int2 keep[4][kK][64];
    const int lane = (int)threadIdx.x & 63, wv = (int)threadIdx.x >> 6;
    const int nsc = (S + 63) >> 6;
    const int pg = (int)blockIdx.x / nsc, s = ((int)blockIdx.x - pg * nsc) * 64 + lane;
    const int q0 = pg * kLF + wv * (kLF / 4), q1 = min(P, q0 + kLF / 4);
    const int ss = min(s, S - 1);
    if (s < 64) {  // the base lists: the first scenario chunk's lanes, a pod each
#pragma unroll 4
        for (int p = q0 + lane; p < q1; p += 64) {
            const int pos = atomicAdd(&cur[base[p]], 1);  // from list_scan's offsets: guarded (dev_err)
            if ((unsigned)pos < (unsigned)P) pod[pos] = p;
            else *err = kErrListFill;
        }
    }
    constexpr int kB = 16;
    int n = 0;
    for (int p0 = q0; p0 < q1; p0 += kB) {
        int a[kB], b[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int p = min(p0 + u, q1 - 1);  // clamped: always a valid row
            a[u] = assign[(size_t)p * S + ss];
            b[u] = base[p];
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int x = (unsigned)a[u] < (unsigned)N ? a[u] : N;
            if (p0 + u < q1 && x != b[u]) {
                if (n < kK) keep[wv][n][lane] = make_int2(p0 + u, x);
                ++n;
            }
        }
    }
    wc[wv][lane] = n;
    __syncthreads();
    if (wv == 0) {
        const int tot = wc[0][lane] + wc[1][lane] + wc[2][lane] + wc[3][lane];
        int at = (s < S && tot) ? atomicAdd(&dcnt[s], tot) : 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int c = wc[w][lane];
            wc[w][lane] = at;
            at += c;
        }
    }
    __syncthreads();
    if (s >= S || n == 0) return;
    int q = wc[wv][lane];
    if (n <= kK) {  // the kept entries
        for (int k = 0; k < n; ++k, ++q)
            if (q < cap) {
                const int2 e = keep[wv][k][lane];
                lnode[(size_t)s * cap + q] = e.y;
                lpc[(size_t)s * cap + q] = make_int2(e.x, pod_cpu[e.x]);
            }
        return;
    }
    for (int p0 = q0; p0 < q1; p0 += kB) {
        int a[kB], b[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int p = min(p0 + u, q1 - 1);
            a[u] = assign[(size_t)p * S + ss];
            b[u] = base[p];
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int x = (unsigned)a[u] < (unsigned)N ? a[u] : N;
            if (p0 + u < q1 && x != b[u]) {
                if (q < cap) {
                    lnode[(size_t)s * cap + q] = x;
                    lpc[(size_t)s * cap + q] = make_int2(p0 + u, pod_cpu[p0 + u]);
                }
                ++q;
            }
        }
    }
}

// ---- the persistent loop (rsk_rounds_run): every round of a scenario in one workgroup ----
// Scenarios never touch each other's state, so a workgroup can run all R rounds
// of its scenario without a grid-wide step: detect kept incrementally (a move
// changes the CPU of two nodes; their 64-node blocks' maxima are recomputed and
// the scenario's maxima re-reduced over the blocks), the pick over the pod
// lists, CAR and the update by car_move_one.
struct BlkArgs {
    unsigned long long *bm;  // [S][NB] packed (pct, ~node) max over the block's hazard nodes (0: none)
    unsigned long long *bz;  // [S][NB] packed (cap - use, ~node) max over its non-hazard nodes
    int *bc;                 // [S][NB] its non-hazard nodes
    int NB;
};

__device__ __forceinline__ int pct_of(int u, int c) {  // get_resource_usage.py:37 (cpu_pct_kernel)
    return c == 0 ? -1 : (int)rint((double)u / (double)c * 100.0);
}

// setup: hazard flags and every (scenario, block) entry; lane = scenario,
// wave = (64-scenario chunk, block)
__global__ __launch_bounds__(256) void blk_detect_kernel(const int *__restrict__ use, const int *__restrict__ cap,
                                                         int N, int S, int thr, uint8_t *__restrict__ haz,
                                                         BlkArgs ba) {
    const int lane = (int)threadIdx.x & 63;
    const int nsc = (S + 63) >> 6;
    const int w = (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int b = w / nsc, sc = w - b * nsc;
    if (b >= ba.NB) return;
    const int s = sc * 64 + lane;
    if (s >= S) return;
    const int n0 = b * kBlkNodes, n1 = min(N, n0 + kBlkNodes);
    unsigned long long m = 0ull, z = 0ull;
    int cnt = 0;
    for (int n = n0; n < n1; ++n) {
        const size_t i = (size_t)n * S + s;
        const int c = cap[n], u = use[i], v = pct_of(u, c);
        const bool h = v >= thr;
        haz[i] = h;
        if (h) {
            const unsigned long long k = ((unsigned long long)((unsigned)v ^ 0x80000000u) << 32) | (unsigned long long)(~(unsigned)n);
            m = k > m ? k : m;
        } else {
            ++cnt;
            const unsigned long long k = ((unsigned long long)((unsigned)(c - u) ^ 0x80000000u) << 32) | (unsigned long long)(~(unsigned)n);
            z = k > z ? k : z;
        }
    }
    const size_t o = (size_t)s * ba.NB + b;
    ba.bm[o] = m;
    ba.bz[o] = z;
    ba.bc[o] = cnt;
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(x, o, 64);
        x = y > x ? y : x;
    }
    return x;
}

__device__ __forceinline__ int wave_sum(int x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}


// the scenario's maxima over its NB block entries (every thread; ends with a barrier)
// (sb: the scenario's row of the block arrays, in LDS or global memory)
__device__ __forceinline__ void scn_reduce(const BlkArgs &sb, ScnState *st, unsigned long long *r64, int *r32) {
    const int t = (int)threadIdx.x;
    const BlkArgs &ba = sb;
    const size_t o = 0;
    unsigned long long m = 0ull, z = 0ull;
    int c = 0;
    for (int b = t; b < ba.NB; b += 256) {
        const unsigned long long x = ba.bm[o + b], y = ba.bz[o + b];
        m = x > m ? x : m;
        z = y > z ? y : z;
        c += ba.bc[o + b];
    }
    m = wave_max_u64(m);
    z = wave_max_u64(z);
    c = wave_sum(c);
    if ((t & 63) == 0) {
        r64[t >> 6] = m;
        r64[4 + (t >> 6)] = z;
        r32[t >> 6] = c;
    }
    __syncthreads();
    if (t == 0) {
        for (int w = 1; w < 4; ++w) {
            m = r64[w] > m ? r64[w] : m;
            z = r64[4 + w] > z ? r64[4 + w] : z;
            c += r32[w];
        }
        st->most = m;
        st->zkey = z;
        st->zcnt = c;
    }
    __syncthreads();
}

// block b of scenario s re-reduced after a move, by one wave (lane = node)
template <class NS>
__device__ __forceinline__ void blk_update(const NS &ns, const int *__restrict__ cap, int N, int thr,
                                           const BlkArgs &sb, int b, int o, int t) {
    const int lane = (int)threadIdx.x & 63;
    const int n = b * kBlkNodes + lane;
    unsigned long long m = 0ull, z = 0ull;
    int cnt = 0;
    if (n < N) {
        const int c = cap[n], u = ns.u(n), v = pct_of(u, c);
        const bool h = v >= thr;
        if (n == o || n == t) ns.set_h(n, h);
        if (h) m = ((unsigned long long)((unsigned)v ^ 0x80000000u) << 32) | (unsigned long long)(~(unsigned)n);
        else {
            cnt = 1;
            z = ((unsigned long long)((unsigned)(c - u) ^ 0x80000000u) << 32) | (unsigned long long)(~(unsigned)n);
        }
    }
    m = wave_max_u64(m);
    z = wave_max_u64(z);
    cnt = wave_sum(cnt);
    if (lane == 0) {
        sb.bm[b] = m;
        sb.bz[b] = z;
        sb.bc[b] = cnt;
    }
}

// The persistent loop's detect update after a move of `cpu` from o (the
// scenario's most hazardous node: the pick's node) to t (a non-hazard node:
// CAR never targets a hazard node), by wave 0 alone, incrementally:
//   o's pct falls: its block's hazard max (bm) is recomputed (lane = node; the
//     block's capacities were loaded at the round's start, c_bo), and o joins
//     the block's non-hazard set (bz, bc) when it leaves the hazard set;
//   t's pct rises: t joins its block's hazard max when it becomes a hazard; its
//     non-hazard key falls (or leaves), so bz[bt] is recomputed only when t held
//     it; the count follows;
//   the scenario's most hazardous node is re-reduced over the blocks (o held
//     it), its zero-case count follows the two changes and its zero-case key is
//     re-reduced only when the block that held it lost t's key.
// A block holding both o and t is recomputed in full.  Every value equals what
// blk_update + scn_reduce compute from scratch (harzard_detect.py:3-27 with
// get_resource_usage.py:37's pct; the zero case of rescheduling.py:199-214).
template <class NS>
__device__ __forceinline__ void detect_move_wave(const NS &ns, const int *__restrict__ cap, int N, int thr,
                                                 const BlkArgs &sb, ScnState *st, int o, int t, int c_bo,
                                                 int rem_t_old, int cpu) {
    const int lane = (int)threadIdx.x & 63;
    const int bo = o / kBlkNodes, bt = t / kBlkNodes;
    auto hkey = [](int v, int n) {
        return ((unsigned long long)((unsigned)v ^ 0x80000000u) << 32) | (unsigned long long)(~(unsigned)n);
    };
    // node t after the move (uniform): rem_t_old = cap[t] - use_old[t]
    const int ut = ns.u(t), ct = rem_t_old + ut - cpu, vt = pct_of(ut, ct);
    const bool ht = vt >= thr;
    const unsigned long long zt_old = hkey(rem_t_old, t);
    // block bo, lane = node: o's state is new (usage updated), the others unchanged
    const int n = bo * kBlkNodes + lane;
    unsigned long long m = 0ull, z = 0ull;
    int cnt = 0;
    bool h = false;
    if (n < N) {
        const int u = ns.u(n), v = pct_of(u, c_bo);
        h = v >= thr;
        if (h) m = hkey(v, n);
        else {
            cnt = 1;
            z = hkey(c_bo - u, n);
        }
    }
    const bool ho = __builtin_amdgcn_readlane((int)h, o & 63) != 0;  // o's new hazard flag
    const unsigned long long zb_old = sb.bz[bo], zt_blk_old = sb.bz[bt], zs_old = st->zkey;
    bool zs_recompute = false;
    if (bo == bt) {  // both nodes in one block: the block in full (t's new state is in the lanes too)
        m = dpp_max_u64(m);
        z = dpp_max_u64(z);
        cnt = dpp_sum(cnt);
        if (lane == 0) {
            sb.bm[bo] = m;
            sb.bz[bo] = z;
            sb.bc[bo] = cnt;
        }
        zs_recompute = z < zb_old && zb_old == zs_old;
    } else {
        m = dpp_max_u64(m);  // o held its block's hazard max: recomputed
        unsigned long long zbo = zb_old;
        const int co = __builtin_amdgcn_readlane(c_bo, o & 63);  // cap[o]
        if (!ho) zbo = max(zbo, hkey(co - ns.u(o), o));  // o joins its block's non-hazard set
        unsigned long long zbt = zt_blk_old;
        if (zt_blk_old == zt_old) {  // t held its block's zero-case key: recomputed (t's key fell or left)
            const int nt = bt * kBlkNodes + lane;
            const int cn = cap[min(nt, N - 1)];
            unsigned long long zz = 0ull;
            if (nt < N) {
                const int u = ns.u(nt), v = pct_of(u, cn);
                if (v < thr) zz = hkey(cn - u, nt);
            }
            zbt = dpp_max_u64(zz);
        } else if (!ht) {
            zbt = max(zbt, hkey(ct - ut, t));  // (t's key fell and did not hold the max: unchanged max)
        }
        if (lane == 0) {
            sb.bm[bo] = m;
            sb.bz[bo] = zbo;
            if (!ho) sb.bc[bo] += 1;
            if (ht) {
                sb.bm[bt] = max(sb.bm[bt], hkey(vt, t));
                sb.bc[bt] -= 1;
            }
            sb.bz[bt] = zbt;
        }
        zs_recompute = zbt < zt_blk_old && zt_blk_old == zs_old;
    }
    if (lane == (o & 63)) ns.set_h(o, ho);
    if (lane == 0 && ht) ns.set_h(t, true);
    // the scenario: most hazardous node over the blocks (o held it); the zero case
    const int dz = (ho ? 0 : 1) - (ht ? 1 : 0);
    unsigned long long mm = 0ull, zz = 0ull;
    for (int b = lane; b < sb.NB; b += 64) {
        const unsigned long long x = sb.bm[b];
        mm = x > mm ? x : mm;
        if (zs_recompute) {
            const unsigned long long y = sb.bz[b];
            zz = y > zz ? y : zz;
        }
    }
    mm = dpp_max_u64(mm);
    if (zs_recompute) zz = dpp_max_u64(zz);
    if (lane == 0) {
        st->most = mm;
        st->zcnt += dz;
        st->zkey = zs_recompute ? zz : max(zs_old, max(sb.bz[bo], sb.bz[bt]));
    }
}

// delete_replaced_pod.py:41-61 for scenario s by the workgroup: the pods on
// the most hazardous node m are m's base pods still on m (their assign word
// checked) and the list entries whose node is m (the entry carries the pod's
// CPU); an overflowed list scans every pod's assign word.  Both lists' loads
// are issued together, so the pick costs two dependent round trips after the
// node's base range (ids / entries, then the base pods' assign words).  The
// first max (CPU, -pod) wins, as the reference's strict '>' from -1 over pods
// in order; returns the pod (-1 none) to every thread, the winning list entry
// in *src (-1: a base pod) and its CPU in *pcpu.
template <typename T>
__device__ __forceinline__ int scn_pick(const T *__restrict__ asg, const int *__restrict__ pod_cpu, int P, int S,
                                        int s, unsigned long long kd, const int *__restrict__ off,
                                        const int *__restrict__ pod, const DevLists &dl, unsigned long long *wbest,
                                        int *wsrc, int *src_out, int *pcpu) {
    constexpr int kU = 8;  // 2,048 ids / entries per pass: config 5's lists (~1.3k entries) in one
    const int t = (int)threadIdx.x;
    if (!kd) return -1;  // uniform
    const int m = (int)~(unsigned)(kd & 0xffffffffull);
    const int b0 = off[m], nb = off[m + 1] - b0;
    const int nd = *dl.cnt;
    const bool full = nd > dl.cap;
    const int *ln = dl.lnode;
    auto key = [](int p, int c) {
        return c >= 0 ? ((unsigned long long)((unsigned)c ^ 0x80000000u) << 32) | (unsigned long long)(~(unsigned)p)
                      : 0ull;
    };
    unsigned long long best = 0ull;
    int bsrc = -1;  // the list entry of this thread's best (-1: a base pod)
    if (full) {  // uniform: an overflowed list — every pod's assign word
        for (int i0 = 0; i0 < P; i0 += 256 * kU) {
            int a[kU], c[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int q = min(i0 + u * 256 + t, P - 1);
                a[u] = (int)asg[(size_t)q * S + s];
                c[u] = pod_cpu[q];
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int q = i0 + u * 256 + t;
                const unsigned long long kb = (q < P && a[u] == m) ? key(q, c[u]) : 0ull;
                if (kb > best) best = kb;
            }
        }
    } else {
        // m's base pods (~P/N: one per thread and pass) and the list's node
        // words (kU per thread and pass) loaded together; a base pod's assign
        // word and CPU after its id, an entry's (pod, CPU) only when it is on m
        const int nl = nd;
        for (int i0 = 0, j0 = 0; i0 < nb || j0 < nl; i0 += 256, j0 += 256 * kU) {
            const int q = pod[min(b0 + i0 + t, P - 1)];  // (clamped: always a valid id)
            int en[kU];
            if (j0 < nl) {  // uniform
#pragma unroll
                for (int u = 0; u < kU; ++u) en[u] = ln[min(j0 + u * 256 + t, nl - 1)];
            }
            const int a = (int)asg[(size_t)q * S + s], c = pod_cpu[q];
            const unsigned long long kb = (i0 + t < nb && a == m) ? key(q, c) : 0ull;
            if (kb > best) best = kb, bsrc = -1;
            if (j0 < nl) {
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const int jj = j0 + u * 256 + t;
                    if (jj < nl && en[u] == m) {  // an entry on m (rare): its pod and CPU
                        const int2 e = dl.lpc[jj];
                        const unsigned long long ke = key(e.x, e.y);
                        // >=: an entry of the same pod as a base hit carries the pod's entry index
                        if (ke && ke >= best) best = ke, bsrc = jj;
                    }
                }
            }
        }
    }
    // the wave's best and its list entry (at most one entry per pod), then the
    // workgroup's from the four waves' slots: one barrier, every thread reads
    // the same winner (the slots are rewritten only after the round's tail barrier)
    const unsigned long long wb = dpp_max_u64(best);
    const unsigned long long hit = __builtin_amdgcn_ballot_w64(wb && best == wb && bsrc >= 0);
    const int ws = hit ? __builtin_amdgcn_readlane(bsrc, __builtin_ctzll(hit)) : -1;
    if ((t & 63) == 0) {
        wbest[t >> 6] = wb;
        wsrc[t >> 6] = ws;
    }
    __syncthreads();
    unsigned long long B = wbest[0];
    for (int w = 1; w < kMoveThreads / 64; ++w) B = wbest[w] > B ? wbest[w] : B;
    int src = -1;
    for (int w = 0; w < kMoveThreads / 64; ++w) src = (B && wbest[w] == B && wsrc[w] >= 0) ? wsrc[w] : src;
    *src_out = src;
    *pcpu = (int)((unsigned)(B >> 32) ^ 0x80000000u);  // the winner's CPU (the key's high word)
    return B ? (int)~(unsigned)(B & 0xffffffffull) : -1;
}

struct PersistArgs {
    const int *row_ptr, *col, *pod_cpu, *cap;
    int *assign, *use;
    uint8_t *haz;
    const int *off, *pod;             // the base nodes' pod lists
    DevLists dl;
    BlkArgs ba;
    int *out_evict, *out_target;      // [R][S]
    int P, N, S, H, R, thr;
    int blk_lds;                      // the scenario's block row kept in LDS (after the hash when it is there)
    unsigned hash_bytes;              // dynamic LDS of the hash (0: global work areas)
    unsigned cols_off;                // kCols: byte offset of the usage column and hazard bits in the LDS
    unsigned long long *prof;         // RSK_ROUNDS_PROF builds: [grid][16] per-phase real-time ticks
};

// kCols: the scenario's usage column and hazard bits live in LDS for its R
// rounds (loaded at its start, the usage written back at its end): CAR's
// hazard and cap - use reads, the update and the block re-reductions are LDS
// round trips instead of L2 ones.
template <bool kGlobal, bool kCols>
__global__ __launch_bounds__(kMoveThreads) void rounds_persist_kernel(PersistArgs a, unsigned *__restrict__ gtab) {
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    __shared__ unsigned long long r64[8];
    __shared__ int r32[4];
    __shared__ int lsrc, lcnt;  // the scenario's pick source entry and list length
    __shared__ ScnState st;
    __shared__ unsigned long long pk_best[kMoveThreads / 64];  // scn_pick's per-wave winners
    __shared__ int pk_src[kMoveThreads / 64];
#ifdef RSK_ROUNDS_PROF
    __shared__ PhaseClock pclk;
    PhaseClock *pc = &pclk;
    if (threadIdx.x < kRProfPhases) pclk.acc[threadIdx.x] = 0ull;
#else
    PhaseClock *pc = nullptr;
#endif
    unsigned *tab = kGlobal ? gtab + (size_t)blockIdx.x * (size_t)(2 * a.H + 8) : lds;
    const int t = (int)threadIdx.x;
    NodeCols nc;
    if (kCols) {
        char *cb = reinterpret_cast<char *>(lds) + a.cols_off;
        nc.use = reinterpret_cast<int *>(cb);
        nc.hb = reinterpret_cast<unsigned *>(cb + (size_t)a.N * 4);
    }
    for (int s = (int)blockIdx.x; s < a.S; s += (int)gridDim.x) {
        BlkArgs sb;
        sb.NB = a.ba.NB;
        const size_t row = (size_t)s * a.ba.NB;
        if (a.blk_lds) {  // the row in LDS for the scenario's rounds (written back never: per call)
            char *base = reinterpret_cast<char *>(lds) + a.hash_bytes;
            sb.bm = reinterpret_cast<unsigned long long *>(base);
            sb.bz = sb.bm + sb.NB;
            sb.bc = reinterpret_cast<int *>(sb.bz + sb.NB);
            for (int b = t; b < sb.NB; b += kMoveThreads) {
                sb.bm[b] = a.ba.bm[row + b];
                sb.bz[b] = a.ba.bz[row + b];
                sb.bc[b] = a.ba.bc[row + b];
            }
        } else {
            sb.bm = a.ba.bm + row;
            sb.bz = a.ba.bz + row;
            sb.bc = a.ba.bc + row;
        }
        if (kCols) {  // the usage column (8 loads in flight per thread) and its hazard bits (blk_detect's rule)
            const int nw = (a.N + 31) >> 5;
            for (int w = t; w < nw; w += kMoveThreads) nc.hb[w] = 0u;
            __syncthreads();
            constexpr int kU = 8;
            for (int n0 = t; n0 < a.N; n0 += kMoveThreads * kU) {
                int u[kU], c[kU];
#pragma unroll
                for (int k = 0; k < kU; ++k) {
                    const int n = min(n0 + k * kMoveThreads, a.N - 1);
                    u[k] = a.use[(size_t)n * a.S + s];
                    c[k] = a.cap[n];
                }
#pragma unroll
                for (int k = 0; k < kU; ++k) {
                    const int n = n0 + k * kMoveThreads;
                    if (n >= a.N) break;
                    nc.use[n] = u[k];
                    if (pct_of(u[k], c[k]) >= a.thr) atomicOr(&nc.hb[n >> 5], 1u << (n & 31));
                }
            }
        }
        if (t == 0) lcnt = a.dl.cnt[s];  // the list setup's count (the loop keeps it in LDS)
        DevLists dl = a.dl;
        dl.cnt = &lcnt;
        dl.src = &lsrc;
        dl.lnode = a.dl.lnode + (size_t)s * a.dl.cap;
        dl.lpc = a.dl.lpc + (size_t)s * a.dl.cap;
        __syncthreads();
        scn_reduce(sb, &st, r64, r32);
        // A round: the pick (one barrier), the move, then — wave 0 alone —
        // the detect update of the two changed blocks and the scenario's
        // maxima; the tail barrier publishes the state for the next round.  A
        // row of <= 64 neighbours is scored by wave 0 alone (car_move_one), so
        // such a round holds two workgroup barriers.
        auto rounds = [&](const auto &ns) {
#ifdef RSK_ROUNDS_PROF
            if (t == 0) pclk.start();
#endif
            for (int r = 0; r < a.R; ++r) {
                const unsigned long long kd = st.most;
                const int o = (int)~(unsigned)(kd & 0xffffffffull);  // the hazard node (the pick's pod sits on it)
                // wave 0: the capacities of o's block, consumed by the detect update after the move
                const int c_bo = a.cap[min((kd ? o / kBlkNodes : 0) * kBlkNodes + (t & 63), a.N - 1)];
                int pcpu, src;
                const int p = scn_pick<int>(a.assign, a.pod_cpu, a.P, a.S, s, kd, a.off, a.pod, dl, pk_best, pk_src,
                                            &src, &pcpu);
                RPROF_MARK(pc, 0);
                int *tg_row = a.out_target + (size_t)r * a.S;
                if (t == 0) {
                    a.out_evict[(size_t)r * a.S + s] = p;
                    lsrc = src;  // (read by car_move_one's thread 0)
                }
                if (p < 0) {  // uniform: the state is unchanged
                    if (t == 0) tg_row[s] = kNoEvict;
                    __syncthreads();  // the pick's slots are read before the next round rewrites them
                    continue;
                }
                int tt = car_move_one<kGlobal>(a.row_ptr, a.col, a.pod_cpu, a.assign, ns, a.cap, nullptr, s, a.S, a.N,
                                               a.H, 1, tg_row, nullptr, tab, nullptr, nullptr, nullptr, nullptr,
                                               nullptr, 0, INT_MAX, dl, p, o, pcpu, pc, st.zcnt, st.zkey);
                if (kGlobal) move_sync<true>();  // (global work areas: the update through the agent-scope fence)
                RPROF_MARK(pc, 5);
                if (t < 64) {  // wave 0: thread 0's target, the two changed blocks, the scenario's maxima
                    tt = __builtin_amdgcn_readfirstlane(tt);
                    if (tt >= 0) {
                        detect_move_wave(ns, a.cap, a.N, a.thr, sb, &st, o, tt, c_bo, (int)tab[2 * a.H + 6], pcpu);
                        RPROF_MARK(pc, 6);
                    }
                }
                __syncthreads();  // tail: the detect state, usage, lists and hash free for the next round
                RPROF_MARK(pc, 8);
            }
        };
        if constexpr (kCols) {
            rounds(nc);
            for (int n = t; n < a.N; n += kMoveThreads) a.use[(size_t)n * a.S + s] = nc.use[n];  // the usage back
            __syncthreads();  // the columns are free before the next scenario loads its own
        } else {
            rounds(NodeGlobal{a.use, a.haz, a.S, s});
        }
    }
#ifdef RSK_ROUNDS_PROF
    if (t < kRProfPhases) a.prof[(size_t)blockIdx.x * 16 + t] = pclk.acc[t];
#endif
}

// ---- one-launch CAR for small batches (rsk_car_plan_execute, S <= 4) ----
// A workgroup per (row, scenario) scores the row with car_move_one (lanes =
// neighbours, the LDS hash of their nodes, exact remaining CPU from cap / use):
// no node-code pass, no tiles, no side launch — the latency-bound case
// (config 2: 2k rows x S = 1) in one launch.  Same rule as every CAR path
// (rescheduling.py:183-214, the deduplicated rows without self edges).
template <bool kGlobal>
__global__ __launch_bounds__(kMoveThreads) void car_direct_kernel(const int *__restrict__ rp, const int *__restrict__ ci,
                                                                  const int *__restrict__ rows,
                                                                  const int *__restrict__ items, int istride, int Q,
                                                                  const int *__restrict__ assign,
                                                                  const int *__restrict__ use,
                                                                  const int *__restrict__ cap,
                                                                  const uint8_t *__restrict__ haz, int S, int N, int H,
                                                                  int *__restrict__ out_target,
                                                                  unsigned *__restrict__ gtab) {
    extern __shared__ __attribute__((aligned(16))) unsigned lds[];
    unsigned *tab = kGlobal ? gtab + (size_t)blockIdx.x * (size_t)(2 * H + 8) : lds;
    const int units = Q * S;
    for (int u = (int)blockIdx.x; u < units; u += (int)gridDim.x) {
        const int k = u / S, s = u - k * S;
        const int i = items ? items[(size_t)k * istride] : k;  // the plan row (its target row)
        const int p = rows ? rows[i] : i;
        car_move_one<kGlobal>(rp, ci, nullptr, const_cast<int *>(assign),
                              NodeGlobal{const_cast<int *>(use), const_cast<uint8_t *>(haz), S, s}, cap, nullptr,
                              s, S, N, H, 0, out_target + (size_t)i * S, nullptr, tab, nullptr, nullptr, nullptr,
                              nullptr, nullptr, 0, INT_MAX, DevLists(), p);
        move_sync<kGlobal>();  // the hash is free before the next unit clears it
    }
}

// Row-sharded loop glue: one thread per scenario.
__global__ void rows_evict_key_kernel(const int *__restrict__ local_pod, int S, int r0, const int *__restrict__ pod_cpu,
                                      long long *__restrict__ key) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= S) return;
    const int l = local_pod[s];
    if (l < 0) { key[s] = -1; return; }
    const long long g = (long long)r0 + l;
    key[s] = ((long long)pod_cpu[g] << 32) | (0xffffffffll - g);
}

// A key that does not decode to a pod in [0, P) (a reduced buffer read before
// its producer finished, or garbage) becomes "no eviction", never an index.
__global__ void rows_evict_decode_kernel(const long long *__restrict__ key, int S, int P, int *__restrict__ evict) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= S) return;
    const long long k = key[s];
    const long long g = k >= 0 ? 0xffffffffll - (k & 0xffffffffll) : -1;
    evict[s] = g >= 0 && g < P ? (int)g : -1;
}

// scenario s owns assign[:, s] and the partials' column s: no two threads touch one word
__global__ void rows_apply_kernel(int *__restrict__ assign, int S, const int *__restrict__ evict,
                                  const int *__restrict__ target, int r0, int r1, int P, int N,
                                  const int *__restrict__ pod_cpu, const long long *__restrict__ pod_mem,
                                  long long *__restrict__ cpu_part, long long *__restrict__ mem_part,
                                  unsigned short *__restrict__ shadow) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= S) return;
    const int e = evict[s], t = target[s];
    // no move (None / no candidate / no eviction), and never an index outside
    // the replica: e in [0, P), t in [0, N)
    if (e < 0 || e >= P || t < 0 || t >= N) return;
    int *a = assign + (size_t)e * S + s;
    const int old = *a;
    *a = t;
    if (e < r0 || e >= r1) return;
    if (shadow) shadow[(size_t)(e - r0) * S + s] = (unsigned short)t;
    const long long c = pod_cpu[e], m = pod_mem[e];
    if ((unsigned)old < (unsigned)N) {
        cpu_part[(size_t)old * S + s] -= c;
        mem_part[(size_t)old * S + s] -= m;
    }
    cpu_part[(size_t)t * S + s] += c;
    mem_part[(size_t)t * S + s] += m;
}

// The change of the directed cut over rows [r0, r1) (communicationcost.py:
// 37-45 restricted to this rank's rows, as rsk_cut_cost_rows counts it) when
// scenario s moves pod e from o = assign[e, s] to t — read before the move.
// Only edges at e change: e -> q (row e, when e is this rank's) and q -> e
// (rows q of this rank whose lists hold e: the reverse CSR).  One wave per
// scenario, lanes over the edges; cut[s] += delta.
__global__ __launch_bounds__(256) void rows_cut_delta_kernel(const int *__restrict__ rp, const int *__restrict__ ci,
                                                             const int *__restrict__ rvp, const int *__restrict__ rvi,
                                                             int P, int r0, int r1, const int *__restrict__ assign,
                                                             int S, const int *__restrict__ evict,
                                                             const int *__restrict__ target, int N,
                                                             long long *__restrict__ cut) {
    const int lane = threadIdx.x & 63;
    const int s = (int)blockIdx.x * 4 + ((int)threadIdx.x >> 6);
    if (s >= S) return;  // whole wave
    const int e = evict[s], t = target[s];
    if (e < 0 || e >= P || t < 0 || t >= N) return;  // no move (rows_apply's rule)
    const int o = assign[(size_t)e * S + s];
    int d = 0;
    if (e >= r0 && e < r1)
        for (int k = rp[e] + lane; k < rp[e + 1]; k += 64) {
            const int q = ci[k];
            if (q == e) continue;
            const int a = assign[(size_t)q * S + s];
            d += (int)(t != a) - (int)(o != a);
        }
    for (int k = rvp[e] + lane; k < rvp[e + 1]; k += 64) {
        const int q = rvi[k];
        if (q == e || q < r0 || q >= r1) continue;
        const int a = assign[(size_t)q * S + s];
        d += (int)(a != t) - (int)(a != o);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
    if (lane == 0 && d) cut[s] += d;
}

// ---- the row-sharded loop, fused (rsk_rows_detect_setup / _pick / _place / _move) ----
// delete_replaced_pod.py:41-61 over this rank's rows (T = u16 shadow or int32
// rows): the first max-CPU pod on most[s] (decoded from the detect key), as the
// all-reduce MAX key pod_cpu << 32 | (2^32 - 1 - global pod); 0 = none.
template <typename T>
__global__ __launch_bounds__(256) void rows_pick_kernel(const T *__restrict__ rows, const int *__restrict__ pod_cpu,
                                                        int q, int S, int r0, int ppt, unsigned total,
                                                        const unsigned long long *__restrict__ most,
                                                        unsigned long long *__restrict__ key) {
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (t >= total) return;
    const int s = (int)(t % (unsigned)S);
    const unsigned long long mk = most[s];
    if (!mk) return;
    const int m = (int)~(unsigned)(mk & 0xffffffffull);
    const int p0 = (int)(t / (unsigned)S) * ppt, p1 = min(q, p0 + ppt);
    unsigned long long b = 0;
    for (int p = p0; p < p1; ++p) {
        if ((int)rows[(size_t)p * S + s] != m) continue;
        const long long g = (long long)r0 + p;
        const int c = pod_cpu[g];
        if (c < 0) continue;
        const unsigned long long k = ((unsigned long long)(unsigned)c << 32) | (0xffffffffull - (unsigned long long)g);
        b = k > b ? k : b;
    }
    if (b) atomicMax(&key[s], b);
}

// The round's move for rows [r0, r1): the cut delta of rows_cut_delta_kernel
// (lanes over the moved pod's edges, read before the move), then lane 0 applies
// it as rows_apply_kernel does.  One wave per scenario: scenario s owns
// assign[:, s] and the partials' column s.
__global__ __launch_bounds__(256) void rows_move_kernel(const int *__restrict__ rp, const int *__restrict__ ci,
                                                        const int *__restrict__ rvp, const int *__restrict__ rvi, int P,
                                                        int r0, int r1, int *__restrict__ assign, int S,
                                                        const int *__restrict__ evict, const int *__restrict__ target,
                                                        int N, const int *__restrict__ pod_cpu,
                                                        const long long *__restrict__ pod_mem,
                                                        long long *__restrict__ cpu_part, long long *__restrict__ mem_part,
                                                        unsigned short *__restrict__ shadow, long long *__restrict__ cut) {
    const int lane = threadIdx.x & 63;
    const int s = (int)blockIdx.x * 4 + ((int)threadIdx.x >> 6);
    if (s >= S) return;  // whole wave
    const int e = evict[s], t = target[s];
    if (e < 0 || e >= P || t < 0 || t >= N) return;  // no move (rows_apply's rule)
    int *ae = assign + (size_t)e * S + s;
    const int o = *ae;
    int d = 0;
    if (e >= r0 && e < r1)
        for (int k = rp[e] + lane; k < rp[e + 1]; k += 64) {
            const int q = ci[k];
            if (q == e) continue;
            const int a = assign[(size_t)q * S + s];
            d += (int)(t != a) - (int)(o != a);
        }
    for (int k = rvp[e] + lane; k < rvp[e + 1]; k += 64) {
        const int q = rvi[k];
        if (q == e || q < r0 || q >= r1) continue;
        const int a = assign[(size_t)q * S + s];
        d += (int)(a != t) - (int)(a != o);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
    if (lane != 0) return;
    if (d) cut[s] += d;
    *ae = t;
    if (e < r0 || e >= r1) return;
    if (shadow) shadow[(size_t)(e - r0) * S + s] = (unsigned short)t;
    const long long c = pod_cpu[e], m = pod_mem[e];
    if ((unsigned)o < (unsigned)N) {
        cpu_part[(size_t)o * S + s] -= c;
        mem_part[(size_t)o * S + s] -= m;
    }
    cpu_part[(size_t)t * S + s] += c;
    mem_part[(size_t)t * S + s] += m;
}

// rows_move_kernel with the usage replica and the detection kept in step (one
// workgroup per scenario): wave 0 moves the pod (cut delta, assign, the owner's
// partials and shadow, every rank's usage replica: the round's moves are known
// to all ranks after the target all-gather), waves 0 / 1 re-reduce the two
// changed 64-node blocks, then the workgroup re-reduces the scenario's blocks
// into the next round's most-hazardous key and zero case (rsk_rows_place zeroed
// them).  Same results as a full detect pass over the updated usage.
__global__ __launch_bounds__(256) void rows_move_detect_kernel(
    const int *__restrict__ rp, const int *__restrict__ ci, const int *__restrict__ rvp, const int *__restrict__ rvi,
    int P, int r0, int r1, int *__restrict__ assign, int S, const int *__restrict__ evict,
    const int *__restrict__ target, int N, const int *__restrict__ pod_cpu, const long long *__restrict__ pod_mem,
    long long *__restrict__ cpu_part, long long *__restrict__ mem_part, unsigned short *__restrict__ shadow,
    long long *__restrict__ cut, int *__restrict__ use, const int *__restrict__ cap, int thr,
    uint8_t *__restrict__ haz, BlkArgs ba, unsigned long long *__restrict__ most, int *__restrict__ zc_cnt,
    unsigned long long *__restrict__ zc_key) {
    __shared__ unsigned long long r64[8];
    __shared__ int r32[4];
    __shared__ ScnState st;
    const int lane = (int)threadIdx.x & 63, w = (int)threadIdx.x >> 6;
    const int s = (int)blockIdx.x;
    const int e = evict[s], t = target[s];
    const bool moved = e >= 0 && e < P && t >= 0 && t < N;  // rows_apply's rule (uniform)
    int o = -1;
    if (moved) {
        int *ae = assign + (size_t)e * S + s;
        o = *ae;
        __syncthreads();  // every wave holds the old node before wave 0 stores the new one
        if (w == 0) {
            int d = 0;
            if (e >= r0 && e < r1)
                for (int k = rp[e] + lane; k < rp[e + 1]; k += 64) {
                    const int q = ci[k];
                    if (q == e) continue;
                    const int a = assign[(size_t)q * S + s];
                    d += (int)(t != a) - (int)(o != a);
                }
            for (int k = rvp[e] + lane; k < rvp[e + 1]; k += 64) {
                const int q = rvi[k];
                if (q == e || q < r0 || q >= r1) continue;
                const int a = assign[(size_t)q * S + s];
                d += (int)(a != t) - (int)(a != o);
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
            if (lane == 0) {
                if (d) cut[s] += d;
                *ae = t;
                const int c = pod_cpu[e];
                if ((unsigned)o < (unsigned)N) use[(size_t)o * S + s] -= c;
                use[(size_t)t * S + s] += c;
                if (e >= r0 && e < r1) {
                    if (shadow) shadow[(size_t)(e - r0) * S + s] = (unsigned short)t;
                    const long long m = pod_mem[e];
                    if ((unsigned)o < (unsigned)N) {
                        cpu_part[(size_t)o * S + s] -= c;
                        mem_part[(size_t)o * S + s] -= m;
                    }
                    cpu_part[(size_t)t * S + s] += c;
                    mem_part[(size_t)t * S + s] += m;
                }
            }
        }
        __syncthreads();  // the usage update before the blocks read it
        BlkArgs sb = ba;
        sb.bm = ba.bm + (size_t)s * ba.NB;
        sb.bz = ba.bz + (size_t)s * ba.NB;
        sb.bc = ba.bc + (size_t)s * ba.NB;
        const int bo = (unsigned)o < (unsigned)N ? o / kBlkNodes : -1, bt = t / kBlkNodes;
        const NodeGlobal ng{use, haz, S, s};
        if (w == 0) blk_update(ng, cap, N, thr, sb, bt, o, t);
        if (w == 1 && bo >= 0 && bo != bt) blk_update(ng, cap, N, thr, sb, bo, o, t);
        __syncthreads();
    }
    BlkArgs sb = ba;
    sb.bm = ba.bm + (size_t)s * ba.NB;
    sb.bz = ba.bz + (size_t)s * ba.NB;
    sb.bc = ba.bc + (size_t)s * ba.NB;
    scn_reduce(sb, &st, r64, r32);
    if (threadIdx.x == 0) {
        most[s] = st.most;
        zc_cnt[s] = st.zcnt;
        zc_key[s] = st.zkey;
    }
}

// the scenario maxima from the block arrays (setup), one workgroup per scenario
__global__ __launch_bounds__(256) void blk_scn_kernel(BlkArgs ba, unsigned long long *__restrict__ most,
                                                      int *__restrict__ zc_cnt, unsigned long long *__restrict__ zc_key) {
    __shared__ unsigned long long r64[8];
    __shared__ int r32[4];
    __shared__ ScnState st;
    const int s = (int)blockIdx.x;
    BlkArgs sb = ba;
    sb.bm = ba.bm + (size_t)s * ba.NB;
    sb.bz = ba.bz + (size_t)s * ba.NB;
    sb.bc = ba.bc + (size_t)s * ba.NB;
    scn_reduce(sb, &st, r64, r32);
    if (threadIdx.x == 0) {
        most[s] = st.most;
        zc_cnt[s] = st.zcnt;
        zc_key[s] = st.zkey;
    }
}

}  // namespace

int launch_car_direct(hipStream_t st, const int *rp, const int *ci, const int *rows, int Q, const int *assign,
                      const int *use, const int *cap, const uint8_t *haz, int S, int N, int dmax, int *out_target,
                      DevBuf *scratch, const int *items, int istride) {
    if (Q <= 0) return RSK_OK;
    int H = 1;
    while (H < std::max(2, 2 * std::min(dmax, N))) H <<= 1;
    const size_t bytes = move_tab_bytes(H);
    const int64_t units = (int64_t)Q * S;
    RSK_CHECK(units < INT32_MAX, "direct grid too large");
    if (bytes <= 160 * 1024) {
        const int grid = (int)std::min<int64_t>(units, 65536);
        if (bytes > 64 * 1024)
            RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&car_direct_kernel<false>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
        car_direct_kernel<false><<<dim3((unsigned)grid), dim3(kMoveThreads), bytes, st>>>(
            rp, ci, rows, items, istride, Q, assign, use, cap, haz, S, N, H, out_target, nullptr);
    } else {  // a table beyond the LDS: global work areas, one per resident workgroup
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>({units, 1024, (int64_t)((256u << 20) / bytes)}));
        RSK_CHECK(scratch, "direct CAR: no scratch for a %zu-B table", bytes);
        RSK_TRY(scratch->reserve((size_t)grid * bytes));
        car_direct_kernel<true><<<dim3((unsigned)grid), dim3(kMoveThreads), 0, st>>>(
            rp, ci, rows, items, istride, Q, assign, use, cap, haz, S, N, H, out_target, scratch->as<unsigned>());
    }
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

}  // namespace rsk

using namespace rsk;

extern "C" {

int rsk_rounds_create(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, int32_t P, const int32_t *pod_cpu,
                      rsk_rounds **out) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(out && row_ptr && pod_cpu && P >= 0 && (P == 0 || col_idx || row_ptr[P] == 0), "bad arguments");
    // deduplicated rows without the self edge (the evicted pod is off the cluster, main.py:73)
    std::vector<int32_t> rp(1, 0), ci;
    ci.reserve(P ? (size_t)row_ptr[P] : 0);
    int dmax = 0;
    for (int p = 0; p < P; ++p) {
        RSK_CHECK(row_ptr[p + 1] >= row_ptr[p], "row_ptr not monotone at %d", p);
        const size_t r0 = ci.size();
        for (int k = row_ptr[p]; k < row_ptr[p + 1]; ++k) {
            RSK_CHECK(col_idx[k] >= 0 && col_idx[k] < P, "col_idx[%d] = %d out of range", k, col_idx[k]);
            if (col_idx[k] != p) ci.push_back(col_idx[k]);
        }
        std::sort(ci.begin() + r0, ci.end());
        ci.erase(std::unique(ci.begin() + r0, ci.end()), ci.end());
        dmax = std::max(dmax, (int)(ci.size() - r0));
        rp.push_back((int32_t)ci.size());
    }
    auto *r = new rsk_rounds();
    r->ctx = ctx;
    r->P = P;
    r->dmax = dmax;
    int rc = r->row_ptr.reserve(rp.size() * 4);
    if (rc == RSK_OK) rc = r->col.reserve(std::max<size_t>(1, ci.size()) * 4);
    if (rc == RSK_OK) rc = r->pod_cpu.reserve(std::max<size_t>(1, (size_t)P) * 4);
    if (rc != RSK_OK) { delete r; return rc; }
    RSK_HIP(hipMemcpy(r->row_ptr.ptr, rp.data(), rp.size() * 4, hipMemcpyHostToDevice));
    if (!ci.empty()) RSK_HIP(hipMemcpy(r->col.ptr, ci.data(), ci.size() * 4, hipMemcpyHostToDevice));
    if (P) RSK_HIP(hipMemcpy(r->pod_cpu.ptr, pod_cpu, (size_t)P * 4, hipMemcpyHostToDevice));
    *out = r;
    return RSK_OK;
}

int rsk_rounds_destroy(rsk_rounds *r) {
    if (!r) return RSK_OK;
    (void)hipSetDevice(r->ctx->device);
    (void)hipStreamSynchronize(r->ctx->stream);
    delete r;
    return RSK_OK;
}

int rsk_rounds_run(rsk_rounds *r, int32_t *assign, int32_t S, const int32_t *cap_cpu, int32_t *use_cpu, int32_t N,
                   int32_t threshold, int32_t R, int32_t *out_evict, int32_t *out_target, uint32_t flags) {
    RSK_CHECK(r, "null rounds object");
    rsk_ctx *ctx = r->ctx;
    RSK_TRY(activate(ctx));
    RSK_CHECK(assign && cap_cpu && use_cpu && out_evict && out_target, "null argument");
    RSK_CHECK(S > 0 && N > 0 && R >= 0 && (int64_t)N * S < INT32_MAX && (int64_t)r->P * S < INT32_MAX &&
                  (int64_t)R * S < INT32_MAX,
              "bad sizes S=%d N=%d R=%d", S, N, R);
    const bool dev = flags & RSK_F_DEVICE;
    const size_t NS = (size_t)N * S, PS = (size_t)r->P * S, RS = (size_t)R * S;
    hipStream_t st = ctx->stream;
    // in-out state: host callers' arrays are staged and copied back at the end
    int *d_assign, *d_use, *d_evict, *d_target;
    const int *d_cap;
    RSK_TRY(stage_out(ctx, 0, assign, std::max<size_t>(PS, 1) * 4, dev, reinterpret_cast<void **>(&d_assign)));
    RSK_TRY(stage_out(ctx, 1, use_cpu, NS * 4, dev, reinterpret_cast<void **>(&d_use)));
    RSK_TRY(stage_in(ctx, 2, cap_cpu, (size_t)N * 4, dev, reinterpret_cast<const void **>(&d_cap)));
    RSK_TRY(stage_out(ctx, 3, out_evict, std::max<size_t>(RS, 1) * 4, dev, reinterpret_cast<void **>(&d_evict)));
    RSK_TRY(stage_out(ctx, 4, out_target, std::max<size_t>(RS, 1) * 4, dev, reinterpret_cast<void **>(&d_target)));
    if (!dev) {
        if (PS) RSK_HIP(hipMemcpyAsync(d_assign, assign, PS * 4, hipMemcpyHostToDevice, st));
        RSK_HIP(hipMemcpyAsync(d_use, use_cpu, NS * 4, hipMemcpyHostToDevice, st));
    }
    RSK_TRY(r->haz.reserve(NS));
    const MoveGeom g = move_geometry(r, N, S);
    RSK_TRY(g.rc);
    RSK_TRY(ws_check_u64(N, S, g.H));
    if (R > 0 && r->P == 0) {  // no pod to evict: every round is RSK_TARGET_NO_EVICT
        fill_i32_kernel<<<(unsigned)ceil_div((int64_t)RS, 256), 256, 0, st>>>(d_evict, RS, -1);
        fill_i32_kernel<<<(unsigned)ceil_div((int64_t)RS, 256), 256, 0, st>>>(d_target, RS, kNoEvict);
        RSK_HIP(hipGetLastError());
    } else if (R > 0) {
        // The eviction pick over pod lists: the pods on a node in scenario s are
        // the node's base pods (scenario 0's node) plus those of s's list of pods
        // off their base node; the move appends a pod that leaves its base node.
        // Per round a scenario reads ~(P/N + list) pods instead of its P-pod
        // column.  Built per call from one read of assign.
        DevLists dl;
        const int P = r->P;
        {
            int cap = (int)std::max<int64_t>(256, P / 16);
            cap = (int)std::max<int64_t>(64, std::min<int64_t>(cap, ((int64_t)256 << 20) / ((int64_t)S * 16)));
            RSK_TRY(r->lbase.reserve((size_t)P * 4));
            RSK_TRY(r->loff.reserve((size_t)(N + 2) * 4 * 2));
            RSK_TRY(r->lpod.reserve((size_t)P * 4));
            RSK_TRY(r->lcnt.reserve((size_t)S * 8));  // counts, then the picks' source entries
            const size_t lpc_off = ((size_t)S * cap * 4 + 15) & ~(size_t)15;  // lnode[S * cap], then lpc
            RSK_TRY(r->llist.reserve(lpc_off + (size_t)S * cap * 8));
            int *lnode = r->llist.as<int>();
            int2 *lpc = reinterpret_cast<int2 *>(r->llist.as<char>() + lpc_off);
            int *cntb = r->loff.as<int>() + (N + 2);  // N + 1 counts, then the fill cursors
            ScopedTimer tm(ctx, "rounds_lists");
            RSK_HIP(hipMemsetAsync(cntb, 0, (size_t)(N + 1) * 4, st));
            RSK_HIP(hipMemsetAsync(r->lcnt.ptr, 0, (size_t)S * 4, st));
            list_base_kernel<<<(unsigned)ceil_div(P, 256), 256, 0, st>>>(d_assign, P, S, N, r->lbase.as<int>(), cntb);
            list_scan_kernel<<<1, 1024, 0, st>>>(cntb, N + 1, r->loff.as<int>());
            RSK_HIP(hipMemcpyAsync(cntb, r->loff.ptr, (size_t)(N + 1) * 4, hipMemcpyDeviceToDevice, st));
            const int64_t blocks = ceil_div(P, kLF) * ceil_div(S, 64);
            RSK_CHECK(blocks < INT32_MAX, "list grid too large");
            unsigned *derr = dev_err(ctx);
            RSK_CHECK(derr, "no device error word (mapped pinned memory)");
            list_fill_kernel<<<(unsigned)blocks, 256, 0, st>>>(d_assign, P, S, N, r->lbase.as<int>(), cntb,
                                                                 r->lpod.as<int>(), r->lcnt.as<int>(),
                                                                 r->pod_cpu.as<int>(), lnode, lpc, cap, derr);
            RSK_HIP(hipGetLastError());
            dl.base = r->lbase.as<int>();
            dl.cnt = r->lcnt.as<int>();
            dl.src = dl.cnt + S;
            dl.lnode = lnode;
            dl.lpc = lpc;
            dl.cap = cap;
        }
        // one launch for all R rounds: the hazard flags and the block maxima
        // once, then a workgroup per scenario walks its rounds
        PersistArgs pa;
        pa.ba.NB = (int)blk_nb(N);
        const size_t nbs = (size_t)S * pa.ba.NB;
        RSK_TRY(r->blk.reserve(nbs * 20));
        pa.ba.bm = r->blk.as<unsigned long long>();
        pa.ba.bz = pa.ba.bm + nbs;
        pa.ba.bc = reinterpret_cast<int *>(pa.ba.bz + nbs);
        pa.row_ptr = r->row_ptr.as<int>();
        pa.col = r->col.as<int>();
        pa.pod_cpu = r->pod_cpu.as<int>();
        pa.cap = d_cap;
        pa.assign = d_assign;
        pa.use = d_use;
        pa.haz = r->haz.as<uint8_t>();
        pa.off = r->loff.as<int>();
        pa.pod = r->lpod.as<int>();
        pa.dl = dl;
        pa.out_evict = d_evict;
        pa.out_target = d_target;
        pa.P = r->P;
        pa.N = N;
        pa.S = S;
        pa.H = g.H;
        pa.R = R;
        pa.thr = threshold;
        {
            ScopedTimer tm(ctx, "rounds_detect");
            const int64_t waves = (int64_t)pa.ba.NB * ceil_div(S, 64);
            blk_detect_kernel<<<(unsigned)ceil_div(waves, 4), 256, 0, st>>>(d_use, d_cap, N, S, threshold,
                                                                           r->haz.as<uint8_t>(), pa.ba);
            RSK_HIP(hipGetLastError());
        }
        // the scenario's block row in LDS while it fits beside the hash
        const size_t blk_bytes = (size_t)pa.ba.NB * 20;
        pa.hash_bytes = (unsigned)g.lds;  // move_tab_bytes(H) or 0: the block row's u64 slices start 8-B aligned
        pa.blk_lds = blk_bytes <= 32 * 1024 && g.lds + blk_bytes <= 160 * 1024;
        size_t lds = g.lds + (pa.blk_lds ? blk_bytes : 0);
        // the scenario's usage column and hazard bits in LDS while four
        // workgroups still fit a CU (config 5: 16.4 + 1.6 + 20 + 0.6 KB)
        const size_t cols_bytes = (size_t)N * 4 + (size_t)((N + 31) / 32) * 4;
        const bool cols = g.lds && pa.blk_lds && lds + cols_bytes <= kPersistLdsCols;
        pa.cols_off = cols ? (unsigned)((lds + 15) & ~(size_t)15) : 0u;
        if (cols) lds = pa.cols_off + cols_bytes;
        ScopedTimer tm(ctx, "rounds_persist");
        auto *kern = !g.lds ? &rounds_persist_kernel<true, false>
                            : (cols ? &rounds_persist_kernel<false, true> : &rounds_persist_kernel<false, false>);
        if (lds > 64 * 1024)
            RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)lds));
#ifdef RSK_ROUNDS_PROF
        DevBuf profb;
        RSK_TRY(profb.reserve((size_t)g.grid * 16 * 8));
        RSK_HIP(hipMemsetAsync(profb.ptr, 0, (size_t)g.grid * 16 * 8, st));
        pa.prof = profb.as<unsigned long long>();
#else
        pa.prof = nullptr;
#endif
        kern<<<dim3((unsigned)g.grid), dim3(kMoveThreads), lds, st>>>(pa, g.lds ? nullptr : r->gtab.as<unsigned>());
        RSK_HIP(hipGetLastError());
#ifdef RSK_ROUNDS_PROF
        {   // the per-phase sums, per (scenario, round), to stderr (experiment builds only)
            std::vector<unsigned long long> h((size_t)g.grid * 16);
            RSK_HIP(hipStreamSynchronize(st));
            RSK_HIP(hipMemcpy(h.data(), profb.ptr, h.size() * 8, hipMemcpyDeviceToHost));
            static const char *names[kRProfPhases] = {"pick", "move_setup", "move_count", "move_max", "move_best",
                                                      "move_final", "blk_update", "scn_reduce", "round_tail", "-"};
            double tot = 0;
            for (int k = 0; k < kRProfPhases - 1; ++k) {
                double sum = 0;
                for (int w = 0; w < g.grid; ++w) sum += (double)h[(size_t)w * 16 + k];
                const double us = sum * 0.01 / ((double)S * R);  // 100 MHz ticks -> us per (scenario, round)
                tot += us;
                fprintf(stderr, "[rounds_prof] %-11s %8.4f us per scenario-round\n", names[k], us);
            }
            fprintf(stderr, "[rounds_prof] total       %8.4f us per scenario-round (S=%d R=%d grid=%d)\n", tot, S, R,
                    g.grid);
        }
        profb.release();
#endif
    }
    if (!dev) {
        if (PS) RSK_TRY(copy_back(ctx, assign, d_assign, PS * 4, false));
        RSK_TRY(copy_back(ctx, use_cpu, d_use, NS * 4, false));
        if (RS) {
            RSK_TRY(copy_back(ctx, out_evict, d_evict, RS * 4, false));
            RSK_TRY(copy_back(ctx, out_target, d_target, RS * 4, false));
        }
        RSK_HIP(hipStreamSynchronize(st));
        RSK_TRY(check_dev_err(ctx));
    }
    return RSK_OK;
}

int rsk_rounds_place(rsk_rounds *r, const int32_t *assign, int32_t S, const int32_t *cap_cpu, const int32_t *use_cpu,
                     const uint8_t *hazard, int32_t N, const int32_t *evict, int32_t *out_target, uint32_t flags) {
    RSK_CHECK(r, "null rounds object");
    rsk_ctx *ctx = r->ctx;
    RSK_TRY(activate(ctx));
    RSK_CHECK(assign && cap_cpu && use_cpu && hazard && evict && out_target, "null argument");
    RSK_CHECK(S > 0 && N > 0 && (int64_t)N * S < INT32_MAX && (int64_t)r->P * S < INT32_MAX, "bad sizes S=%d N=%d", S,
              N);
    const bool dev = flags & RSK_F_DEVICE;
    const size_t NS = (size_t)N * S, PS = (size_t)r->P * S;
    const int *d_assign, *d_cap, *d_use, *d_evict;
    const uint8_t *d_haz;
    int *d_target;
    RSK_TRY(stage_in(ctx, 0, assign, std::max<size_t>(PS, 1) * 4, dev, reinterpret_cast<const void **>(&d_assign)));
    RSK_TRY(stage_in(ctx, 1, use_cpu, NS * 4, dev, reinterpret_cast<const void **>(&d_use)));
    RSK_TRY(stage_in(ctx, 2, cap_cpu, (size_t)N * 4, dev, reinterpret_cast<const void **>(&d_cap)));
    RSK_TRY(stage_in(ctx, 3, hazard, NS, dev, reinterpret_cast<const void **>(&d_haz)));
    RSK_TRY(stage_in(ctx, 5, evict, (size_t)S * 4, dev, reinterpret_cast<const void **>(&d_evict)));
    RSK_TRY(stage_out(ctx, 4, out_target, (size_t)S * 4, dev, reinterpret_cast<void **>(&d_target)));
    const MoveGeom g = move_geometry(r, N, S);
    RSK_TRY(g.rc);
    {
        ScopedTimer tm(ctx, "rounds_place");
        RSK_TRY(launch_move(r, ctx->stream, g, const_cast<int *>(d_assign), const_cast<int *>(d_use), d_cap, d_haz,
                            d_evict, S, N, 0, d_target, nullptr));
    }
    if (!dev) {
        RSK_TRY(copy_back(ctx, out_target, d_target, (size_t)S * 4, false));
        RSK_HIP(hipStreamSynchronize(ctx->stream));
    }
    return RSK_OK;
}

// ---- row-sharded loop glue (rsk/dist.py RowShardedRounds) -----------------
int rsk_rows_evict_key(rsk_ctx *ctx, const int32_t *local_pod, int32_t S, int32_t r0, const int32_t *pod_cpu,
                       int64_t *out_key, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK((flags & RSK_F_DEVICE) && local_pod && pod_cpu && out_key && S > 0 && r0 >= 0,
              "rsk_rows_evict_key: device pointers and S > 0 required");
    rows_evict_key_kernel<<<(unsigned)ceil_div(S, 256), 256, 0, ctx->stream>>>(local_pod, S, r0, pod_cpu,
                                                                              reinterpret_cast<long long *>(out_key));
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int rsk_rows_evict_decode(rsk_ctx *ctx, const int64_t *key, int32_t S, int32_t P, int32_t *out_evict, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK((flags & RSK_F_DEVICE) && key && out_evict && S > 0 && P > 0, "rsk_rows_evict_decode: bad arguments");
    rows_evict_decode_kernel<<<(unsigned)ceil_div(S, 256), 256, 0, ctx->stream>>>(
        reinterpret_cast<const long long *>(key), S, P, out_evict);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int rsk_rows_apply(rsk_ctx *ctx, int32_t *assign, int32_t S, const int32_t *evict, const int32_t *target, int32_t r0,
                   int32_t r1, int32_t P, int32_t N, const int32_t *pod_cpu, const int64_t *pod_mem, int64_t *cpu_part,
                   int64_t *mem_part, uint16_t *shadow16, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK((flags & RSK_F_DEVICE) && assign && evict && target && pod_cpu && pod_mem && cpu_part && mem_part &&
                  S > 0 && N > 0 && 0 <= r0 && r0 <= r1 && r1 <= P,
              "rsk_rows_apply: bad arguments (S=%d N=%d rows [%d, %d) of P=%d)", S, N, r0, r1, P);
    rows_apply_kernel<<<(unsigned)ceil_div(S, 256), 256, 0, ctx->stream>>>(
        assign, S, evict, target, r0, r1, P, N, pod_cpu, reinterpret_cast<const long long *>(pod_mem),
        reinterpret_cast<long long *>(cpu_part), reinterpret_cast<long long *>(mem_part), shadow16);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int rsk_rows_cut_delta(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, const int32_t *rev_ptr,
                       const int32_t *rev_idx, int32_t P, int32_t r0, int32_t r1, const int32_t *assign, int32_t S,
                       const int32_t *evict, const int32_t *target, int32_t N, int64_t *cut_inout, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK((flags & RSK_F_DEVICE) && row_ptr && col_idx && rev_ptr && rev_idx && assign && evict && target &&
                  cut_inout && P > 0 && S > 0 && N > 0 && 0 <= r0 && r0 <= r1 && r1 <= P,
              "rsk_rows_cut_delta: bad arguments (device pointers, rows [%d, %d) of P=%d)", r0, r1, P);
    ScopedTimer tm(ctx, "rows_cut_delta");
    rows_cut_delta_kernel<<<(unsigned)ceil_div(S, 4), 256, 0, ctx->stream>>>(
        row_ptr, col_idx, rev_ptr, rev_idx, P, r0, r1, assign, S, evict, target, N,
        reinterpret_cast<long long *>(cut_inout));
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int rsk_pick_max_pod16(rsk_ctx *ctx, const uint16_t *assign16, const int32_t *pod_cpu, int32_t P, int32_t S,
                       const int32_t *most, int32_t *out_pod, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK((flags & RSK_F_DEVICE) && assign16 && pod_cpu && most && out_pod && P >= 0 && S > 0 && S % 8 == 0 &&
                  ((uintptr_t)assign16 % 16) == 0,
              "rsk_pick_max_pod16: device pointers, S %% 8 == 0 and a 16-B aligned shadow required (S=%d)", S);
    RSK_TRY(ctx->work[0].reserve((size_t)S * 8));
    unsigned long long *key = ctx->work[0].as<unsigned long long>();
    ScopedTimer tm(ctx, "pick_max_pod16");
    RSK_HIP(hipMemsetAsync(key, 0, (size_t)S * 8, ctx->stream));
    if (P > 0) {
        const int S8 = S / 8;
        const int ppt = (int)std::max<int64_t>(1, ceil_div((int64_t)P * S8, (int64_t)256 * 4096));
        const int64_t tot = ceil_div(P, ppt) * S8;
        RSK_CHECK(tot < INT32_MAX, "grid too large");
        pick16_kernel<<<(unsigned)ceil_div(tot, 256), 256, 0, ctx->stream>>>(
            reinterpret_cast<const uint4 *>(assign16), pod_cpu, P, S8, most, ppt, (unsigned)tot, key);
        RSK_HIP(hipGetLastError());
    }
    return launch_decode_first_max(ctx->stream, key, S, out_pod);
}

// ---- the row-sharded loop, fused (device pointers; keys zeroed on entry) ----
int rsk_rows_pick(rsk_ctx *ctx, const void *rows, int32_t elem_bytes, int32_t q, int32_t S, int32_t r0,
                  const int32_t *pod_cpu, const int64_t *key_most, int64_t *key_evict, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK((flags & RSK_F_DEVICE) && pod_cpu && key_most && key_evict && (elem_bytes == 2 || elem_bytes == 4) &&
                  q >= 0 && S > 0 && r0 >= 0 && (q == 0 || rows),
              "rsk_rows_pick: device pointers, 2- or 4-byte rows required");
    RSK_TRY(ws_check_ptr(key_most, "key_most"));
    RSK_TRY(ws_check_ptr(key_evict, "key_evict"));
    if (q == 0) return RSK_OK;
    const int ppt = (int)std::max<int64_t>(1, ceil_div((int64_t)q * S, (int64_t)256 * 2048));
    const int64_t tot = ceil_div(q, ppt) * S;
    RSK_CHECK(tot < INT32_MAX, "grid too large");
    ScopedTimer tm(ctx, "rows_pick");
    const auto *mk = reinterpret_cast<const unsigned long long *>(key_most);
    auto *ke = reinterpret_cast<unsigned long long *>(key_evict);
    if (elem_bytes == 2)
        rows_pick_kernel<unsigned short><<<(unsigned)ceil_div(tot, 256), 256, 0, ctx->stream>>>(
            static_cast<const unsigned short *>(rows), pod_cpu, q, S, r0, ppt, (unsigned)tot, mk, ke);
    else
        rows_pick_kernel<int><<<(unsigned)ceil_div(tot, 256), 256, 0, ctx->stream>>>(
            static_cast<const int *>(rows), pod_cpu, q, S, r0, ppt, (unsigned)tot, mk, ke);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int rsk_rows_place(rsk_rounds *r, const int32_t *assign, int32_t S, const int32_t *cap_cpu, const int32_t *use_cpu,
                   const uint8_t *hazard, int32_t N, int32_t r0, int32_t r1, int64_t *key_most, int64_t *key_evict,
                   int32_t *zc_cnt, int64_t *zc_key, int32_t *out_evict, int32_t *out_target, uint32_t flags) {
    RSK_CHECK(r, "null rounds object");
    rsk_ctx *ctx = r->ctx;
    RSK_TRY(activate(ctx));
    RSK_CHECK((flags & RSK_F_DEVICE) && assign && cap_cpu && use_cpu && hazard && key_most && key_evict && zc_cnt &&
                  zc_key && out_evict && out_target && S > 0 && N > 0 && 0 <= r0 && r0 <= r1 && r1 <= r->P &&
                  (int64_t)N * S < INT32_MAX && (int64_t)r->P * S < INT32_MAX,
              "rsk_rows_place: device pointers and rows [%d, %d) of P=%d required", r0, r1, r->P);
    RSK_TRY(ws_check_ptr(key_most, "key_most"));
    RSK_TRY(ws_check_ptr(key_evict, "key_evict"));
    RSK_TRY(ws_check_ptr(zc_key, "zc_key"));
    const MoveGeom g = move_geometry(r, N, S);
    RSK_TRY(g.rc);
    RSK_TRY(ws_check_u64(N, S, g.H));
    ScopedTimer tm(ctx, "rows_place");
    return launch_move(r, ctx->stream, g, const_cast<int *>(assign), const_cast<int *>(use_cpu), cap_cpu, hazard,
                       nullptr, S, N, 0, out_target, nullptr, reinterpret_cast<unsigned long long *>(key_evict),
                       reinterpret_cast<unsigned long long *>(key_most), out_evict, zc_cnt,
                       reinterpret_cast<unsigned long long *>(zc_key), r0, r1);
}

int64_t rsk_rows_blk_bytes(int32_t N, int32_t S) {
    if (N <= 0 || S <= 0) return 0;
    return (int64_t)S * (int64_t)blk_nb(N) * 20;
}

static BlkArgs blk_args(void *blk, int N, int S) {
    BlkArgs ba;
    ba.NB = (int)blk_nb(N);
    const size_t nbs = (size_t)S * ba.NB;
    ba.bm = static_cast<unsigned long long *>(blk);
    ba.bz = ba.bm + nbs;
    ba.bc = reinterpret_cast<int *>(ba.bz + nbs);
    return ba;
}

int rsk_rows_detect_setup(rsk_ctx *ctx, const int32_t *use_cpu, const int32_t *cap_cpu, int32_t N, int32_t S,
                          int32_t threshold, uint8_t *out_hazard, void *blk, int64_t *key_most, int32_t *zc_cnt,
                          int64_t *zc_key, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK((flags & RSK_F_DEVICE) && use_cpu && cap_cpu && out_hazard && blk && key_most && zc_cnt && zc_key &&
                  N > 0 && S > 0 && (int64_t)N * S < INT32_MAX,
              "rsk_rows_detect_setup: device pointers and N, S > 0 required");
    RSK_TRY(ws_check_ptr(blk, "blk"));
    RSK_TRY(ws_check_ptr(key_most, "key_most"));
    RSK_TRY(ws_check_ptr(zc_key, "zc_key"));
    RSK_TRY(ws_check_u64(N, S, 0));
    const BlkArgs ba = blk_args(blk, N, S);
    ScopedTimer tm(ctx, "rows_detect");
    const int64_t waves = (int64_t)ba.NB * ceil_div(S, 64);
    blk_detect_kernel<<<(unsigned)ceil_div(waves, 4), 256, 0, ctx->stream>>>(use_cpu, cap_cpu, N, S, threshold,
                                                                            out_hazard, ba);
    blk_scn_kernel<<<(unsigned)S, 256, 0, ctx->stream>>>(ba, reinterpret_cast<unsigned long long *>(key_most), zc_cnt,
                                                         reinterpret_cast<unsigned long long *>(zc_key));
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int rsk_rows_move(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, const int32_t *rev_ptr,
                  const int32_t *rev_idx, int32_t P, int32_t r0, int32_t r1, int32_t *assign, int32_t S,
                  const int32_t *evict, const int32_t *target, int32_t N, const int32_t *pod_cpu, const int64_t *pod_mem,
                  int64_t *cpu_part, int64_t *mem_part, uint16_t *shadow16, int64_t *cut_inout, int32_t *use_cpu,
                  const int32_t *cap_cpu, int32_t threshold, uint8_t *hazard, void *blk, int64_t *key_most,
                  int32_t *zc_cnt, int64_t *zc_key, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK((flags & RSK_F_DEVICE) && row_ptr && col_idx && rev_ptr && rev_idx && assign && evict && target && pod_cpu &&
                  pod_mem && cpu_part && mem_part && cut_inout && P > 0 && S > 0 && N > 0 && 0 <= r0 && r0 <= r1 &&
                  r1 <= P,
              "rsk_rows_move: device pointers and rows [%d, %d) of P=%d required", r0, r1, P);
    ScopedTimer tm(ctx, "rows_move");
    if (blk) {  // the usage replica and the detection kept in step
        RSK_CHECK(use_cpu && cap_cpu && hazard && key_most && zc_cnt && zc_key,
                  "rsk_rows_move: the detect state (use, cap, hazard, keys) is required with blk");
        RSK_TRY(ws_check_ptr(blk, "blk"));
        RSK_TRY(ws_check_ptr(key_most, "key_most"));
        RSK_TRY(ws_check_ptr(zc_key, "zc_key"));
        RSK_TRY(ws_check_u64(N, S, 0));
        rows_move_detect_kernel<<<(unsigned)S, 256, 0, ctx->stream>>>(
            row_ptr, col_idx, rev_ptr, rev_idx, P, r0, r1, assign, S, evict, target, N, pod_cpu,
            reinterpret_cast<const long long *>(pod_mem), reinterpret_cast<long long *>(cpu_part),
            reinterpret_cast<long long *>(mem_part), shadow16, reinterpret_cast<long long *>(cut_inout), use_cpu,
            cap_cpu, threshold, hazard, blk_args(blk, N, S), reinterpret_cast<unsigned long long *>(key_most), zc_cnt,
            reinterpret_cast<unsigned long long *>(zc_key));
    } else {
        rows_move_kernel<<<(unsigned)ceil_div(S, 4), 256, 0, ctx->stream>>>(
            row_ptr, col_idx, rev_ptr, rev_idx, P, r0, r1, assign, S, evict, target, N, pod_cpu,
            reinterpret_cast<const long long *>(pod_mem), reinterpret_cast<long long *>(cpu_part),
            reinterpret_cast<long long *>(mem_part), shadow16, reinterpret_cast<long long *>(cut_inout));
    }
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

}  // extern "C"
