// rsk_pivot.hip — CAR for the rows above the tile classes (degree > 32) on
// the compact path (N <= 65535), any degree with min(deg, N) <= kPivMaxDistinct.
//
// Reference: the score loop + argmax of `communication`,
// rescheduling.py:183-214 (see rsk_car.hip for the full statement).
//
// Workgroup = (row, chunk of 64 scenarios), lanes = scenarios in all four
// waves, the row's neighbours split over the waves.  What-if scenarios share
// most of their assignment, so per neighbour j the wave takes a pivot node
// p_j — the value most of its 64 lanes hold — and:
//   pass A   the pivot histogram Hp (an LDS hash keyed by node) and, per lane,
//            the few deltas (p_j -> its own node) where it differs;
//   masks    every pivot node touched by a lane's delta gets that lane's bit:
//            the set A_s of nodes whose count differs from the pivot's;
//   pass B   each unchanged entry whose node is not in A_s counts exactly
//            Hp(node): the running (count, code, -node) maximum over them and
//            the number of entries at the maximum count (a node with count c
//            shows c entries) and at the best code;
//   A_s      the lane's own nodes with their exact counts Hp + deltas.
// The union decides as the tile scorers do.  Lanes whose deltas overflow the
// per-lane list, and ties between distinct nodes with equal codes >= 2, are
// finished by the whole workgroup one scenario at a time with exact counts
// and exact remaining CPU (rare: a few lanes per thousand rows).
#include <algorithm>
#include <climits>

#include "rsk_car.h"

namespace rsk {

constexpr int kPW = 4;              // waves per workgroup
constexpr int kPT = 64 * kPW;
constexpr int kPK = 8;              // delta slots per (wave, lane)
constexpr int kPU = 16;             // neighbours in flight per wave (rows up to kPW * kPU stay in registers)

// LDS open-addressing table keyed by node + 1 (16 bits): word = key << 16 |
// count, plus the lanes (64-bit mask) whose delta touches the node.
struct PivTab {
    unsigned *kc, *mlo, *mhi;
    unsigned mask;
    int shift;  // 32 - log2(slots)
    __device__ __forceinline__ unsigned home(unsigned k) const { return (k * 2654435761u) >> shift; }
    // one lane inserts / increments (the key is wave-uniform)
    __device__ __forceinline__ void add(unsigned k) const {
        unsigned h = home(k);
        while (true) {
            const unsigned prev = atomicCAS(&kc[h], 0u, (k << 16) | 1u);
            if (prev == 0u) return;
            if ((prev >> 16) == k) { atomicAdd(&kc[h], 1u); return; }
            h = (h + 1u) & mask;
        }
    }
    __device__ __forceinline__ int find(unsigned k) const {
        unsigned h = home(k);
        while (true) {
            const unsigned w = kc[h];
            if ((w >> 16) == k) return (int)h;
            if (w == 0u) return -1;
            h = (h + 1u) & mask;
        }
    }
    __device__ __forceinline__ int count(unsigned k) const {
        const int h = find(k);
        return h < 0 ? 0 : (int)(kc[h] & 0xffffu);
    }
};

// The wave's pivot for a neighbour: the value held by lane 0 or by the first
// lane that differs from it, whichever more lanes hold (any choice is exact;
// the majority keeps the deltas few).
__device__ __forceinline__ int wave_pivot(int v) {
    const int c0 = __builtin_amdgcn_readfirstlane(v);
    const unsigned long long b0 = __builtin_amdgcn_ballot_w64(v == c0);
    const int n0 = __builtin_popcountll(b0);
    if (n0 >= 33) return c0;
    const int l1 = __builtin_ctzll(~b0);
    const int c1 = __builtin_amdgcn_readlane(v, l1);
    const int n1 = __builtin_popcountll(__builtin_amdgcn_ballot_w64(v == c1));
    return n1 > n0 ? c1 : c0;
}

// Running maximum over entries (main pass) or nodes (A set): M the count, e the
// entries / nodes at M, bw the best (code, -node) word among them, eb how many
// of them carry bw's code.
struct Run {
    int M, e, eb;
    unsigned bw;
    __device__ __forceinline__ void init() { M = 0; e = 0; eb = 0; bw = 0u; }
    __device__ __forceinline__ void put(bool cand, int c, unsigned w) {
        const bool gt = cand && c > M, eq = cand && c == M;
        const unsigned kw = cell_code(w), kb = cell_code(bw);
        eb = gt ? 1 : (eq ? (kw > kb ? 1 : (kw == kb ? eb + 1 : eb)) : eb);
        bw = gt ? w : (eq ? max(bw, w) : bw);
        e = gt ? 1 : (eq ? e + 1 : e);
        M = gt ? c : M;
    }
};

__device__ __forceinline__ int norm_node(int v, int N) { return (unsigned)v < (unsigned)N ? v : -1; }

__global__ __launch_bounds__(kPT) void car_pivot_kernel(PivotArgs a, int shift) {
    extern __shared__ __attribute__((aligned(16))) unsigned plds[];
    const int H = 1 << (32 - shift);
    PivTab tb;
    tb.kc = plds;
    tb.mlo = plds + H;
    tb.mhi = plds + 2 * H;
    tb.mask = (unsigned)H - 1u;
    tb.shift = shift;
    unsigned *dl = plds + 3 * H;                       // [kPW][kPK][64] deltas (old << 16 | new)
    unsigned *dlc = dl + kPW * kPK * 64;               // [kPW][kPK][64] their codes (code old << 16 | code new)
    int *dcnt = reinterpret_cast<int *>(dlc + kPW * kPK * 64);  // [kPW][64] deltas kept
    int *part = dcnt + kPW * 64;                        // [kPW][8][64] per-wave partial results
    int *res = part + kPW * 8 * 64;                     // [3][64]: target, score, slow flag
    int *red = res + 3 * 64;                            // cooperative reductions (4 ints, 8-B aligned)

    const int nchunk = (a.S + 63) >> 6;
    const int item = blockIdx.x % a.n_items;
    const int s0 = (blockIdx.x / a.n_items) * 64;
    (void)nchunk;
    const HeavyItem it = a.items[item];
    const int d = it.d;
    const unsigned S = (unsigned)a.S;
    const int N = a.N;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int s = min(s0 + lane, a.S - 1);
    const cint_ptr col = const_ptr(a.hcol) + it.rb;

    for (int i = tid; i < 3 * H; i += kPT) plds[i] = 0u;
    if (tid < 64) res[2 * 64 + tid] = 0;
    __syncthreads();

    // ---- pass A: pivot histogram + per-lane deltas ----
    // Rows of at most kPW * kPU neighbours are one batch per wave: its
    // assignments, pivots and pivot codes stay in registers for pass B.
    const bool one = d <= kPW * kPU;
    int nv[kPU], pv[kPU];
    unsigned cd[kPU];
    int cnt = 0;
    bool ovf = false;
    for (int j0 = wave * kPU; j0 < d; j0 += kPW * kPU) {
#pragma unroll
        for (int u = 0; u < kPU; ++u) {
            const int q = col[min(j0 + u, d - 1)];
            nv[u] = norm_node(ld32(a.assign, (unsigned)q * S + (unsigned)s), N);
        }
        int mine = -1;  // lane u inserts neighbour u's pivot: the batch's table updates in parallel
#pragma unroll
        for (int u = 0; u < kPU; ++u) {
            pv[u] = j0 + u < d ? wave_pivot(nv[u]) : -1;
            mine = lane == u ? pv[u] : mine;
        }
        if (mine >= 0) tb.add((unsigned)mine + 1u);
        // pivot codes (coalesced: one node per batch entry) and, where the lane
        // differs, its own node's code (elsewhere the same address again)
        unsigned cn[kPU];
#pragma unroll
        for (int u = 0; u < kPU; ++u) {
            cd[u] = ld16(a.code, pv[u] >= 0 ? (unsigned)pv[u] * S + (unsigned)s : 0u);
            const int own = nv[u] >= 0 && nv[u] != pv[u] ? nv[u] : max(pv[u], 0);
            cn[u] = ld16(a.code, (unsigned)own * S + (unsigned)s);
        }
#pragma unroll
        for (int u = 0; u < kPU; ++u) {
            if (j0 + u < d && nv[u] != pv[u]) {
                if (cnt < kPK) {
                    const int o = ((wave * kPK + cnt) << 6) + lane;
                    dl[o] = ((unsigned)(pv[u] & 0xffff) << 16) | (unsigned)(nv[u] & 0xffff);
                    dlc[o] = ((pv[u] >= 0 ? cd[u] : 0u) << 16) | (nv[u] >= 0 ? cn[u] : 0u);
                } else {
                    ovf = true;
                }
                ++cnt;
            }
        }
    }
    dcnt[wave * 64 + lane] = min(cnt, kPK);
    if (ovf) atomicOr(&res[2 * 64 + lane], 1);
    __syncthreads();
    if (a.ablate & 2) return;  // profiling: pass A only (no output)
    if (a.ablate & 32) {  // diagnostics: each lane's delta count (all waves) as its target
        if (wave == 0 && s0 + lane < a.S) {
            int t = 0;
            for (int w = 0; w < kPW; ++w) t += dcnt[w * 64 + lane];
            a.out_target[(size_t)it.oi * S + (unsigned)(s0 + lane)] = t + (res[2 * 64 + lane] ? 1000 : 0);
        }
        return;
    }

    // ---- masks: lanes mark the pivot nodes their deltas touch ----
    {
        const int kc = min(cnt, kPK);
        for (int k = 0; k < kc; ++k) {
            const unsigned pk = dl[((wave * kPK + k) << 6) + lane];
            const unsigned o = pk >> 16, n = pk & 0xffffu;
            const unsigned bit = 1u << (lane & 31);
            unsigned *m = lane < 32 ? tb.mlo : tb.mhi;
            if (o != 0xffffu) { const int h = tb.find(o + 1u); if (h >= 0) atomicOr(&m[h], bit); }
            if (n != 0xffffu) { const int h = tb.find(n + 1u); if (h >= 0) atomicOr(&m[h], bit); }
        }
    }
    __syncthreads();

    if (a.ablate & 4) return;  // profiling: through the masks
    // ---- pass B: unchanged entries on nodes outside A_s ----
    Run rm;
    rm.init();
    for (int j0 = wave * kPU; j0 < d; j0 += kPW * kPU) {
        if (!one) {  // multi-batch rows: reload (L2) the batch and gather its pivots' codes
#pragma unroll
            for (int u = 0; u < kPU; ++u) {
                const int q = col[min(j0 + u, d - 1)];
                nv[u] = norm_node(ld32(a.assign, (unsigned)q * S + (unsigned)s), N);
            }
#pragma unroll
            for (int u = 0; u < kPU; ++u) {
                pv[u] = j0 + u < d ? wave_pivot(nv[u]) : -1;
                cd[u] = ld16(a.code, pv[u] >= 0 ? (unsigned)pv[u] * S + (unsigned)s : 0u);
            }
        }
        // lane u looks up neighbour u's pivot (count, lane masks): one parallel probe per batch
        int mine = -1;
#pragma unroll
        for (int u = 0; u < kPU; ++u) mine = lane == u ? pv[u] : mine;
        unsigned mc = 0u, ml = 0u, mh = 0u;
        if (mine >= 0) {
            const int h = tb.find((unsigned)mine + 1u);
            mc = tb.kc[h] & 0xffffu;
            ml = tb.mlo[h];
            mh = tb.mhi[h];
        }
#pragma unroll
        for (int u = 0; u < kPU; ++u) {
            if (pv[u] < 0) continue;  // uniform
            const int c = __builtin_amdgcn_readlane((int)mc, u);
            const unsigned m = (unsigned)__builtin_amdgcn_readlane((int)(lane < 32 ? ml : mh), u);
            const unsigned m2 = (unsigned)__builtin_amdgcn_readlane((int)mh, u);
            const bool inA = ((lane < 32 ? m : m2) >> (lane & 31)) & 1u;
            const bool cand = nv[u] == pv[u] && !inA && cd[u] != kCodeHaz;
            rm.put(cand, c, (cd[u] << 16) | (0xffffu - (unsigned)pv[u]));
        }
    }

    if (a.ablate & 8) return;  // profiling: through pass B
    // ---- A_s: this wave's delta nodes, exact counts over every wave's deltas ----
    Run ra;
    ra.init();
    if (!(a.ablate & 16)) {
        const int kc = dcnt[wave * 64 + lane];
        for (int k = 0; k < 2 * kc; ++k) {
            const unsigned pk = dl[((wave * kPK + (k >> 1)) << 6) + lane];
            const unsigned x = (k & 1) ? (pk >> 16) : (pk & 0xffffu);
            if (x == 0xffffu) continue;
            // first occurrence only (wave-major, then slot, new before old)
            bool seen = false;
            int adj = 0;
            for (int w2 = 0; w2 < kPW; ++w2) {
                const int k2n = dcnt[w2 * 64 + lane];
                for (int k2 = 0; k2 < k2n; ++k2) {
                    const unsigned p2 = dl[((w2 * kPK + k2) << 6) + lane];
                    const unsigned o2 = p2 >> 16, n2 = p2 & 0xffffu;
                    adj += (n2 == x) - (o2 == x);
                    const int pos2 = (w2 * kPK + k2) * 2, pos = (wave * kPK + (k >> 1)) * 2 + (k & 1);
                    seen |= (pos2 < pos && n2 == x) || (pos2 + 1 < pos && o2 == x);
                }
            }
            if (seen) continue;
            const int c = tb.count(x + 1u) + adj;
            const unsigned pc = dlc[((wave * kPK + (k >> 1)) << 6) + lane];
            const unsigned code = (k & 1) ? (pc >> 16) : (pc & 0xffffu);
            ra.put(c > 0 && code != kCodeHaz, c, (code << 16) | (0xffffu - x));
        }
    }
    {
        int *pp = part + wave * 8 * 64 + lane;
        pp[0] = rm.M; pp[64] = rm.e; pp[128] = rm.eb; pp[192] = (int)rm.bw;
        pp[256] = ra.M; pp[320] = ra.e; pp[384] = ra.eb; pp[448] = (int)ra.bw;
    }
    __syncthreads();

    // ---- combine (wave 0) ----
    if (wave == 0) {
        int Mm = 0, Ma = 0;
        for (int w = 0; w < kPW; ++w) {
            Mm = max(Mm, part[w * 512 + lane]);
            Ma = max(Ma, part[w * 512 + 256 + lane]);
        }
        unsigned bm = 0u, ba = 0u;
        int em = 0, ea = 0;
        for (int w = 0; w < kPW; ++w) {
            const int *pp = part + w * 512 + lane;
            if (Mm > 0 && pp[0] == Mm) { em += pp[64]; bm = max(bm, (unsigned)pp[192]); }
            if (Ma > 0 && pp[256] == Ma) { ea += pp[320]; ba = max(ba, (unsigned)pp[448]); }
        }
        int ebm = 0, eba = 0;
        for (int w = 0; w < kPW; ++w) {
            const int *pp = part + w * 512 + lane;
            if (Mm > 0 && pp[0] == Mm && cell_code((unsigned)pp[192]) == cell_code(bm)) ebm += pp[128];
            if (Ma > 0 && pp[256] == Ma && cell_code((unsigned)pp[448]) == cell_code(ba)) eba += pp[384];
        }
        const int M = max(Mm, Ma);
        int nodes = 0, namb = 0;
        unsigned bw = 0u;
        if (M > 0) {
            if (Mm == M) bw = max(bw, bm);
            if (Ma == M) bw = max(bw, ba);
            if (Mm == M) {
                nodes += em / M;
                if (cell_code(bm) == cell_code(bw)) namb += ebm / M;
            }
            if (Ma == M) {
                nodes += ea;
                if (cell_code(ba) == cell_code(bw)) namb += eba;
            }
        }
        int t, sc = M;
        bool slow = res[2 * 64 + lane] != 0;
        if (M == 0) {
            t = zero_target(load_zc(a.zc_cnt, a.zc_key, s), sc);
        } else if (nodes == 1) {
            t = cand_node(bw);
        } else if (cell_code(bw) < 2u) {
            t = RSK_TARGET_NONE;
        } else {
            t = cand_node(bw);
            slow |= namb > 1 && code_inexact(cell_code(bw));
        }
        res[lane] = t;
        res[64 + lane] = sc;
        res[2 * 64 + lane] = slow ? 1 : 0;
    }
    __syncthreads();

    // ---- slow lanes: the whole workgroup, one scenario at a time, exact ----
    const unsigned long long slow_mask = __builtin_amdgcn_ballot_w64(res[2 * 64 + lane] != 0);
    unsigned long long rest = (a.ablate & 1) ? 0ull : slow_mask;  // identical in every wave
    while (rest) {
        const int ln = __builtin_ctzll(rest);
        rest &= rest - 1ull;
        const int ss = min(s0 + ln, a.S - 1);
        for (int i = tid; i < H; i += kPT) tb.kc[i] = 0u;
        if (tid == 0) { red[0] = 0; red[1] = 0; red[2] = 0; red[3] = 0; }
        __syncthreads();
        for (int j = tid; j < d; j += kPT) {
            const int n = norm_node(ld32(a.assign, (unsigned)col[j] * S + (unsigned)ss), N);
            if (n >= 0 && ld16(a.code, (unsigned)n * S + (unsigned)ss) != kCodeHaz) tb.add((unsigned)n + 1u);
        }
        __syncthreads();
        int cmax = 0;
        for (int j = tid; j < d; j += kPT) {
            const int n = norm_node(ld32(a.assign, (unsigned)col[j] * S + (unsigned)ss), N);
            if (n >= 0) cmax = max(cmax, tb.count((unsigned)n + 1u));
        }
        atomicMax(&red[0], cmax);
        __syncthreads();
        const int M = red[0];
        unsigned long long *best = reinterpret_cast<unsigned long long *>(red + 2);
        for (int j = tid; j < d; j += kPT) {
            const int n = norm_node(ld32(a.assign, (unsigned)col[j] * S + (unsigned)ss), N);
            if (M > 0 && n >= 0 && tb.count((unsigned)n + 1u) == M) {
                atomicAdd(&red[1], 1);
                const int ex = a.cap[n] - ld32(a.use, (unsigned)n * S + (unsigned)ss);
                atomicMax(best, ((unsigned long long)((unsigned)ex ^ 0x80000000u) << 32) | (unsigned long long)(~(unsigned)n));
            }
        }
        __syncthreads();
        if (tid == 0) {
            int t, sc;
            if (M == 0) {
                t = zero_target(load_zc(a.zc_cnt, a.zc_key, ss), sc);
            } else {
                const unsigned long long b = *best;
                const int n = (int)(~(unsigned)(b & 0xffffffffull));
                const int ex = (int)((unsigned)(b >> 32) ^ 0x80000000u);
                const int nodes = red[1] / M;
                sc = M;
                t = nodes == 1 ? n : (ex >= 0 ? n : RSK_TARGET_NONE);
            }
            res[ln] = t;
            res[64 + ln] = sc;
        }
        __syncthreads();
    }

    if (wave == 0 && s0 + lane < a.S) {
        const size_t o = (size_t)it.oi * S + (unsigned)(s0 + lane);
        a.out_target[o] = res[lane];
        if (a.out_score) a.out_score[o] = res[64 + lane];
    }
}

size_t pivot_lds_bytes(int log2_slots) {
    const size_t H = (size_t)1 << log2_slots;
    return (3 * H + (size_t)2 * kPW * kPK * 64 + kPW * 64 + (size_t)kPW * 8 * 64 + 3 * 64 + 4) * 4;
}

int launch_pivot(hipStream_t stream, const PivotArgs &a, int max_distinct) {
    if (a.n_items == 0) return RSK_OK;
    int lg = 6;
    while ((1 << lg) < 2 * max_distinct) ++lg;
    const size_t lds = pivot_lds_bytes(lg);
    RSK_CHECK(lds <= 160 * 1024, "pivot rows: %d distinct nodes need %zu B of LDS", max_distinct, lds);
    if (lds > 64 * 1024)
        RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&car_pivot_kernel),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int64_t blocks = ceil_div(a.S, 64) * (int64_t)a.n_items;
    RSK_CHECK(blocks < INT32_MAX, "pivot grid too large");
    car_pivot_kernel<<<dim3((unsigned)blocks), dim3(kPT), lds, stream>>>(a, 32 - lg);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

}  // namespace rsk
