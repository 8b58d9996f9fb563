// rsk_car.hip — CAR (communication-aware rescheduling) placement on gfx950.
//
// Replaces the score loop + argmax of `communication` (reference
// rescheduling.py:183-214) for a batch of moving pods x what-if scenarios.
//
// For moving pod p and scenario s:
//   score[n] = #{q in row p of the relation CSR : assign[q,s] == n},  n not hazard
//   target   = argmax score; ties (|best| > 1) -> largest cap-use, first index,
//              None if that remaining CPU is < 0; a single best node wins even
//              when overloaded; no candidate at all -> the reference's ValueError.
//
// The dense score row has N entries but only the nodes holding p's neighbours
// can score > 0, so each (p, s) cell is a histogram of deg(p) node ids:
//   * max score M > 0: the winner is among the neighbour nodes: the largest
//     (count, remaining CPU, -node); |best| == 1 iff exactly M entries reach M.
//   * M == 0: every non-hazard node ties at 0 -> a per-scenario constant
//     ("zero case"), computed once by car_prep_kernel.
//
// Kernels (all integer, no order-dependent atomics on the decision path).
// N <= 65535 (the compact path): car_prep16 / car_tile16 (rsk_car16.hip) and
// car_side16 (rsk_side16.hip).  N > 65535 (the wide path, this file):
//   car_prep_kernel   nodekey[n*S+s] = hazard ? KEY_HAZ : cap[n]-use[n*S+s]
//                     (one gather word per node later) + the zero case.
//   car_tile_kernel   deg <= 32 rows, grouped into tiles of <= 128 rows whose
//                     neighbours (<= 144 image rows) are staged once per
//                     32-scenario chunk in LDS together with their node keys;
//                     scoring runs from LDS with per-degree-class scorers
//                     (register pairwise counts up to deg 16, register bitonic
//                     sort of packed (node, image row) words up to deg 32).
//   car_mid_kernel    33..64 rows (17..64 when N is too large for the packed
//                     sort, N >= 2^24 - 1): per-lane register sort of node ids.
//   car_hub_kernel    deg 65..4096: columns of {node, key} staged in LDS,
//                     per-wave LDS count tables, DPP wave reductions.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <unordered_map>
#include <vector>

#include "rsk_car.h"

namespace rsk {

// Bounds-checked debug build (make debug -> librsk_dbg.so, -DRSK_DEBUG_BOUNDS):
// tile-kernel global accesses check their element index against the buffer
// size; a violation sets a bit in rsk_dbg_flags (reported by execute) and the
// access is redirected to element 0 instead of faulting the GPU.
#ifdef RSK_DEBUG_BOUNDS
__device__ unsigned rsk_dbg_flags;
__device__ __forceinline__ unsigned dbg_bound(unsigned idx, unsigned lim, unsigned code) {
    if (idx < lim) return idx;
    atomicOr(&rsk_dbg_flags, code);
    return 0u;
}
#define RSK_BOUND(idx, lim, code) dbg_bound((unsigned)(idx), (unsigned)(lim), (code))
#else
#define RSK_BOUND(idx, lim, code) (idx)
#endif

// ---------------------------------------------------------------------------
// K1: rows with deg <= 32 in LDS tiles.
//
// The plan groups these rows (in DFS order of the relation graph, so a row's
// neighbours are mostly its tile-mates) into tiles of <= 128 rows whose
// distinct neighbours — the tile's image rows — number <= 144.  Workgroup =
// (tile, chunk of SL = 2^lsl <= 32 scenarios), 4 waves:
//   phase 1  every image row's SL-scenario slice of assign, lanes = scenarios
//            (whole 128-B lines), and its node key per scenario gathered from
//            nodekey (L2) -> LDS img[row][SL] = {node, key}; records -> LDS.
//   phase 2  lanes = (record slot, scenario).  A record is
//            [out_row, (deg,) image rows packed 2 x u16 per int]; scorers
//            specialised per degree class read node + key from LDS and store one
//            target word per lane (SL*4 contiguous bytes per row).
// Every access is issued from a clamped, always-valid index and never guarded
// by a branch (hipcc otherwise branches around each guarded load and waits
// vmcnt(0) per element).
// ---------------------------------------------------------------------------
struct TileArgs {
    const int *img_pods;   // concatenated per-tile image pod lists
    const int *meta;       // [T][kMetaW]
    const int *recs;       // concatenated per-tile record blobs (16-B aligned)
    const int *assign;
    const int *nodekey;
    const int *zc_cnt;
    const unsigned long long *zc_key;
    int *out_target;
    int *out_score;
    int S, N, T, lsl, rmax;  // SL = 1 << lsl scenarios per workgroup
    int rec_cap;             // record ints reserved in LDS (largest tile, x4); the unit counter follows
    int ablate;              // profiling only (RSK_ABLATE_TILE): 1 skip image load, 2 skip scoring
    int xcd_per;             // (tile, chunk) units per XCD (XCD-contiguous order)
    unsigned n_assign, n_out, n_pods, n_recs, n_key;  // element counts (debug bounds build)
};

// Element offsets: 32-bit (saddr form, one VGPR) when every offset * 4 < 2^32.
template <bool kOff32>
__device__ __forceinline__ size_t cell(unsigned i, unsigned S, unsigned s) {
    if (kOff32) return (size_t)((i * S + s) << 2);
    return ((size_t)i * S + s) << 2;
}
#ifndef RSK_TILE_NT
#define RSK_TILE_NT 3  // streamed tile loads / stores non-temporal (nodekey lines stay in L2)
#endif
template <bool kOff32>
__device__ __forceinline__ void st_cell(int *base, unsigned i, unsigned S, unsigned s, int v) {
    int *p = reinterpret_cast<int *>(reinterpret_cast<char *>(base) + cell<kOff32>(i, S, s));
    if (RSK_TILE_NT & 2) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Per-lane constants of the scoring phase.  Lanes past the last scenario (a
// partial chunk) and record slots past a class's end redo a valid cell — the
// last scenario / the last record — and store the identical value again.
struct TileLane {
    int slot, PS;
    int col;    // image column of the lane's (clamped) scenario
    int s;      // clamped scenario
    int zt, zs; // zero-case target / score of the scenario
};

template <bool kScore, bool kOff32>
__device__ __forceinline__ void tile_emit(const TileArgs &a, int oi, const TileLane &L, int t, int sc) {
#ifdef RSK_DEBUG_BOUNDS
    if ((size_t)(unsigned)oi * a.S + L.s >= a.n_out || oi < 0) { atomicOr(&rsk_dbg_flags, 1u); return; }
#endif
    st_cell<kOff32>(a.out_target, (unsigned)oi, (unsigned)a.S, (unsigned)L.s, t);
    if (kScore) st_cell<kOff32>(a.out_score, (unsigned)oi, (unsigned)a.S, (unsigned)L.s, sc);
}

// The tile image in LDS: {node, key} int2 per (image row, scenario column).
// This kernel serves N > 65535 only (rsk_car16.hip's 32-bit cells cover the
// rest), so node ids are full ints and an assignment outside [0, N) can never
// alias a real node.
struct TileImg {
    int2 *w;
    int lsl;
    __device__ __forceinline__ int2 at(int row, int col) const { return w[(row << lsl) + col]; }
    __device__ __forceinline__ void put(int i, int n, int k) const { w[i] = make_int2(n, k); }
};

// d == 1: the neighbour's node is the single best unless hazard (zero case).
template <int U, bool kScore, bool kOff32, class Img>
__device__ __forceinline__ void tile_d1(const TileArgs &a, const Img &img, const int *rec, int n, const TileLane &L,
                                        int p0) {
    const int2 *r2 = reinterpret_cast<const int2 *>(rec);
    {
        int2 r[U], e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = r2[min((p0 + u) * L.PS + L.slot, n - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) e[u] = img.at(r[u].y, L.col);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool h = e[u].y == kKeyHaz;
            tile_emit<kScore, kOff32>(a, r[u].x, L, h ? L.zt : e[u].x, h ? L.zs : 1);
        }
    }
}

// d == 2: same node -> score 2; one hazard -> the other; two distinct
// candidates -> tie of two: larger remaining CPU (then lower index), None if < 0.
template <int U, bool kScore, bool kOff32, class Img>
__device__ __forceinline__ void tile_d2(const TileArgs &a, const Img &img, const int *rec, int n, const TileLane &L,
                                        int p0) {
    const int2 *r2 = reinterpret_cast<const int2 *>(rec);
    {
        int2 r[U], e0[U], e1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = r2[min((p0 + u) * L.PS + L.slot, n - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            e0[u] = img.at(r[u].y & 0xffff, L.col);
            e1[u] = img.at((int)((unsigned)r[u].y >> 16), L.col);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int n0 = e0[u].x, k0 = e0[u].y, n1 = e1[u].x, k1 = e1[u].y;
            const bool h0 = k0 == kKeyHaz, h1 = k1 == kKeyHaz;
            const bool w0 = !h0 && (h1 || k0 > k1 || (k0 == k1 && n0 <= n1));
            const int nb = w0 ? n0 : n1, kb = w0 ? k0 : k1;
            const bool single = h0 || h1 || n0 == n1;
            const int tt = single ? nb : (kb >= 0 ? nb : RSK_TARGET_NONE);
            const bool zero = h0 && h1;
            tile_emit<kScore, kOff32>(a, r[u].x, L, zero ? L.zt : tt, zero ? L.zs : (n0 == n1 ? 2 : 1));
        }
    }
}

template <int W>
__device__ __forceinline__ void load_rec(const int *rec, int (&r)[W]) {
    const int4 *r4 = reinterpret_cast<const int4 *>(rec);
#pragma unroll
    for (int w = 0; w < W / 4; ++w) {
        const int4 x = r4[w];
        r[4 * w] = x.x; r[4 * w + 1] = x.y; r[4 * w + 2] = x.z; r[4 * w + 3] = x.w;
    }
}
template <int W>
__device__ __forceinline__ int rec_row(const int (&r)[W], int j) {
    const unsigned pr = (unsigned)r[2 + j / 2];
    return (j & 1) ? (int)(pr >> 16) : (int)(pr & 0xffffu);
}

// 0 or 3 <= d <= D (D = 4, 8, 16): pairwise equality counts in registers,
// c[j] = #{i < j : node i == node j}, so a node's last entry holds its count
// - 1 and the entries at the maximum are exactly one per maximal node; then
// the lexicographic (count, key, -node) maximum over them in 32-bit steps.
template <int D, int W, bool kScore, bool kOff32, class Img>
__device__ __forceinline__ void tile_dn(const TileArgs &a, const Img &img, const int *rec, int n, const TileLane &L,
                                        int p0) {
    {
        int r[W];
        load_rec<W>(rec + min(p0 * L.PS + L.slot, n - 1) * W, r);
        const int d = r[1];
        int nd[D], ky[D], c[D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const int2 e = img.at(rec_row<W>(r, j), L.col);
            // padding entries (j >= d) read row 0: masked out of the counts
            // (a node id no real entry can hold) and of the candidates
            nd[j] = j < d ? e.x : -1 - j;
            ky[j] = j < d ? e.y : kKeyHaz;
            c[j] = 0;
        }
#pragma unroll
        for (int j = 1; j < D; ++j)
#pragma unroll
            for (int i2 = 0; i2 < j; ++i2) c[j] += nd[j] == nd[i2];
        // hazard nodes (all their entries carry KEY_HAZ) leave the count
        int M1 = -1;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            c[j] = ky[j] == kKeyHaz ? -1 : c[j];
            M1 = max(M1, c[j]);
        }
        int kb = INT_MIN;
#pragma unroll
        for (int j = 0; j < D; ++j) kb = max(kb, c[j] == M1 ? ky[j] : INT_MIN);
        int nb = INT_MAX, nm = 0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const bool m = c[j] == M1;
            nb = min(nb, (m && ky[j] == kb) ? nd[j] : INT_MAX);
            nm += m;
        }
        const int tt = nm == 1 ? nb : (kb >= 0 ? nb : RSK_TARGET_NONE);
        tile_emit<kScore, kOff32>(a, r[0], L, M1 < 0 ? L.zt : tt, M1 < 0 ? L.zs : M1 + 1);
    }
}

// 17 <= d <= D (D = 32), record [oi, d, -, -, rows...]: each lane packs its
// entries as node << 8 | image
// row (excluded ones as a sentinel above every node: N < kPackMaxN), sorts them
// with a register bitonic network (min/max only), then walks the sorted runs
// once: a run's key comes from the LDS image of its entry's row; it keeps the
// lexicographic (count, key, -node) maximum and the number of runs at the max.
template <int D, int W, bool kScore, bool kOff32, class Img>
__device__ __forceinline__ void tile_ds(const TileArgs &a, const Img &img, const int *rec, int n, const TileLane &L,
                                        int p0) {
    const unsigned lim = (unsigned)a.N << 8;
    constexpr unsigned kSentinel = 0xffffff00u;  // row 0, node 2^24 - 1 >= N
    {
        // the record stays in LDS: rows are read 8 at a time (one int4), so only
        // the D sort words are live across the network
        const int *rc = rec + min(p0 * L.PS + L.slot, n - 1) * W;
        const int2 hd = *reinterpret_cast<const int2 *>(rc);
        const int d = hd.y;
        unsigned v[D];
#pragma unroll
        for (int j0 = 0; j0 < D; j0 += 8) {
            if (j0 % 16 == 0) __builtin_amdgcn_sched_barrier(0);
            const int4 pk = *reinterpret_cast<const int4 *>(rc + 4 + (j0 >> 1));  // sorted records: rows from int 4
            const unsigned pw[4] = {(unsigned)pk.x, (unsigned)pk.y, (unsigned)pk.z, (unsigned)pk.w};
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int j = j0 + t;
                const int row = (t & 1) ? (int)(pw[t >> 1] >> 16) : (int)(pw[t >> 1] & 0xffffu);
                const int2 e = img.at(row, L.col);
                v[j] = (j < d && e.y != kKeyHaz) ? (((unsigned)e.x << 8) | (unsigned)row) : kSentinel;
            }
        }
        bitonic_sort<D, unsigned>(v);
        unsigned long long best = 0;
        int M = 0, R = 0, c = 0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            // keep the key reads 16 at a time: hoisting all D of them would hold
            // D more registers across the scan
            if (j % 16 == 0) __builtin_amdgcn_sched_barrier(0);
            const unsigned nd = v[j] >> 8;
            c = (j > 0 && nd == (v[j > 0 ? j - 1 : 0] >> 8)) ? c + 1 : 1;
            const bool end = j == D - 1 || (v[j < D - 1 ? j + 1 : j] >> 8) != nd;
            const bool cand = end && v[j] < lim;
            const int k = img.at((int)(v[j] & 0xffu), L.col).y;
            const unsigned long long key = cand ? pack_cand(c, k, (int)nd) : 0ull;
            best = key > best ? key : best;
            const bool gt = cand && c > M, eq = cand && c == M;
            R = gt ? 1 : (eq ? R + 1 : R);
            M = gt ? c : M;
        }
        const CarState st = cand_state(best, M * R);
        const int tt = st.nm == st.bc ? st.bn : (st.br >= 0 ? st.bn : RSK_TARGET_NONE);
        tile_emit<kScore, kOff32>(a, rc[0], L, M == 0 ? L.zt : tt, M == 0 ? L.zs : M);
    }
}

// Phase 1: image rows -> LDS as {node, key} pairs.  Lane = scenario: every
// wave-instruction reads SL contiguous words of 64/SL rows (assign and nodekey
// alike), i.e. whole 128-B lines.  Elements past the end redo the last element
// (identical LDS writes), so nothing is guarded.
template <bool kOff32, class Img>
__device__ __forceinline__ void tile_load_image(const TileArgs &a, const Img &img, int img_off, int nrows, int s0) {
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    const int *__restrict__ pods = a.img_pods + img_off;
    const char *__restrict__ asg = reinterpret_cast<const char *>(a.assign);
    constexpr int kE = kTileRows * 32 / kTileThreads;  // 144 rows x 32 scenarios in one batch
    const int total = nrows << a.lsl;
    const int msk = (1 << a.lsl) - 1;
    for (int b = 0; b < total; b += kTileThreads * kE) {
        int e[kE], pod[kE], v[kE];
#pragma unroll
        for (int u = 0; u < kE; ++u) {
            e[u] = min(b + u * kTileThreads + (int)threadIdx.x, total - 1);
            pod[u] = pods[RSK_BOUND(e[u] >> a.lsl, a.n_pods - img_off, 2u)];
        }
#pragma unroll
        for (int u = 0; u < kE; ++u) {
            const unsigned s = (unsigned)min(s0 + (e[u] & msk), (int)S - 1);
#ifdef RSK_DEBUG_BOUNDS
            if ((size_t)(unsigned)pod[u] * S + s >= a.n_assign) { atomicOr(&rsk_dbg_flags, 4u); pod[u] = 0; }
#endif
            const int *pa = reinterpret_cast<const int *>(asg + cell<kOff32>((unsigned)pod[u], S, s));
            v[u] = (RSK_TILE_NT & 1) ? __builtin_nontemporal_load(pa) : *pa;
        }
#pragma unroll
        for (int u = 0; u < kE; ++u) {
            const int s = s0 + (e[u] & msk);
            const bool ok = (unsigned)v[u] < N && s < (int)S;
            const int key = ld32(a.nodekey, RSK_BOUND(ok ? (unsigned)v[u] * S + (unsigned)s : 0u, a.n_key, 8u));
            img.put(e[u], v[u], ok ? key : kKeyHaz);
        }
    }
}

template <bool kScore, bool kOff32>
__global__ __launch_bounds__(kTileThreads, 4) void car_tile_kernel(TileArgs a) {
    extern __shared__ __attribute__((aligned(16))) int lds[];  // img {node,key} [rmax][SL], then records
    // XCD-contiguous order: blocks b and b + 8 share an XCD, and each XCD walks
    // its own run of chunk-major units, so a chunk's nodekey slice is fetched
    // into one L2 instead of all eight
    const int nchunk = (a.S + (1 << a.lsl) - 1) >> a.lsl;
    const int unit = (int)(blockIdx.x & 7u) * a.xcd_per + (int)(blockIdx.x >> 3);
    if (unit >= nchunk * a.T) return;  // whole workgroup, before any barrier
    const int tile = unit % a.T;
    const int chunk = unit / a.T;
    const int lane = threadIdx.x & 63;
    const int SL = 1 << a.lsl;
    const int s0 = chunk * SL;
    const int cells = a.rmax * SL;
    TileImg img;
    img.lsl = a.lsl;
    img.w = reinterpret_cast<int2 *>(lds);
    int *rec = lds + ((2 * cells + 3) & ~3);  // 16-B aligned for the int4 record reads
    const cint_ptr m = const_ptr(a.meta) + (size_t)tile * kMetaW;
    const int img_off = m[0], nrows = m[1], rec_off = m[2], rec_ints = m[3];

    {   // records -> LDS: one int4 per thread (static_assert above), clamped
        const int i = min((int)threadIdx.x * 4, rec_ints - 4);
        *reinterpret_cast<int4 *>(rec + i) =
            *reinterpret_cast<const int4 *>(a.recs + RSK_BOUND(rec_off + i + 3, a.n_recs, 16u) - 3);
    }
    if (!(RSK_ABL(a) & 1)) tile_load_image<kOff32>(a, img, img_off, nrows, s0);

    TileLane L;
    L.PS = 64 >> a.lsl;
    L.slot = lane >> a.lsl;
    L.s = min(s0 + (lane & (SL - 1)), a.S - 1);
    L.col = L.s - s0;
    {
        int zs;
        L.zt = zero_target(load_zc(a.zc_cnt, a.zc_key, L.s), zs);
        L.zs = zs;
    }
    if (threadIdx.x == 0) rec[a.rec_cap] = 0;  // work-unit counter
    __syncthreads();
    if (RSK_ABL(a) & 2) return;  // profiling ablation: no scoring (results are wrong)
    // Scoring work units (pairs of PS records: d1 4 pairs, d2 2, the rest 1),
    // most expensive class first, handed out by an LDS counter so the few
    // costly high-degree records do not all land on one wave.
    const int n0 = m[4], n1 = m[5], n2 = m[6], n3 = m[7], n4 = m[8], n5 = m[9];
    const int lp = 6 - a.lsl;  // log2(PS), PS = 64 / SL
    const int u5 = (n5 + L.PS - 1) >> lp, u4 = (n4 + L.PS - 1) >> lp, u3 = (n3 + L.PS - 1) >> lp;
    const int u2 = (n2 + L.PS - 1) >> lp, u1 = (((n1 + L.PS - 1) >> lp) + 1) >> 1;
    const int u0 = (((n0 + L.PS - 1) >> lp) + 3) >> 2;
    const int total = u5 + u4 + u3 + u2 + u1 + u0;
    int *ctr = rec + a.rec_cap;
    int k = grab(ctr, lane);
    while (k < total) {
        const int kn = grab(ctr, lane);
        int u = k;
        if (u < u5) {
            tile_ds<32, 20, kScore, kOff32>(a, img, rec + m[15], n5, L, u);
        } else if ((u -= u5) < u4) {
            tile_dn<16, 12, kScore, kOff32>(a, img, rec + m[14], n4, L, u);
        } else if ((u -= u4) < u3) {
            tile_dn<8, 8, kScore, kOff32>(a, img, rec + m[13], n3, L, u);
        } else if ((u -= u3) < u2) {
            tile_dn<4, 4, kScore, kOff32>(a, img, rec + m[12], n2, L, u);
        } else if ((u -= u2) < u1) {
            tile_d2<2, kScore, kOff32>(a, img, rec + m[11], n1, L, 2 * u);
        } else {
            tile_d1<4, kScore, kOff32>(a, img, rec + m[10], n0, L, 4 * (u - u1));
        }
        k = kn;
    }
}

// ---------------------------------------------------------------------------
// K2: mid rows (33..64; 17..64 when N >= kPackMaxN), one wave per (row,
// 64-scenario chunk), lane = scenario.  Each lane loads its deg node ids
// (coalesced 256-B rows), sorts them in registers, then scans the sorted runs
// once, gathering nodekey words 32 at a time.
// ---------------------------------------------------------------------------
struct ScoreCtx {
    const int *nodekey;
    const int *zc_cnt;
    const unsigned long long *zc_key;
    int *out_target;
    int *out_score;
    int S, N, PS;
};

struct MidArgs {
    ScoreCtx sc;
    const int *rec[kNumMid];
    int n_items[kNumMid];
    int prefix[kNumMid + 1];   // waves (rows) per chunk, prefix over buckets
    const int *assign;
    int SL, blocks_per_chunk;
};

template <int D, int W>
__device__ __forceinline__ void mid_row(const MidArgs &a, const int *__restrict__ rec, int slot, int s, bool lane_ok) {
    const int S = a.sc.S;
    const int s_ld = min(s, S - 1);
    const int4 *r4 = reinterpret_cast<const int4 *>(rec);
    const int2 hd = *reinterpret_cast<const int2 *>(rec);
    const int oi = hd.x, d = hd.y;
    int v[D];
#pragma unroll
    for (int w = 0; w < W / 4; ++w) {
        const int4 x = r4[w];
        const int q[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = 4 * w + t - 2;
            if (j >= 0 && j < D) v[j] = a.assign[(size_t)q[t] * S + s_ld];
        }
    }
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = (j < d && (unsigned)v[j] < (unsigned)a.sc.N) ? v[j] : INT_MAX;
    bitonic_sort<D, int>(v);
    constexpr int kC = D > 32 ? 16 : 32;  // key gathers in flight (D = 64: keeps 3 waves per SIMD)
    unsigned long long best = 0;
    int M = 0, R = 0, c = 0;
#pragma unroll
    for (int j0 = 0; j0 < D; j0 += kC) {
        int ky[kC];
#pragma unroll
        for (int t = 0; t < kC; ++t)
            ky[t] = ld32(a.sc.nodekey, (unsigned)(v[j0 + t] == INT_MAX ? 0 : v[j0 + t]) * (unsigned)S + (unsigned)s_ld);
#pragma unroll
        for (int t = 0; t < kC; ++t) {
            const int j = j0 + t;
            c = (j > 0 && v[j] == v[j - (j > 0 ? 1 : 0)]) ? c + 1 : 1;
            const bool end = (j == D - 1) || v[j + (j < D - 1 ? 1 : 0)] != v[j];
            const bool cand = end && v[j] != INT_MAX && ky[t] != kKeyHaz;
            const unsigned long long key = cand ? pack_cand(c, ky[t], v[j]) : 0ull;
            best = key > best ? key : best;
            const bool gt = cand && c > M, eq = cand && c == M;
            R = gt ? 1 : (eq ? R + 1 : R);
            M = gt ? c : M;
        }
    }
    const CarState st = cand_state(best, M * R);
    const ZeroCase z = load_zc(a.sc.zc_cnt, a.sc.zc_key, s_ld);
    if (lane_ok) {
        int sc;
        const int t = car_finalize(st, z, sc);
        const size_t o = (size_t)oi * S + s;
        a.sc.out_target[o] = t;
        if (a.sc.out_score) a.sc.out_score[o] = sc;
    }
}

__global__ __launch_bounds__(256) void car_mid_kernel(MidArgs a) {
    const int chunk = blockIdx.x / a.blocks_per_chunk;
    const int wave = (blockIdx.x % a.blocks_per_chunk) * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (wave >= a.prefix[kNumMid]) return;
    const int slot = lane / a.SL;
    const int s = chunk * a.SL + lane % a.SL;
    const int b = wave >= a.prefix[1] ? 1 : 0;
    const int item = (wave - a.prefix[b]) * a.sc.PS + slot;
    const bool lane_ok = slot < a.sc.PS && s < a.sc.S && item < a.n_items[b];
    const int it = min(item, a.n_items[b] - 1);
    if (b == 0) mid_row<32, 36>(a, a.rec[0] + (size_t)it * 36, slot, s, lane_ok);
    else mid_row<64, 68>(a, a.rec[1] + (size_t)it * 68, slot, s, lane_ok);
}

// ---------------------------------------------------------------------------
// K3: hub rows (deg > 64), see car_hub_kernel below.
// ---------------------------------------------------------------------------
// Per-wave count table of one scenario's neighbour nodes: direct u8 / u16
// counters packed 4 / 2 per word (node < kDirectMaxN; u8 only when the class
// degree is <= 255, so a counter never carries into its neighbour), or an
// open-addressing hash keyed by node+1 (keys[H] then cnts[H]).
enum { kHubHash = 0, kHubU8 = 8, kHubU16 = 16 };

template <int kCnt>
struct HubTable {
    unsigned *keys, *cnts;
    unsigned mask;
    static constexpr int kSh = kCnt == kHubU8 ? 2 : 1;  // log2(counters per word)
    __device__ __forceinline__ unsigned slot(int n) const {  // hash: the slot holding n (inserted)
        const unsigned k = (unsigned)n + 1u;
        unsigned h = (k * 2654435761u) & mask;
        while (keys[h] != k) h = (h + 1u) & mask;
        return h;
    }
    __device__ __forceinline__ unsigned shift(int n) const { return ((unsigned)n & ((1u << kSh) - 1u)) * (unsigned)kCnt; }
    __device__ __forceinline__ void add(int n) const {
        if (kCnt != kHubHash) {
            atomicAdd(&cnts[n >> kSh], 1u << shift(n));
        } else {
            const unsigned k = (unsigned)n + 1u;
            unsigned h = (k * 2654435761u) & mask;
            while (true) {
                const unsigned prev = atomicCAS(&keys[h], 0u, k);
                if (prev == 0u || prev == k) break;
                h = (h + 1u) & mask;
            }
            atomicAdd(&cnts[h], 1u);
        }
    }
    __device__ __forceinline__ int get(int n) const {
        if (kCnt != kHubHash) return (int)((cnts[n >> kSh] >> shift(n)) & ((1u << kCnt) - 1u));
        return (int)cnts[slot(n)];
    }
    __device__ __forceinline__ void clear(int n) const { cnts[n >> kSh] = 0u; }  // direct only
};

// K3 hub rows (deg > 64): one workgroup per (row, group of G = 2^lg
// scenarios), kW waves.  The row's {node, key} columns for the G scenarios
// are staged in LDS (3 dependent rounds of loads: hcol -> assign -> nodekey),
// then each wave takes scenarios wave, wave+kW, ...: lanes = neighbours (NJ
// per lane, kept in registers; NJ = 0: any degree, re-read from LDS), counts
// into the wave's table (A), max count by DPP (B), best (count, rem, -node)
// and the number of maximal entries by DPP/ballot (C), table cleared (D).
template <int kCnt, int NJ, int kW>
__global__ __launch_bounds__(64 * kW) void car_hub_kernel(const HeavyItem *__restrict__ items, int n_items,
                                                          const int *__restrict__ hcol, const int *__restrict__ assign,
                                                          const int *__restrict__ nodekey, int S, int N, int lg, int dpad,
                                                          int H, int gpw, const int *__restrict__ zc_cnt,
                                                          const unsigned long long *__restrict__ zc_key,
                                                          int *__restrict__ out_target, int *__restrict__ out_score) {
    extern __shared__ __attribute__((aligned(16))) int lds[];
    constexpr int kT = 64 * kW;
    const int G = 1 << lg;
    const int ngroups = (S + G - 1) >> lg;
    const int g0 = (blockIdx.x / n_items) * gpw;
    const int g1 = min(g0 + gpw, ngroups);
    const HeavyItem it = items[blockIdx.x % n_items];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int2 *col = reinterpret_cast<int2 *>(lds);                       // [G][dpad]
    unsigned *tabs = reinterpret_cast<unsigned *>(col + G * dpad);   // [kW][Hw]
    const int d = it.d;
    const int total = d << lg;
    // stage: element e -> (neighbour j = e >> lg, scenario si = e & (G-1)); loads
    // unconditional (clamped), duplicates rewrite identical values.  When one
    // batch covers the row (single), the neighbour ids stay in registers across
    // the workgroup's groups and the next group's assign words load beside the
    // current group's key gathers.
    constexpr int kB = 4096 / kT;
    const bool single = total <= kT * kB;
    int e[kB], q[kB], n[kB];
    if (single) {
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            e[u] = min(u * kT + tid, total - 1);
            q[u] = hcol[it.rb + (e[u] >> lg)];
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) n[u] = assign[(size_t)q[u] * S + min(g0 * G + (e[u] & (G - 1)), S - 1)];
    }
    const int Hw = kCnt == kHubHash ? 2 * H : H;  // words per wave table
    for (int k = tid; k < kW * Hw; k += kT) tabs[k] = 0u;
    HubTable<kCnt> tb;
    tb.keys = tabs + wave * Hw;
    tb.cnts = tb.keys + (kCnt == kHubHash ? H : 0);
    tb.mask = (unsigned)H - 1u;
    constexpr int R = NJ > 0 ? NJ : 1;
    const int nj = NJ > 0 ? NJ : (d + 63) >> 6;  // entry slots per lane
    for (int g = g0; g < g1; ++g) {
        const int s0 = g * G;
        if (single) {
            int k[kB], nn[kB];
    #pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int s = s0 + (e[u] & (G - 1));
                const bool ok = (unsigned)n[u] < (unsigned)N && s < S;
                k[u] = ld32(nodekey, ok ? (unsigned)n[u] * (unsigned)S + (unsigned)s : 0u);
            }
    #pragma unroll
            for (int u = 0; u < kB; ++u) nn[u] = assign[(size_t)q[u] * S + min(s0 + G + (e[u] & (G - 1)), S - 1)];
    #pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int si = e[u] & (G - 1), s = s0 + si;
                const bool ok = (unsigned)n[u] < (unsigned)N && s < S;
                col[si * dpad + (e[u] >> lg)] = make_int2(n[u], ok ? k[u] : kKeyHaz);
                n[u] = nn[u];
            }
        } else {
            for (int e0 = 0; e0 < total; e0 += kT * kB) {
                int eb[kB], qb[kB], nb[kB];
    #pragma unroll
                for (int u = 0; u < kB; ++u) {
                    eb[u] = min(e0 + u * kT + tid, total - 1);
                    qb[u] = hcol[it.rb + (eb[u] >> lg)];
                }
    #pragma unroll
                for (int u = 0; u < kB; ++u) nb[u] = assign[(size_t)qb[u] * S + min(s0 + (eb[u] & (G - 1)), S - 1)];
    #pragma unroll
                for (int u = 0; u < kB; ++u) {
                    const int si = eb[u] & (G - 1), s = s0 + si;
                    const bool ok = (unsigned)nb[u] < (unsigned)N && s < S;
                    const int key = ld32(nodekey, ok ? (unsigned)nb[u] * (unsigned)S + (unsigned)s : 0u);
                    col[si * dpad + (eb[u] >> lg)] = make_int2(nb[u], ok ? key : kKeyHaz);
                }
            }
        }
        __syncthreads();
        for (int si = wave; si < G && s0 + si < S; si += kW) {
            const int2 *c = col + si * dpad;
            int M = 0;
            unsigned long long best = 0;
            int nm = 0;
            if (NJ > 0) {
                int xn[R], xk[R], cn[R];
    #pragma unroll
                for (int i = 0; i < R; ++i) {
                    const int j = i * 64 + lane;
                    const int2 x = c[min(j, d - 1)];
                    xn[i] = x.x;
                    xk[i] = j < d ? x.y : kKeyHaz;
                }
    #pragma unroll
                for (int i = 0; i < R; ++i)  // A
                    if (xk[i] != kKeyHaz) tb.add(xn[i]);
    #pragma unroll
                for (int i = 0; i < R; ++i) {  // B
                    cn[i] = xk[i] != kKeyHaz ? tb.get(xn[i]) : 0;
                    M = max(M, cn[i]);
                }
                M = dpp_max(M);
    #pragma unroll
                for (int i = 0; i < R; ++i) {  // C
                    const bool m = cn[i] == M;
                    nm += __builtin_popcountll(__builtin_amdgcn_ballot_w64(m));
                    const unsigned long long k = m ? pack_rn(xk[i], xn[i]) : 0ull;
                    best = k > best ? k : best;
                }
                if (M > 0) best = dpp_max_u64(best);
                if (kCnt != kHubHash) {  // D
    #pragma unroll
                    for (int i = 0; i < R; ++i)
                        if (xk[i] != kKeyHaz) tb.clear(xn[i]);
                }
            } else {
                for (int i = 0; i < nj; ++i) {  // A
                    const int j = i * 64 + lane;
                    const int2 x = c[min(j, d - 1)];
                    if (j < d && x.y != kKeyHaz) tb.add(x.x);
                }
                for (int i = 0; i < nj; ++i) {  // B
                    const int j = i * 64 + lane;
                    const int2 x = c[min(j, d - 1)];
                    if (j < d && x.y != kKeyHaz) M = max(M, tb.get(x.x));
                }
                M = dpp_max(M);
                if (M > 0) {
                    for (int i = 0; i < nj; ++i) {  // C
                        const int j = i * 64 + lane;
                        const int2 x = c[min(j, d - 1)];
                        const bool m = j < d && x.y != kKeyHaz && tb.get(x.x) == M;
                        nm += __builtin_popcountll(__builtin_amdgcn_ballot_w64(m));
                        const unsigned long long k = m ? pack_rn(x.y, x.x) : 0ull;
                        best = k > best ? k : best;
                    }
                    best = dpp_max_u64(best);
                }
                if (kCnt != kHubHash) {  // D
                    for (int i = 0; i < nj; ++i) {
                        const int j = i * 64 + lane;
                        const int2 x = c[min(j, d - 1)];
                        if (j < d && x.y != kKeyHaz) tb.clear(x.x);
                    }
                }
            }
            if (kCnt == kHubHash)  // a probe may still need a slot another lane cleared: wipe the whole table
                for (int k = lane; k < Hw; k += 64) tb.keys[k] = 0u;
            const int rb = (int)((unsigned)(best >> kNodeBits) ^ 0x80000000u);
            const int nb = (int)(kNodeMask - (unsigned)(best & kNodeMask));
            if (lane == 0) {
                const int s = s0 + si;
                int sc, t;
                if (M == 0) {
                    t = zero_target(load_zc(zc_cnt, zc_key, s), sc);
                } else {
                    sc = M;
                    t = nm == M ? nb : (rb >= 0 ? nb : RSK_TARGET_NONE);
                }
                const size_t o = (size_t)it.oi * S + s;
                out_target[o] = t;
                if (out_score) out_score[o] = sc;
            }
        }
        __syncthreads();  // the next group restages the columns
    }
}

}  // namespace rsk

using namespace rsk;


// Wide path (N > 65535), rows above kHubMax neighbours: one workgroup per
// (row, scenario), looping over them; each workgroup owns an open-addressing
// table of (node + 1, count) in global memory (2^lg slots, load <= 1/2).  The
// scores are rescheduling.py:183-195's histogram over the candidate nodes; the
// decision :199-214 — the largest count, a single best node wins, else the
// largest cap - use (first index), None when it is < 0; no candidate at all:
// the zero case.  Every table access is an atomic performed in L2 (the slots
// are reused across items: no stale L1 lines).
struct BigRowArgs {
    const HeavyItem *items;  // {out row, offset into col, degree}
    int n_items;
    const int *col, *assign, *nodekey;
    const int *zc_cnt;
    const unsigned long long *zc_key;
    int *out_target, *out_score;
    int S, N, lg;
    unsigned *keys, *cnts;  // [gridDim.x][1 << lg]
};
constexpr int kBigThreads = 256;
__global__ __launch_bounds__(kBigThreads) void car_bigrow_kernel(BigRowArgs a) {
    __shared__ unsigned long long red[kBigThreads / 64];
    __shared__ int redi[kBigThreads / 64];
    const int H = 1 << a.lg;
    const unsigned mask = (unsigned)H - 1u;
    unsigned *keys = a.keys + (size_t)blockIdx.x * (size_t)H, *cnts = a.cnts + (size_t)blockIdx.x * (size_t)H;
    const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
    const int64_t total = (int64_t)a.n_items * a.S;
    for (int64_t it = blockIdx.x; it < total; it += gridDim.x) {  // workgroup-uniform
        const int r = (int)(it / a.S), s = (int)(it - (int64_t)r * a.S);
        const HeavyItem h = a.items[r];
        for (int i = (int)threadIdx.x; i < H; i += kBigThreads) {
            __hip_atomic_store(&keys[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&cnts[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        for (int j = (int)threadIdx.x; j < h.d; j += kBigThreads) {
            const int n = a.assign[(size_t)a.col[h.rb + j] * a.S + s];
            if (n < 0 || n >= a.N || a.nodekey[(size_t)n * a.S + s] == kKeyHaz) continue;  // not a candidate
            const unsigned k = (unsigned)n + 1u;
            unsigned slot = (k * 2654435761u) >> (32 - a.lg);
            while (true) {
                const unsigned prev = atomicCAS(&keys[slot], 0u, k);
                if (prev == 0u || prev == k) break;
                slot = (slot + 1u) & mask;
            }
            atomicAdd(&cnts[slot], 1u);
        }
        __syncthreads();
        // the largest count
        int mc = 0;
        for (int i = (int)threadIdx.x; i < H; i += kBigThreads)
            mc = max(mc, (int)__hip_atomic_load(&cnts[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        mc = dpp_max(mc);
        if (lane == 0) redi[wave] = mc;
        __syncthreads();
        int M = 0;
        for (int w = 0; w < kBigThreads / 64; ++w) M = max(M, redi[w]);
        __syncthreads();
        // among the nodes at M: the largest (cap - use, -node) and how many there are
        unsigned long long best = 0ull;
        int cnt_at_m = 0;
        if (M > 0)
            for (int i = (int)threadIdx.x; i < H; i += kBigThreads) {
                if ((int)__hip_atomic_load(&cnts[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != M) continue;
                const int n = (int)__hip_atomic_load(&keys[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - 1;
                const unsigned long long k = pack_rn(a.nodekey[(size_t)n * a.S + s], n);
                best = k > best ? k : best;
                ++cnt_at_m;
            }
        best = dpp_max_u64(best);
        if (lane == 0) red[wave] = best;
        for (int o = 32; o >= 1; o >>= 1) cnt_at_m += __shfl_xor(cnt_at_m, o, 64);
        __syncthreads();  // every wave has read redi (M) and written red
        if (lane == 0) redi[wave] = cnt_at_m;
        __syncthreads();
        for (int w = 0; w < kBigThreads / 64; ++w) best = red[w] > best ? red[w] : best;
        if (threadIdx.x == 0) {
            int nbest = 0;
            for (int w = 0; w < kBigThreads / 64; ++w) nbest += redi[w];
            int t, sc;
            if (M == 0) {
                t = zero_target(load_zc(a.zc_cnt, a.zc_key, s), sc);
            } else {
                sc = M;
                const int bn = (int)(kNodeMask - (unsigned)(best & kNodeMask));
                const int br = (int)((unsigned)(best >> kNodeBits) ^ 0x80000000u);
                t = nbest == 1 ? bn : (br >= 0 ? bn : RSK_TARGET_NONE);
            }
            const size_t o = (size_t)(unsigned)h.oi * (size_t)a.S + (size_t)s;
            a.out_target[o] = t;
            if (a.out_score) a.out_score[o] = sc;
        }
        __syncthreads();
    }
}

struct rsk_car_plan {
    rsk_ctx *ctx = nullptr;
    int P = 0, Q = 0, max_deg = 0;
    int light_max = kLightMax;  // rows with deg <= light_max go to the tiles
    // tiles
    int T = 0, T_lean = 0, rmax = 0, recmax = 0, n_tile_rows = 0, n_sorted_rows = 0;  // T_lean == T (info field)
    int n_lean_rows = 0;  // == n_tile_rows (info field)
    int owners_cap = kTileOwners, rows_cap = kTileRows;  // tile limits
    int64_t img_rows_total = 0, img_pods_distinct = 0, n_img_pods = 0, n_recs = 0;
    DevBuf img_pods, meta, recs;
    // mid rows (17..64), only in a plan with light_max = kPairMax
    int n_mid[kNumMid] = {0, 0};
    DevBuf mid[kNumMid];
    // hub rows (> 64) of the wide path
    int n_heavy[kNumHeavy] = {};
    int heavy_dmax[kNumHeavy] = {};
    DevBuf heavy_items[kNumHeavy];
    DevBuf hcol;
    // compact path: every side row (deg > light_max) for car_side16, degree
    // descending, split into the kSideMax classes (neighbours in pcol)
    DevBuf side_items, pcol;
    DevBuf side_scratch;  // work areas of side rows whose table exceeds the LDS
    // wide path: rows above kHubMax neighbours (car_bigrow_kernel), neighbours in pcol
    DevBuf big_items;
    int n_big = 0, big_dmax = 0;
    // distinct neighbour pods of the tile rows plus the side classes [0, hi)
    // (nb_distinct[hi]; [0]: the tile rows alone): the algorithmic assign
    // bytes of the fused launch; fused_lo / fused_hi: the side classes the last
    // execute ran inside the lean tile launch ([lo, hi), empty when lo == hi)
    int64_t nb_distinct[kNumSide + 1] = {};
    int fused_lo = 0, fused_hi = 0;
    int side_beg[kNumSide] = {}, side_end[kNumSide] = {};
    int side_dmax[kNumSide] = {};
    // per-execute workspace
    DevBuf nodekey, code, zc;
    int zc_S = 0, zc_half = 0;  // the zero-case words' double buffer (S it is sized for, the half in use)
    // the deduplicated CSR and the row map on the device (the one-launch path of small batches)
    DevBuf drp, dci, drows;
    int ddmax = 0;
    // the inputs, kept for the N >= kPackMaxN variant (built on first use)
    std::vector<int32_t> h_row_ptr, h_col_idx, h_rows;
    bool has_rows = false;
    rsk_car_plan *alt = nullptr;
    ~rsk_car_plan() {
        delete alt;
        img_pods.release();
        meta.release();
        recs.release();
        for (auto &b : mid) b.release();
        for (auto &b : heavy_items) b.release();
        hcol.release();
        side_items.release();
        side_scratch.release();
        drp.release();
        dci.release();
        drows.release();
        big_items.release();
        pcol.release();
        nodekey.release();
        code.release();
        zc.release();
    }
};

namespace {


int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

struct HeavyGeom {
    int lg, dpad, H, mode, waves;
    size_t lds;
};

constexpr int kDirectMaxN = 16384;  // direct count tables up to 32 KiB per wave

HeavyGeom heavy_geometry(int dmax, int S, int N) {
    // Count table per wave: u8 / u16 direct counters (N <= kDirectMaxN), else a
    // hash of 2 * next_pow2(2 * dmax) words.  Then the widest (waves, G = 2^lg
    // scenario group) whose staged columns + tables fit 80 KiB (2 workgroups
    // per CU), preferring 8 waves, then 4; else the same within 160 KiB.
    HeavyGeom g;
    g.dpad = dmax | 1;
    if (N <= kDirectMaxN) {
        g.mode = dmax <= 255 ? kHubU8 : kHubU16;
        g.H = g.mode == kHubU8 ? (N + 3) / 4 : (N + 1) / 2;
    } else {
        g.mode = kHubHash;
        g.H = next_pow2(2 * dmax);
    }
    const size_t words = g.mode == kHubHash ? 2 * (size_t)g.H : (size_t)g.H;
    const int gmax = std::min(64, next_pow2(S));
    for (size_t lim : {(size_t)80 * 1024, (size_t)160 * 1024})
        for (int w : {8, 4})
            for (int G = gmax; G >= std::min(gmax, 8); G >>= 1) {
                g.waves = w;
                g.lds = (size_t)G * g.dpad * 8 + (size_t)w * words * 4;
                g.lg = 0;
                while ((1 << g.lg) < G) ++g.lg;
                if (g.lds <= lim) return g;
            }
    for (int G = gmax; G >= 1; G >>= 1) {  // last resort: 4 waves, small groups
        g.waves = 4;
        g.lds = (size_t)G * g.dpad * 8 + 4 * words * 4;
        g.lg = 0;
        while ((1 << g.lg) < G) ++g.lg;
        if (g.lds <= (size_t)160 * 1024) return g;
    }
    return g;
}

typedef void (*HubKern)(const HeavyItem *, int, const int *, const int *, const int *, int, int, int, int, int, int,
                        const int *, const unsigned long long *, int *, int *);

template <int kCnt, int kW>
HubKern hub_kern_nj(int nj) {
    switch (nj) {
        case 2: return &car_hub_kernel<kCnt, 2, kW>;
        case 4: return &car_hub_kernel<kCnt, 4, kW>;
        case 8: return &car_hub_kernel<kCnt, 8, kW>;
        case 16: return &car_hub_kernel<kCnt, 16, kW>;
        default: return &car_hub_kernel<kCnt, 0, kW>;
    }
}

template <int kW>
HubKern hub_kern_mode(int mode, int nj) {
    if (mode == kHubU8) return hub_kern_nj<kHubU8, kW>(nj);
    if (mode == kHubU16) return hub_kern_nj<kHubU16, kW>(nj);
    return hub_kern_nj<kHubHash, kW>(nj);
}

int upload(DevBuf &buf, const void *src, size_t bytes) {
    if (!bytes) return RSK_OK;
    RSK_TRY(buf.reserve(bytes));
    RSK_HIP(hipMemcpy(buf.ptr, src, bytes, hipMemcpyHostToDevice));
    return RSK_OK;
}

int build_plan(rsk_car_plan *plan, const int32_t *row_ptr, const int32_t *col_idx, int32_t P, const int32_t *rows,
               int32_t Q) {
    PlanHost h;
    RSK_TRY(plan_build_host(row_ptr, col_idx, P, rows, Q, plan->light_max, plan->owners_cap, plan->rows_cap, &h));
    {   // the deduplicated CSR for the one-launch path (rsk_rounds.hip car_direct_kernel)
        RSK_TRY(plan->drp.reserve(h.rp.size() * 4));
        RSK_TRY(plan->dci.reserve(std::max<size_t>(1, h.ci.size()) * 4));
        RSK_HIP(hipMemcpy(plan->drp.ptr, h.rp.data(), h.rp.size() * 4, hipMemcpyHostToDevice));
        if (!h.ci.empty()) RSK_HIP(hipMemcpy(plan->dci.ptr, h.ci.data(), h.ci.size() * 4, hipMemcpyHostToDevice));
        if (rows && Q > 0) {
            RSK_TRY(plan->drows.reserve((size_t)Q * 4));
            RSK_HIP(hipMemcpy(plan->drows.ptr, rows, (size_t)Q * 4, hipMemcpyHostToDevice));
        }
        plan->ddmax = h.ddmax;
    }
    plan->max_deg = h.max_deg;
    plan->T = plan->T_lean = h.T;
    plan->n_lean_rows = h.n_tile_rows;
    plan->rmax = std::max(1, h.rmax);
    plan->recmax = h.recmax;
    plan->n_tile_rows = h.n_tile_rows;
    plan->n_sorted_rows = h.n_sorted_rows;
    plan->img_rows_total = h.img_rows_total;
    plan->img_pods_distinct = h.img_pods_distinct;
    plan->n_img_pods = (int64_t)h.img_pods.size();
    plan->n_recs = h.n_recs;
    if (h.T > 0) {
        RSK_TRY(upload(plan->img_pods, h.img_pods.data(), h.img_pods.size() * 4));
        RSK_TRY(upload(plan->meta, h.meta.data(), h.meta.size() * 4));
        RSK_TRY(upload(plan->recs, h.recs.data(), h.recs.size() * 4));
    }
    for (int b = 0; b < kNumMid; ++b) {
        plan->n_mid[b] = h.n_mid[b];
        RSK_TRY(upload(plan->mid[b], h.mid[b].data(), h.mid[b].size() * 4));
    }
    for (int c = 0; c < kNumHeavy; ++c) {
        plan->n_heavy[c] = h.n_heavy[c];
        plan->heavy_dmax[c] = h.heavy_dmax[c];
        RSK_TRY(upload(plan->heavy_items[c], h.heavy_items[c].data(), h.heavy_items[c].size() * sizeof(HeavyItem)));
    }
    RSK_TRY(upload(plan->hcol, h.hcol.data(), h.hcol.size() * 4));
    RSK_TRY(upload(plan->pcol, h.pcol.data(), h.pcol.size() * 4));
    plan->n_big = h.n_big;
    plan->big_dmax = h.big_dmax;
    if (h.n_big) RSK_TRY(upload(plan->big_items, h.side_items.data(), (size_t)h.n_big * 4 * 4));
    for (int c = 0; c < kNumSide; ++c) {
        plan->side_beg[c] = h.side_beg[c];
        plan->side_end[c] = h.side_end[c];
        plan->side_dmax[c] = h.side_dmax[c];
    }
    for (int c = 0; c <= kNumSide; ++c) plan->nb_distinct[c] = h.nb_distinct[c];
    RSK_TRY(upload(plan->side_items, h.side_items.data(), h.side_items.size() * 4));
    return RSK_OK;
}

int plan_create(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, int32_t P, const int32_t *rows,
                int32_t Q, int light_max, rsk_car_plan **out) {
    auto plan = new rsk_car_plan();
    plan->ctx = ctx;
    plan->light_max = light_max;
    // tile limits: the image rows the compact kernels are built for (RSK_TILE16_ROWS), owners
    // in the 128 : 144 ratio
    const int rows_built = tile16_rows_built();
    plan->owners_cap = std::min(kTileOwners, std::max(8, rows_built * kTileOwners / kTileRows));
    plan->rows_cap = std::min(rows_built, std::max(kLightMax, rows_built));  // a row fits alone
    plan->P = P;
    plan->Q = Q;
    const int rc = build_plan(plan, row_ptr, col_idx, P, rows, Q);
    if (rc != RSK_OK) {
        std::string keep = last_error();
        delete plan;
        set_error("%s", keep.c_str());
        return rc;
    }
    if (plan->n_sorted_rows > 0) {  // kept for the N >= kPackMaxN variant
        plan->h_row_ptr.assign(row_ptr, row_ptr + P + 1);
        plan->h_col_idx.assign(col_idx, col_idx + (P ? row_ptr[P] : 0));
        plan->has_rows = rows != nullptr;
        if (rows) plan->h_rows.assign(rows, rows + Q);
    }
    *out = plan;
    return RSK_OK;
}

// Mid (17..64, N >= kPackMaxN variant only) and hub (> 64) rows, queued on `stream`.
// Mid and hub launches go round-robin over the `nside` streams in `side`
// (mid, hub classes in degree order), so the few-row latency-bound hub classes
// do not queue behind each other.
struct SideBufs {
    const int *assign, *key, *cap, *use, *zcnt;
    const unsigned short *code;
    const unsigned long long *zkey;
    int *target, *score;
    const uint8_t *haz;   // on-the-fly launches (launch_side16_otf)
};

// car_side16 launches of classes [c0, c1) on `stream`, the longest rows first.
// Classes from kSideBig up (rows above 128 neighbours: few work items, each
// latency-bound) run on a side stream beside the tiles (rsk_car_plan_execute).
constexpr int kSideBig = 2;
// rows beyond the fused grid with at most this many (row, scenario) cells run
// as one workgroup per cell (car_direct_kernel) instead of pivot teams
constexpr int64_t kDirectBigCells = 8192;
SideArgs side16_class_args(const rsk_car_plan *plan, int c, const SideBufs &b, int S, int N) {
    static const int sablate = RSK_ABLATION(RSK_ABLATE_SIDE);
    SideArgs a;
    std::memset(&a, 0, sizeof(a));
    a.items = plan->side_items.as<int>() + (size_t)plan->side_beg[c] * 4;
    a.n_rows = plan->side_end[c] - plan->side_beg[c];
    a.nchunk = (int)ceil_div(S, 64);
    a.col = plan->pcol.as<int>();
    a.assign = b.assign;
    a.code = b.code;
    a.cap = b.cap;
    a.use = b.use;
    a.zc_cnt = b.zcnt;
    a.zc_key = b.zkey;
    a.out_target = b.target;
    a.out_score = b.score;
    a.S = S;
    a.N = N;
    a.ablate = sablate;
    return a;
}

// classes [c0, c1) except `skip` (fused into the tile launch)
int launch_side16_classes(rsk_car_plan *plan, rsk_ctx *ctx, hipStream_t stream, const SideBufs &b, int S, int N,
                          int c0, int c1, int skip = -1, bool otf = false) {
    const bool off32 = (int64_t)std::max(plan->P, plan->Q) * S * 4 < ((int64_t)1 << 32);
    for (int c = c1 - 1; c >= c0; --c) {
        if (c == skip || plan->side_end[c] == plan->side_beg[c]) continue;
        SideArgs a = side16_class_args(plan, c, b, S, N);
        const SideGeom g = side16_geometry(plan->side_dmax[c], N);
        ScopedTimer tm(ctx, "car_side", stream);
        if (otf) {
            a.code = nullptr;
            a.haz = b.haz;
            RSK_TRY(launch_side16_otf(stream, a, g, off32, &plan->side_scratch));
        } else {
            RSK_TRY(launch_side16(stream, a, g, off32, &plan->side_scratch));
        }
    }
    return RSK_OK;
}

// Side rows on `stream`: the compact path's classes below kSideBig (the rest
// are launched beside the tiles by the caller); the wide path's mid (17..64,
// N >= kPackMaxN variant only) and hub (> 64) rows, exact keys.
int launch_side(rsk_car_plan *plan, rsk_ctx *ctx, hipStream_t stream, const SideBufs &b, int S, int N, bool compact,
                int skip = -1) {
    if (compact) return launch_side16_classes(plan, ctx, stream, b, S, N, 0, kSideBig, skip);
    const int *d_assign = b.assign, *d_key = b.key, *d_zcnt = b.zcnt;
    const unsigned long long *d_zkey = b.zkey;
    int *d_target = b.target, *d_score = b.score;
    ScoreCtx sc;
    sc.nodekey = d_key;
    sc.zc_cnt = d_zcnt;
    sc.zc_key = d_zkey;
    sc.out_target = d_target;
    sc.out_score = d_score;
    sc.S = S;
    sc.N = N;
    const int SL = std::min(S, 64);
    sc.PS = 64 / SL;
    const int64_t chunks = ceil_div(S, SL);
    {   // K2 mid rows, exact keys
        MidArgs a;
        std::memset(&a, 0, sizeof(a));
        a.sc = sc;
        a.SL = SL;
        a.prefix[0] = 0;
        for (int k = 0; k < kNumMid; ++k) {
            a.rec[k] = plan->mid[k].as<int>();
            a.n_items[k] = plan->n_mid[k];
            a.prefix[k + 1] = a.prefix[k] + (int)ceil_div(plan->n_mid[k], sc.PS);
        }
        a.assign = d_assign;
        const int waves = a.prefix[kNumMid];
        if (waves > 0) {
            a.blocks_per_chunk = (int)ceil_div(waves, 4);
            const int64_t blocks = chunks * a.blocks_per_chunk;
            RSK_CHECK(blocks < INT32_MAX, "mid grid too large");
            ScopedTimer tm(ctx, "car_mid", stream);
            car_mid_kernel<<<dim3((unsigned)blocks), dim3(256), 0, stream>>>(a);
            RSK_HIP(hipGetLastError());
        }
    }
    for (int c = 0; c < kNumHeavy; ++c) {   // K3 hub rows
        const int n = plan->n_heavy[c];
        if (!n) continue;
        const HeavyGeom g = heavy_geometry(plan->heavy_dmax[c], S, N);
        RSK_CHECK(g.lds <= 160 * 1024, "hub class %d needs %zu B of LDS", c, g.lds);
        const int64_t groups = ceil_div(S, 1 << g.lg);
        // scenario groups per workgroup: enough workgroups to fill the GPU twice over
        const int gpw = (int)std::max<int64_t>(1, std::min<int64_t>(8, groups * n / 1024));
        const int64_t gblocks = ceil_div(groups, gpw);
        RSK_CHECK(gblocks * n < INT32_MAX, "hub grid too large");
        const HubKern kern = g.waves == 8 ? hub_kern_mode<8>(g.mode, kHeavyNJ[c]) : hub_kern_mode<4>(g.mode, kHeavyNJ[c]);
        if (g.lds > 64 * 1024)
            RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)g.lds));
        ScopedTimer tm(ctx, "car_heavy", stream);
        kern<<<dim3((unsigned)(gblocks * n)), dim3(64 * g.waves), g.lds, stream>>>(
            plan->heavy_items[c].as<HeavyItem>(), n, plan->hcol.as<int>(), d_assign, d_key, S, N, g.lg, g.dpad,
            g.H, gpw, d_zcnt, d_zkey, d_target, d_score);
        RSK_HIP(hipGetLastError());
    }
    if (plan->n_big > 0) {  // K4: rows above kHubMax neighbours
        BigRowArgs a;
        std::memset(&a, 0, sizeof(a));
        a.items = plan->big_items.as<HeavyItem>();
        a.n_items = plan->n_big;
        a.col = plan->pcol.as<int>();
        a.assign = d_assign;
        a.nodekey = d_key;
        a.zc_cnt = d_zcnt;
        a.zc_key = d_zkey;
        a.out_target = d_target;
        a.out_score = d_score;
        a.S = S;
        a.N = N;
        a.lg = 1;
        while ((1 << a.lg) < 2 * std::min(plan->big_dmax, N)) ++a.lg;
        const size_t H = (size_t)1 << a.lg;
        const int64_t items = (int64_t)plan->n_big * S;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>({items, 1024, (int64_t)((256u << 20) / (H * 8))}));
        RSK_TRY(plan->side_scratch.reserve((size_t)grid * H * 8));
        a.keys = plan->side_scratch.as<unsigned>();
        a.cnts = a.keys + (size_t)grid * H;
        ScopedTimer tm(ctx, "car_heavy", stream);
        car_bigrow_kernel<<<dim3((unsigned)grid), dim3(kBigThreads), 0, stream>>>(a);
        RSK_HIP(hipGetLastError());
    }
    return RSK_OK;
}


}  // namespace

extern "C" {

int rsk_car_plan_create(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, int32_t P,
                        const int32_t *rows, int32_t Q, rsk_car_plan **out) {
    RSK_CHECK(out, "null output pointer");
    *out = nullptr;
    RSK_TRY(activate(ctx));
    RSK_CHECK(P >= 0 && row_ptr, "bad CSR (P=%d)", P);
    if (!rows) Q = P;
    RSK_CHECK(Q >= 0, "bad row count %d", Q);
    RSK_CHECK(row_ptr[0] == 0, "row_ptr[0] must be 0");
    for (int32_t p = 0; p < P; ++p)
        RSK_CHECK(row_ptr[p + 1] >= row_ptr[p], "row_ptr not monotone at %d", p);
    const int64_t nnz = P ? row_ptr[P] : 0;
    RSK_CHECK(nnz == 0 || col_idx, "null col_idx");
    for (int64_t k = 0; k < nnz; ++k)
        RSK_CHECK(col_idx[k] >= 0 && col_idx[k] < P, "col_idx[%lld]=%d out of range", (long long)k, col_idx[k]);
    if (rows)
        for (int32_t i = 0; i < Q; ++i) RSK_CHECK(rows[i] >= 0 && rows[i] < P, "rows[%d]=%d out of range", i, rows[i]);
    // rows up to kLightMax neighbours go to the LDS tiles, the rest to the side
    // kernels (the wide path's kPairMax variant is built on first use, below)
    return plan_create(ctx, row_ptr, col_idx, P, rows, Q, kLightMax, out);
}

int rsk_car_plan_info(const rsk_car_plan *plan, int64_t *out, int n) {
    RSK_CHECK(plan && out && n >= 0, "bad arguments");
    int64_t mid = 0, heavy = 0, mid_bytes = 0;
    int64_t heavy_bytes = (int64_t)plan->hcol.bytes;
    for (int b = 0; b < kNumMid; ++b) {
        mid += plan->n_mid[b];
        mid_bytes += (int64_t)plan->n_mid[b] * kMidW[b] * 4;
    }
    for (int c = 0; c < kNumHeavy; ++c) {
        heavy += plan->n_heavy[c];
        heavy_bytes += (int64_t)plan->n_heavy[c] * (int64_t)sizeof(HeavyItem);
    }
    const int64_t tile_bytes = plan->T > 0 ? (int64_t)(plan->img_pods.bytes + plan->meta.bytes + plan->recs.bytes) : 0;
    const int64_t side = plan->side_end[0] - plan->side_beg[kNumSide - 1];
    const int64_t side_bytes = (int64_t)plan->side_items.bytes + (int64_t)plan->pcol.bytes;
    int64_t fused_rows = 0;
    for (int c = plan->fused_lo; c < plan->fused_hi; ++c) fused_rows += plan->side_end[c] - plan->side_beg[c];
    // the tile rows' and the fused side rows' distinct neighbour pods (classes [0, hi) counted when lo == 0)
    const int64_t fused_nb = plan->fused_lo == 0 ? plan->nb_distinct[plan->fused_hi] : plan->nb_distinct[0];
    const int64_t v[23] = {plan->n_tile_rows, 0, mid, heavy, plan->T, plan->rmax, plan->owners_cap,
                           tile_bytes, 0, mid_bytes, heavy_bytes, plan->max_deg, plan->img_rows_total,
                           plan->img_pods_distinct, plan->n_sorted_rows, side, side_bytes, plan->light_max,
                           plan->n_lean_rows, plan->T_lean, fused_rows, fused_nb,
                           plan->nb_distinct[kNumSide]};
    const int m = n < 23 ? n : 23;
    for (int i = 0; i < m; ++i) out[i] = v[i];
    return m;
}

int rsk_car_plan_destroy(rsk_car_plan *plan) {
    if (!plan) return RSK_OK;
    (void)hipSetDevice(plan->ctx->device);
    (void)hipStreamSynchronize(plan->ctx->stream);
    delete plan;
    return RSK_OK;
}

int rsk_car_plan_execute(rsk_car_plan *plan, const int32_t *assign, int32_t S, const int32_t *cap_cpu,
                         const int32_t *use_cpu, const uint8_t *hazard, int32_t N, int32_t *out_target,
                         int32_t *out_score, uint32_t flags) {
    RSK_CHECK(plan, "null plan");
    rsk_ctx *ctx = plan->ctx;
    RSK_TRY(activate(ctx));
    RSK_CHECK(S > 0 && N > 0, "need S > 0 and N > 0 (S=%d N=%d)", S, N);
    RSK_CHECK((int64_t)N * S < ((int64_t)1 << 30) && N < (1 << kNodeBits) && (int64_t)plan->P * S < ((int64_t)1 << 40),
              "N*S too large (N=%d S=%d; need N*S < 2^30, N < 2^25)", N, S);
    RSK_CHECK(out_target, "null out_target");
    // compact path (rsk_car16.hip) whenever node ids fit 16 bits
    // (S < 2^23: the tile kernel's 24-bit code offsets, rsk_car16.hip t16_rows64)
    // (rows above kMaxDegree neighbours: the side tables count in 16 bits, so
    // such a plan runs the wide path, whose car_bigrow counts in 32)
    const bool compact = N <= kMaxNodes16 && S < (1 << 23) && plan->max_deg <= kMaxDegree;
    if (!compact && N >= kPackMaxN && plan->n_sorted_rows > 0) {
        // the wide sorted tile classes pack node << 8 | row into 32 bits: route
        // 17..64 rows through the mid kernel instead (variant built once)
        if (!plan->alt)
            RSK_TRY(plan_create(ctx, plan->h_row_ptr.data(), plan->h_col_idx.data(), plan->P,
                                plan->has_rows ? plan->h_rows.data() : nullptr, plan->Q, kPairMax, &plan->alt));
        return rsk_car_plan_execute(plan->alt, assign, S, cap_cpu, use_cpu, hazard, N, out_target, out_score, flags);
    }
    const bool dev = (flags & RSK_F_DEVICE) != 0;
    const size_t PS_ = (size_t)plan->P * S, NS = (size_t)N * S, QS = (size_t)plan->Q * S;

    const int *d_assign, *d_cap, *d_use;
    const uint8_t *d_haz;
    int *d_target, *d_score = nullptr;
    RSK_TRY(stage_in(ctx, 0, assign, PS_ * 4, dev, reinterpret_cast<const void **>(&d_assign)));
    RSK_TRY(stage_in(ctx, 1, cap_cpu, (size_t)N * 4, dev, reinterpret_cast<const void **>(&d_cap)));
    RSK_TRY(stage_in(ctx, 2, use_cpu, NS * 4, dev, reinterpret_cast<const void **>(&d_use)));
    RSK_TRY(stage_in(ctx, 3, hazard, NS, dev, reinterpret_cast<const void **>(&d_haz)));
    RSK_TRY(stage_out(ctx, 4, out_target, QS * 4, dev, reinterpret_cast<void **>(&d_target)));
    if (out_score) RSK_TRY(stage_out(ctx, 5, out_score, QS * 4, dev, reinterpret_cast<void **>(&d_score)));

    // small batches: one launch (a workgroup per (row, scenario), exact rem from
    // cap / use, no node codes); the latency-bound case, config 2
    if (!(flags & RSK_F_TILED) && S <= 4 && QS <= 65536 && !d_score) {
        {
            ScopedTimer tm(ctx, "car_direct");
            RSK_TRY(launch_car_direct(ctx->stream, plan->drp.as<int>(), plan->dci.as<int>(),
                                      plan->drows.ptr ? plan->drows.as<int>() : nullptr, plan->Q, d_assign, d_use,
                                      d_cap, d_haz, S, N, plan->ddmax, d_target, &plan->side_scratch));
        }
        if (!dev) {
            RSK_TRY(copy_back(ctx, out_target, d_target, QS * 4, false));
            RSK_HIP(hipStreamSynchronize(ctx->stream));
            for (size_t k = 0; k < QS; ++k)
                if (out_target[k] == RSK_TARGET_NO_CANDIDATE) return RSK_NO_CANDIDATE;
        }
        return RSK_OK;
    }
    int *d_key = nullptr;
    unsigned short *d_code = nullptr;
    if (!compact) {
        RSK_TRY(plan->nodekey.reserve(NS * 4));
        d_key = plan->nodekey.as<int>();
    }
    if (compact) {
        RSK_TRY(plan->code.reserve((NS + (size_t)S) * 2));  // + row N, zeroed by the prep kernel
        d_code = plan->code.as<unsigned short>();
    }
    // the zero-case words, double-buffered: half h = zc_key[S] u64, zc_cnt[S],
    // zero on entry (cleared by the previous execute's prep kernel, or here
    // when the buffer is new or S changed); this execute's prep clears the
    // other half for the next one — no launch ahead of the prep kernel
    const size_t zc_half = zc_half_bytes(S);  // 16-B aligned halves (u64 atomics)
    RSK_TRY(ws_check_u64(N, S, 0));
    if (plan->zc_S != S) {
        RSK_TRY(plan->zc.reserve(2 * zc_half));
        RSK_HIP(hipMemsetAsync(plan->zc.ptr, 0, 2 * zc_half, ctx->stream));
        plan->zc_S = S;
        plan->zc_half = 0;
    }
    unsigned char *zc_base = plan->zc.as<unsigned char>();
    unsigned long long *d_zkey = reinterpret_cast<unsigned long long *>(zc_base + plan->zc_half * zc_half);
    int *d_zcnt = reinterpret_cast<int *>(d_zkey + S);
    unsigned *zc_other = reinterpret_cast<unsigned *>(zc_base + (plan->zc_half ^ 1) * zc_half);

    // K0: node state (codes and / or exact keys) + the zero case, launched below
    Prep16Args pa;
    pa.cap = d_cap;
    pa.use = d_use;
    pa.haz = d_haz;
    pa.N = N;
    pa.S = S;
    pa.code = d_code;
    pa.nodekey = d_key;
    pa.zc_cnt = d_zcnt;
    pa.zc_key = d_zkey;
    pa.zc_clear = zc_other;
    pa.clear_words = (int)(zc_half / 4);
    SideBufs sb;
    sb.assign = d_assign;
    sb.key = d_key;
    sb.code = d_code;
    sb.cap = d_cap;
    sb.use = d_use;
    sb.zcnt = d_zcnt;
    sb.zkey = d_zkey;
    sb.target = d_target;
    sb.score = d_score;
    sb.haz = d_haz;
    static const int ablate = RSK_ABLATION(RSK_ABLATE_TILE);
    // The compact side rows run inside the lean tile launch (car_fused16_kernel)
    // where they fit its footprint: their latency-bound workgroups share the
    // CUs with the memory-bound tiles instead of running alone.
    //   class 1 (33..128 neighbours): single-wave items interleaved with the tiles;
    //   classes >= kSideBig (above 128): 4-wave teams at the front of the grid,
    //     while the largest row's table fits the tile's LDS; otherwise on a side
    //     stream beside the tiles.
    const size_t lean_lds = tile16_lds_bytes(plan->rmax, 6, 0);
    int fuse_c = -1, fside_blocks = 0;
    SideArgs fsa, fba;
    std::memset(&fsa, 0, sizeof(fsa));
    std::memset(&fba, 0, sizeof(fba));
    const bool fuse_ok = compact && plan->T > 0 && S >= 64;
    if (fuse_ok && plan->side_end[1] > plan->side_beg[1]) {
        const SideGeom g = side16_geometry(plan->side_dmax[1], N);
        if (g.T == 1 && g.W == 4 && g.kB == 16 && 4 * g.lds_team <= lean_lds) {
            fsa = side16_class_args(plan, 1, sb, S, N);
            side16_apply_geometry(fsa, g);
            fsa.xcd_per = 0;
            fside_blocks = (int)ceil_div((int64_t)fsa.n_rows * fsa.nchunk, 4);
            fuse_c = 1;
        }
    }
    // the classes from kSideBig up to big_hi (exclusive) go into the fused grid
    int big_hi = kSideBig;
    if (fuse_ok)
        for (int c = kSideBig; c < kNumSide; ++c) {
            if (plan->side_end[c] == plan->side_beg[c]) continue;
            const SideGeom g = side16_geometry(plan->side_dmax[c], N, 4);
            if (g.kB != 16 || g.lds_team > lean_lds) break;
            big_hi = c + 1;
        }
    const bool fuse_big = big_hi > kSideBig;
    if (fuse_big) {  // rows [side_beg[big_hi - 1], side_end[kSideBig]): degree descending
        int dmax = 0;
        for (int c = kSideBig; c < big_hi; ++c) dmax = std::max(dmax, plan->side_dmax[c]);
        fba = side16_class_args(plan, kSideBig, sb, S, N);
        fba.items = plan->side_items.as<int>() + (size_t)plan->side_beg[big_hi - 1] * 4;
        fba.n_rows = plan->side_end[kSideBig] - plan->side_beg[big_hi - 1];
        side16_apply_geometry(fba, side16_geometry(dmax, N, 4));
        fba.xcd_per = 0;
    }
    // fused classes [lo, hi): class 0 (17..32, the wide path's kPairMax plans only) runs on its own
    const bool c0 = plan->side_end[0] > plan->side_beg[0];
    plan->fused_lo = c0 ? kNumSide : (fuse_c >= 0 || plan->side_end[1] == plan->side_beg[1] ? 0 : kSideBig);
    plan->fused_hi = std::max(big_hi, fuse_c >= 0 ? 2 : 1);
    if (!fuse_ok || (fuse_c < 0 && !fuse_big) || plan->fused_lo == kNumSide) plan->fused_lo = plan->fused_hi = 0;
    bool big_left = false;  // classes above the fused ones
    for (int c = big_hi; c < kNumSide; ++c) big_left = big_left || plan->side_end[c] > plan->side_beg[c];
    // The rows too big for the fused grid's side classes: when few cells
    // (config 4: 8 rows of 1,000-1,800 neighbours x 64 scenarios) and targets
    // only, a workgroup per (row, scenario) at the front of the fused grid
    // (direct16_block: packed LDS hash within the tile's LDS, exact cap - use) —
    // no side stream, no fork / join packets between the launches.
    DirectArgs fda;
    std::memset(&fda, 0, sizeof(fda));
    if (fuse_ok && big_left && !d_score) {
        const int b0 = plan->side_beg[kNumSide - 1], b1 = plan->side_end[big_hi];  // degree descending
        int dmax = 0;
        for (int c = big_hi; c < kNumSide; ++c) dmax = std::max(dmax, plan->side_dmax[c]);
        const int H = direct16_table(dmax, N, lean_lds);
        if (H && (int64_t)(b1 - b0) * S <= kDirectBigCells) {
            fda.rp = plan->drp.as<int>();
            fda.ci = plan->dci.as<int>();
            fda.rows = plan->drows.ptr ? plan->drows.as<int>() : nullptr;
            fda.items = plan->side_items.as<int>() + (size_t)b0 * 4;
            fda.istride = 4;
            fda.Q = b1 - b0;
            fda.assign = d_assign;
            fda.use = d_use;
            fda.cap = d_cap;
            fda.haz = d_haz;
            fda.S = S;
            fda.N = N;
            fda.H = H;
            fda.out_target = d_target;
            big_left = false;
        }
    }
    const bool fuse_direct = fda.Q > 0;
    // (S < 64: the tiles are short, the fork's events would cost more than the overlap)
    const bool big_fork = compact && big_left && plan->T > 0 && S >= 64;
    const int nfork = big_fork ? 1 : 0;
    if (big_fork) {
        // The rows too big for the fused grid run on a side stream from the
        // start, so they depend on no prep kernel and take CUs beside car_prep,
        // before the fused grid fills every slot and starves them.  Few cells
        // (config 4: 8 rows of 1,000-1,800 neighbours x 64 scenarios): a
        // workgroup per (row, scenario) counting that cell's neighbour nodes in
        // an LDS hash with exact cap - use (car_direct_kernel) — 512 workgroups
        // in flight instead of 8 pivot teams; otherwise the pivot teams with
        // node codes computed on the fly (max(cap) by each of their workgroups).
        RSK_TRY(aux_fork(ctx, nfork));
        const int b0 = plan->side_beg[kNumSide - 1], b1 = plan->side_end[big_hi];  // degree descending
        if (!d_score && (int64_t)(b1 - b0) * S <= kDirectBigCells) {  // (targets only: no scores)
            int dmax = 0;
            for (int c = big_hi; c < kNumSide; ++c) dmax = std::max(dmax, plan->side_dmax[c]);
            ScopedTimer tb(ctx, "car_side", ctx->aux[0]);
            RSK_TRY(launch_car_direct(ctx->aux[0], plan->drp.as<int>(), plan->dci.as<int>(),
                                      plan->drows.ptr ? plan->drows.as<int>() : nullptr, b1 - b0, d_assign, d_use,
                                      d_cap, d_haz, S, N, dmax, d_target, &plan->side_scratch,
                                      plan->side_items.as<int>() + (size_t)b0 * 4, 4));
        } else {
            RSK_TRY(launch_side16_classes(plan, ctx, ctx->aux[0], sb, S, N, big_hi, kNumSide, -1, true));
        }
        ScopedTimer tm(ctx, "car_prep");
        RSK_TRY(launch_prep(ctx->stream, pa));
    } else {
        {
            ScopedTimer tm(ctx, "car_prep");
            RSK_TRY(launch_prep(ctx->stream, pa));
        }
        if (compact && big_left)
            RSK_TRY(launch_side16_classes(plan, ctx, ctx->stream, sb, S, N, big_hi, kNumSide));
    }
    plan->zc_half ^= 1;  // the prep kernel is queued: it clears the other half for the next execute
    RSK_TRY(launch_side(plan, ctx, ctx->stream, sb, S, N, compact, fuse_c));
    const bool off32 = (int64_t)std::max(plan->P, plan->Q) * S * 4 < ((int64_t)1 << 32);
    if (plan->T > 0 && compact) {   // K1 tiles, 32-bit {code, node} cells
        Tile16Args a;
        std::memset(&a, 0, sizeof(a));
        a.img_pods = plan->img_pods.as<int>();
        a.meta = plan->meta.as<int>();
        a.recs = plan->recs.as<int>();
        a.assign = d_assign;
        a.code = d_code;
        a.cap = d_cap;
        a.use = d_use;
        a.zc_cnt = d_zcnt;
        a.zc_key = d_zkey;
        a.out_target = d_target;
        a.out_score = d_score;
        a.S = S;
        a.N = N;
        a.T = plan->T;
        a.n_assign = (unsigned)std::min<size_t>(PS_, UINT32_MAX);
        a.n_out = (unsigned)std::min<size_t>(QS, UINT32_MAX);
        a.n_pods = (unsigned)plan->n_img_pods;
        a.n_recs = (unsigned)plan->n_recs;
        a.n_key = (unsigned)NS;
        const int SL = std::min(next_pow2(S), 64);
        a.lsl = 0;
        while ((1 << a.lsl) < SL) ++a.lsl;
        a.ablate = ablate;
        a.rec_cap = (plan->recmax + 3) & ~3;
        a.img_cells = (plan->rmax * SL + 3) & ~3;
        const size_t lds = tile16_lds_bytes(plan->rmax, a.lsl, a.rec_cap);
        RSK_CHECK(plan->recmax <= kTileRecInts, "tile records exceed %d ints", kTileRecInts);
        // S >= 64: 64-scenario tiles (fused with the side rows that fit);
        // S < 64: one generic kernel scores every tile
        ScopedTimer tm(ctx, "car_tile");
        a.tile0 = 0;
        const int64_t units = ceil_div(S, SL) * plan->T;
        a.xcd_per = (int)ceil_div(units, 8);
        const int64_t blocks = 8 * (int64_t)a.xcd_per;
        RSK_CHECK(blocks < INT32_MAX, "tile grid too large");
        if (fuse_c >= 0 || fuse_big || fuse_direct)
            RSK_TRY(launch_fused16(ctx->stream, a, fsa, fside_blocks, fba, fda, d_score != nullptr, off32,
                                   (unsigned)blocks, lds));
        else
            RSK_TRY(launch_tile16(ctx->stream, a, d_score != nullptr, off32, (unsigned)blocks, lds));
    } else if (plan->T > 0) {   // K1 tiles, wide {node, key} pairs
        TileArgs a;
        std::memset(&a, 0, sizeof(a));
        a.img_pods = plan->img_pods.as<int>();
        a.meta = plan->meta.as<int>();
        a.recs = plan->recs.as<int>();
        a.assign = d_assign;
        a.nodekey = d_key;
        a.zc_cnt = d_zcnt;
        a.zc_key = d_zkey;
        a.out_target = d_target;
        a.out_score = d_score;
        a.S = S;
        a.N = N;
        a.T = plan->T;
        a.rmax = plan->rmax;
        a.n_assign = (unsigned)std::min<size_t>(PS_, UINT32_MAX);
        a.n_out = (unsigned)std::min<size_t>(QS, UINT32_MAX);
        a.n_pods = (unsigned)plan->n_img_pods;
        a.n_recs = (unsigned)plan->n_recs;
        a.n_key = (unsigned)NS;
        const int SL = std::min(next_pow2(S), 32);
        a.lsl = 0;
        while ((1 << a.lsl) < SL) ++a.lsl;
        a.ablate = ablate;
        a.rec_cap = (plan->recmax + 3) & ~3;
        const int cells = plan->rmax * SL;
        const size_t lds = ((size_t)((2 * cells + 3) & ~3) + a.rec_cap + 4) * 4;
        RSK_CHECK(lds <= 160 * 1024 && plan->recmax <= kTileRecInts, "tile image needs %zu B of LDS", lds);
        const int64_t units = ceil_div(S, SL) * plan->T;
        a.xcd_per = (int)ceil_div(units, 8);
        const int64_t blocks = 8 * (int64_t)a.xcd_per;
        RSK_CHECK(blocks < INT32_MAX, "tile grid too large");
        using TileKern = void (*)(TileArgs);
        static const TileKern kerns[4] = {&car_tile_kernel<false, false>, &car_tile_kernel<false, true>,
                                          &car_tile_kernel<true, false>, &car_tile_kernel<true, true>};
        const TileKern kern = kerns[(d_score ? 2 : 0) + (off32 ? 1 : 0)];
        if (lds > 64 * 1024)
            RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        ScopedTimer tm(ctx, "car_tile");
        kern<<<dim3((unsigned)blocks), dim3(kTileThreads), lds, ctx->stream>>>(a);
        RSK_HIP(hipGetLastError());
    }
    if (nfork) RSK_TRY(aux_join(ctx, nfork));
#ifdef RSK_DEBUG_BOUNDS
    {
        unsigned flags_h = 0, zero = 0;
        RSK_HIP(hipStreamSynchronize(ctx->stream));
        RSK_HIP(hipMemcpyFromSymbol(&flags_h, HIP_SYMBOL(rsk_dbg_flags), 4));
        RSK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(rsk_dbg_flags), &zero, 4));
        flags_h |= tile16_debug_take();
        RSK_CHECK(flags_h == 0, "debug bounds violation flags=0x%x (1 out, 2 pods, 4 assign, 8 nodekey, 16 recs)",
                  flags_h);
    }
#endif
    if (!dev) {
        RSK_TRY(copy_back(ctx, out_target, d_target, QS * 4, false));
        if (out_score) RSK_TRY(copy_back(ctx, out_score, d_score, QS * 4, false));
        RSK_HIP(hipStreamSynchronize(ctx->stream));
        for (size_t k = 0; k < QS; ++k)
            if (out_target[k] == RSK_TARGET_NO_CANDIDATE) return RSK_NO_CANDIDATE;
    }
    return RSK_OK;
}

int rsk_car_place(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, int32_t P, const int32_t *assign,
                  int32_t S, const int32_t *cap_cpu, const int32_t *use_cpu, const uint8_t *hazard, int32_t N,
                  const int32_t *rows, int32_t Q, int32_t *out_target, int32_t *out_score, uint32_t flags) {
    rsk_car_plan *plan = nullptr;
    RSK_TRY(rsk_car_plan_create(ctx, row_ptr, col_idx, P, rows, Q, &plan));
    const int rc = rsk_car_plan_execute(plan, assign, S, cap_cpu, use_cpu, hazard, N, out_target, out_score, flags);
    if (rc != RSK_OK && rc != RSK_NO_CANDIDATE) {
        std::string keep = last_error();
        rsk_car_plan_destroy(plan);
        set_error("%s", keep.c_str());
        return rc;
    }
    rsk_car_plan_destroy(plan);
    return rc;
}

}  // extern "C"
