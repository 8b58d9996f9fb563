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
// Kernels (one HIP stream, all integer, no atomics on the decision path):
//   car_prep_kernel   nodekey[n*S+s] = hazard ? KEY_HAZ : cap[n]-use[n*S+s]
//                     (one gather word per node later) + the zero case.
//   car_tile_kernel   deg <= 16 rows, grouped into tiles of <= 128 rows whose
//                     neighbours (<= 160 image rows) are staged once per
//                     scenario chunk in LDS together with their node keys;
//                     scoring then runs from LDS with per-degree-class scorers.
//   car_mid_kernel    17 <= deg <= 64: per-lane bitonic sort of the neighbour
//                     node ids in registers + run-length scan.
//   car_heavy_kernel  deg > 64: node ids staged in LDS, per-wave LDS count
//                     tables / hash, coalesced lookups, cross-lane reduce.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <unordered_map>
#include <vector>

#include "rsk_common.h"

namespace rsk {

constexpr int kKeyHaz = INT_MIN;  // cap - use never reaches INT_MIN (both in [0, 2^31))
constexpr int kMaxDegree = 4096;
constexpr int kLightMax = 16;                      // LDS-tile rows: deg <= 16
constexpr int kMidMax = 64;                        // sorted-register rows: 17 <= deg <= 64
constexpr int kNumMid = 2;                         // buckets D = 32, 64
constexpr int kMidW[kNumMid] = {36, 68};           // record ints: oi, d, nb[D], pad to x4
constexpr int kNumHeavy = 3;                       // (64,512] (512,2048] (2048,4096]
constexpr int kHeavyMax[kNumHeavy] = {512, 2048, 4096};

// Light-row tiles.
constexpr int kTileOwners = 128;                   // max rows scored per tile (plan default: 64)
constexpr int kTileRows = 160;                     // max image rows (distinct neighbours) per tile
constexpr int kTileThreads = 256;                  // pipelined kernel geometry
constexpr int kTileWaves = kTileThreads / 64;
constexpr int kNumCls = 5;                         // degree classes d = 1, 2, 3-4, 5-8, 9-16
constexpr int kClsW[kNumCls] = {2, 2, 4, 8, 12};   // record ints
constexpr int kMetaW = 12;                         // tile meta ints (see TileArgs)

struct CarState {
    int bc;  // best count (max score); 0 = no non-hazard neighbour node
    int br;  // remaining CPU of the best node
    int bn;  // best node index
    int nm;  // neighbour entries whose count == bc  (= bc * |best|)
};

__device__ __forceinline__ void st_init(CarState &st) {
    st.bc = 0;
    st.br = INT_MIN;
    st.bn = INT_MAX;
    st.nm = 0;
}

__device__ __forceinline__ void st_add(CarState &st, int c, int r, int n) {
    if (c > st.bc) {
        st.bc = c; st.br = r; st.bn = n; st.nm = 1;
    } else if (c == st.bc) {
        st.nm += 1;
        if (r > st.br || (r == st.br && n < st.bn)) { st.br = r; st.bn = n; }
    }
}

__device__ __forceinline__ CarState st_combine(CarState a, const CarState &b) {
    if (b.bc > a.bc) return b;
    if (b.bc < a.bc) return a;
    a.nm += b.nm;
    if (b.br > a.br || (b.br == a.br && b.bn < a.bn)) { a.br = b.br; a.bn = b.bn; }
    return a;
}

__device__ __forceinline__ CarState st_shfl_xor(const CarState &st, int off) {
    CarState o;
    o.bc = __shfl_xor(st.bc, off, 64);
    o.br = __shfl_xor(st.br, off, 64);
    o.bn = __shfl_xor(st.bn, off, 64);
    o.nm = __shfl_xor(st.nm, off, 64);
    return o;
}

// Candidate key of the sorted-register scorer: lexicographic (count, remaining
// CPU, -node) as one u64 — count 7 bits (<= 64), remaining CPU 32 bits (sign
// flipped), 0x1ffffff - node 25 bits (N < 2^25).  0 = no candidate.
constexpr int kNodeBits = 25;
constexpr unsigned kNodeMask = (1u << kNodeBits) - 1u;
__device__ __forceinline__ unsigned long long pack_cand(int c, int rem, int n) {
    return ((unsigned long long)c << (32 + kNodeBits)) |
           ((unsigned long long)((unsigned)rem ^ 0x80000000u) << kNodeBits) |
           (unsigned long long)(kNodeMask - (unsigned)n);
}
__device__ __forceinline__ int cand_count(unsigned long long k) { return (int)(k >> (32 + kNodeBits)); }
__device__ __forceinline__ CarState cand_state(unsigned long long best, int nm) {
    CarState st;
    st.bc = cand_count(best);
    st.nm = nm;
    st.br = (int)((unsigned)(best >> kNodeBits) ^ 0x80000000u);
    st.bn = (int)(kNodeMask - (unsigned)(best & kNodeMask));
    return st;
}

__device__ __forceinline__ unsigned long long zc_pack(int rem, int n) {
    return ((unsigned long long)((unsigned)rem ^ 0x80000000u) << 32) | (unsigned long long)(~(unsigned)n);
}

// The per-scenario zero case (car_prep_kernel), loaded once per lane.
struct ZeroCase {
    int cnt;                  // non-hazard nodes in the scenario
    unsigned long long key;   // packed (cap-use, ~node) max over them
};

__device__ __forceinline__ ZeroCase load_zc(const int *__restrict__ zc_cnt, const unsigned long long *__restrict__ zc_key,
                                            int s) {
    ZeroCase z;
    z.cnt = zc_cnt[s];
    z.key = zc_key[s];
    return z;
}

// rescheduling.py:199-214 when no neighbour node is a candidate (max score 0):
// every non-hazard node ties; `max` raises on an empty candidate list.
__device__ __forceinline__ int zero_target(const ZeroCase &z, int &score) {
    if (z.cnt == 0) { score = -1; return RSK_TARGET_NO_CANDIDATE; }
    const int n = (int)(~(unsigned)(z.key & 0xffffffffull));
    const int rem = (int)((unsigned)(z.key >> 32) ^ 0x80000000u);
    score = 0;
    if (z.cnt == 1) return n;
    return rem >= 0 ? n : RSK_TARGET_NONE;
}

// rescheduling.py:199-214 applied to the reduced state.
__device__ __forceinline__ int car_finalize(const CarState &st, const ZeroCase &z, int &score) {
    if (st.bc == 0) return zero_target(z, score);
    score = st.bc;
    if (st.nm == st.bc) return st.bn;
    return st.br >= 0 ? st.bn : RSK_TARGET_NONE;
}

// Load with a 32-bit element index: the base stays in SGPRs and the offset is
// one VGPR (global_load saddr form) instead of a 64-bit address pair per
// in-flight load.  Callers guarantee index * 4 < 2^32.
__device__ __forceinline__ int ld32(const int *__restrict__ base, unsigned idx) {
    return *reinterpret_cast<const int *>(reinterpret_cast<const char *>(base) + (idx << 2));
}

// Bounds-checked debug build (make debug -> librsk_dbg.so, -DRSK_DEBUG_BOUNDS):
// every tile-kernel global access checks its element index against the buffer
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
// K0: packed node key + per-scenario zero case.
// Thread t -> (scenario s = t % S, node chunk t / S): consecutive lanes read
// consecutive scenarios of one node, i.e. coalesced rows of use / hazard.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void car_prep_kernel(const int *__restrict__ cap, const int *__restrict__ use,
                                                       const uint8_t *__restrict__ haz, int N, int S, int npb,
                                                       unsigned total, int *__restrict__ nodekey,
                                                       int *__restrict__ zc_cnt,
                                                       unsigned long long *__restrict__ zc_key) {
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (t >= total) return;
    const int s = (int)(t % (unsigned)S);
    const int n0 = (int)(t / (unsigned)S) * npb;
    const int n1 = min(N, n0 + npb);
    int cnt = 0;
    unsigned long long best = 0;
    for (int n = n0; n < n1; ++n) {
        const size_t idx = (size_t)n * S + s;
        const int h = haz[idx];
        const int key = h ? kKeyHaz : cap[n] - use[idx];
        nodekey[idx] = key;
        if (!h) {
            ++cnt;
            const unsigned long long pk = zc_pack(key, n);
            best = pk > best ? pk : best;
        }
    }
    if (cnt) {
        atomicAdd(&zc_cnt[s], cnt);
        atomicMax(&zc_key[s], best);
    }
}

// ---------------------------------------------------------------------------
// K1: light rows (deg <= 16) in LDS tiles.
//
// The plan groups the light rows (in DFS order of the relation graph, so a
// row's neighbours are mostly its tile-mates) into tiles of <= 128 rows whose
// distinct neighbours — the tile's image rows — number <= 160.  Workgroup =
// (tile, chunk of SL = 2^lsl scenarios), 4 waves:
//   phase 1  every image row's SL-scenario slice of assign (SL*4 contiguous
//            bytes; each row leaves HBM once per chunk) -> registers, its node
//            key per scenario gathered from nodekey (L2), both -> LDS
//            nimg[row][SL], kimg[row][SL]; the tile's records -> LDS.
//   phase 2  lanes = (record slot, scenario).  A record is
//            [out_row, (deg,) neighbour image rows packed 2 x u16 per int];
//            scorers specialised per degree class read node + key from LDS and
//            store one target word per lane (SL*4 contiguous bytes per row).
// Meta per tile (kMetaW ints): img_off, nrows, rec_off, rec_ints,
// n[5] records per class, o4, o8, o16 class offsets (ints, 4-aligned).
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
    int ablate;              // profiling only (RSK_ABLATE_TILE): 1 skip image load, 2 skip scoring
    int order;               // 0 chunk-major, 1 tile-major grid (RSK_TILE_ORDER)
    unsigned n_assign, n_out, n_pods, n_recs, n_key, n_meta;  // element counts (debug bounds build)
};
// records -> LDS in two int4 copies per thread: NT * 8 >= owners * 12 + 2 (checked by the host)

// Element offsets: 32-bit (saddr form, one VGPR) when every offset * 4 < 2^32.
template <bool kOff32>
__device__ __forceinline__ size_t cell(unsigned i, unsigned S, unsigned s) {
    if (kOff32) return (size_t)((i * S + s) << 2);
    return ((size_t)i * S + s) << 2;
}
template <bool kOff32>
__device__ __forceinline__ void st_cell(int *base, unsigned i, unsigned S, unsigned s, int v) {
    *reinterpret_cast<int *>(reinterpret_cast<char *>(base) + cell<kOff32>(i, S, s)) = v;
}

// Per-lane constants of the scoring phase.  Lanes past the last scenario (a
// partial chunk) and record slots past a class's end redo a valid cell — the
// last scenario / the last record — and store the identical value again, so
// no load, LDS access or store is ever guarded by a branch.
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

__device__ __forceinline__ int2 img_at(const int2 *img, int row, int lsl, int col) { return img[(row << lsl) + col]; }

// d == 1: the neighbour's node is the single best unless hazard (zero case).
template <int U, bool kScore, bool kOff32, int NW = kTileWaves>
__device__ __forceinline__ void tile_d1(const TileArgs &a, const int2 *img, const int *rec, int n, const TileLane &L,
                                        int wave) {
    const int step = NW * L.PS;
    const int2 *r2 = reinterpret_cast<const int2 *>(rec);
    for (int b0 = wave * L.PS; b0 < n; b0 += step * U) {
        int2 r[U], e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = r2[min(b0 + u * step + L.slot, n - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) e[u] = img_at(img, r[u].y, a.lsl, L.col);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool h = e[u].y == kKeyHaz;
            tile_emit<kScore, kOff32>(a, r[u].x, L, h ? L.zt : e[u].x, h ? L.zs : 1);
        }
    }
}

// d == 2: same node -> score 2; one hazard -> the other; two distinct
// candidates -> tie of two: larger remaining CPU (then lower index), None if < 0.
template <int U, bool kScore, bool kOff32, int NW = kTileWaves>
__device__ __forceinline__ void tile_d2(const TileArgs &a, const int2 *img, const int *rec, int n, const TileLane &L,
                                        int wave) {
    const int step = NW * L.PS;
    const int2 *r2 = reinterpret_cast<const int2 *>(rec);
    for (int b0 = wave * L.PS; b0 < n; b0 += step * U) {
        int2 r[U], e0[U], e1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = r2[min(b0 + u * step + L.slot, n - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            e0[u] = img_at(img, r[u].y & 0xffff, a.lsl, L.col);
            e1[u] = img_at(img, (int)((unsigned)r[u].y >> 16), a.lsl, L.col);
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

// 0 or 3 <= d <= D: pairwise equality counts in registers, then the
// lexicographic (count, key, -node) maximum over the candidates in 32-bit steps.
template <int D, int W, bool kScore, bool kOff32, int NW = kTileWaves>
__device__ __forceinline__ void tile_dn(const TileArgs &a, const int2 *img, const int *rec, int n, const TileLane &L,
                                        int wave) {
    const int step = NW * L.PS;
    for (int b0 = wave * L.PS; b0 < n; b0 += step) {
        const int4 *r4 = reinterpret_cast<const int4 *>(rec + min(b0 + L.slot, n - 1) * W);
        int r[W];
#pragma unroll
        for (int w = 0; w < W / 4; ++w) {
            const int4 x = r4[w];
            r[4 * w] = x.x; r[4 * w + 1] = x.y; r[4 * w + 2] = x.z; r[4 * w + 3] = x.w;
        }
        const int d = r[1];
        int nd[D], ky[D], c[D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const unsigned pr = (unsigned)r[2 + j / 2];
            const int2 e = img_at(img, (j & 1) ? (int)(pr >> 16) : (int)(pr & 0xffffu), a.lsl, L.col);
            // padding entries (j >= d) read row 0: masked out of the counts
            // (a node id no real entry can hold) and of the candidates
            nd[j] = j < d ? e.x : -1 - j;
            ky[j] = j < d ? e.y : kKeyHaz;
            c[j] = 1;
        }
#pragma unroll
        for (int j = 1; j < D; ++j)
#pragma unroll
            for (int i2 = 0; i2 < j; ++i2) {
                const int eq = nd[j] == nd[i2];
                c[j] += eq;
                c[i2] += eq;
            }
        int M = 0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            c[j] = ky[j] == kKeyHaz ? 0 : c[j];
            M = max(M, c[j]);
        }
        int kb = INT_MIN;
#pragma unroll
        for (int j = 0; j < D; ++j) kb = max(kb, c[j] == M ? ky[j] : INT_MIN);
        int nb = INT_MAX, nm = 0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const bool m = c[j] == M;
            nb = min(nb, (m && ky[j] == kb) ? nd[j] : INT_MAX);
            nm += m;
        }
        const int tt = nm == M ? nb : (kb >= 0 ? nb : RSK_TARGET_NONE);
        tile_emit<kScore, kOff32>(a, r[0], L, M == 0 ? L.zt : tt, M == 0 ? L.zs : M);
    }
}

// Phase 1: image rows -> LDS as {node, key} pairs.  kVec: SL >= 4 and S % 4 == 0
// (16-B loads of 4 scenarios).  Elements past the end redo the last element
// (identical LDS writes), so nothing is guarded.
template <bool kVec, bool kOff32, int NT>
__device__ __forceinline__ void tile_load_image(const TileArgs &a, int2 *img, int img_off, int nrows, int s0) {
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    const int *__restrict__ pods = a.img_pods + img_off;
    const char *__restrict__ asg = reinterpret_cast<const char *>(a.assign);
    constexpr int kB = 5;
    if (kVec) {
        const int lq = a.lsl - 2;  // 16-B slots per row = SL / 4
        const int qm = (1 << lq) - 1;
        const int total = nrows << lq;
        for (int b = 0; b < total; b += NT * kB) {
            int e[kB], pod[kB];
            int4 v[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                e[u] = min(b + u * NT + (int)threadIdx.x, total - 1);
                pod[u] = pods[e[u] >> lq];
            }
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const unsigned s = (unsigned)min(s0 + ((e[u] & qm) << 2), (int)S - 4);
                v[u] = *reinterpret_cast<const int4 *>(asg + cell<kOff32>((unsigned)pod[u], S, s));
            }
            int k[kB][4];
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int s = s0 + ((e[u] & qm) << 2);
                const int nn[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int x = 0; x < 4; ++x) {
                    const bool ok = (unsigned)nn[x] < N && s + x < (int)S;
                    const int key = ld32(a.nodekey, ok ? (unsigned)nn[x] * S + (unsigned)(s + x) : 0u);
                    k[u][x] = ok ? key : kKeyHaz;
                }
            }
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                int4 *dst = reinterpret_cast<int4 *>(img + ((e[u] >> lq) << a.lsl) + ((e[u] & qm) << 2));
                dst[0] = make_int4(v[u].x, k[u][0], v[u].y, k[u][1]);
                dst[1] = make_int4(v[u].z, k[u][2], v[u].w, k[u][3]);
            }
        }
    } else {
        const int total = nrows << a.lsl;
        const int msk = (1 << a.lsl) - 1;
        for (int b = 0; b < total; b += NT * kB) {
            int e[kB], pod[kB], v[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                e[u] = min(b + u * NT + (int)threadIdx.x, total - 1);
                pod[u] = pods[e[u] >> a.lsl];
            }
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const unsigned s = (unsigned)min(s0 + (e[u] & msk), (int)S - 1);
                v[u] = *reinterpret_cast<const int *>(asg + cell<kOff32>((unsigned)pod[u], S, s));
            }
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int s = s0 + (e[u] & msk);
                const bool ok = (unsigned)v[u] < N && s < (int)S;
                const int key = ld32(a.nodekey, ok ? (unsigned)v[u] * S + (unsigned)s : 0u);
                img[e[u]] = make_int2(v[u], ok ? key : kKeyHaz);
            }
        }
    }
}

template <bool kVec, bool kScore, bool kOff32, int NT>
__global__ __launch_bounds__(NT) void car_tile_kernel(TileArgs a) {
    constexpr int NW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) int lds[];  // img {node,key} [rmax][SL], then records
    // chunk-major (default: concurrent workgroups share a chunk's nodekey
    // slice in L2) or tile-major (a tile's chunks back to back: DRAM locality)
    const int nchunk = (a.S + (1 << a.lsl) - 1) >> a.lsl;
    const int tile = a.order ? blockIdx.x / nchunk : blockIdx.x % a.T;
    const int chunk = a.order ? blockIdx.x % nchunk : blockIdx.x / a.T;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int SL = 1 << a.lsl;
    const int s0 = chunk * SL;
    int2 *img = reinterpret_cast<int2 *>(lds);
    int *rec = lds + ((2 * a.rmax * SL + 3) & ~3);  // 16-B aligned for the int4 record reads
    const int *m = a.meta + (size_t)tile * kMetaW;
    const int img_off = m[0], nrows = m[1], rec_off = m[2], rec_ints = m[3];

    // records -> LDS: at most 2 int4 per thread (static_assert above), clamped
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int i = min((int)threadIdx.x * 4 + k * NT * 4, rec_ints - 4);
        *reinterpret_cast<int4 *>(rec + i) = *reinterpret_cast<const int4 *>(a.recs + rec_off + i);
    }
    if (!(a.ablate & 1) && nrows > 0) tile_load_image<kVec, kOff32, NT>(a, img, img_off, nrows, s0);

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
    __syncthreads();
    if (a.ablate & 2) return;  // profiling ablation: no scoring (results are wrong)
    const int n1 = m[4], n2 = m[5], n4 = m[6], n8 = m[7], n16 = m[8];
    const int o4 = m[9], o8 = m[10], o16 = m[11];
    if (n1) tile_d1<4, kScore, kOff32, NW>(a, img, rec, n1, L, wave);
    if (n2) tile_d2<2, kScore, kOff32, NW>(a, img, rec + 2 * n1, n2, L, wave);
    if (n4) tile_dn<4, 4, kScore, kOff32, NW>(a, img, rec + o4, n4, L, wave);
    if (n8) tile_dn<8, 8, kScore, kOff32, NW>(a, img, rec + o8, n8, L, wave);
    if (n16) tile_dn<16, 12, kScore, kOff32, NW>(a, img, rec + o16, n16, L, wave);
}

// ---------------------------------------------------------------------------
// K1p: the same light-row tiles as a persistent, wave-specialised pipeline
// (S % 4 == 0, SL = 32).  One workgroup per CU walks the items (tile, chunk)
// blockIdx, blockIdx + gridDim, ... (chunk-major, so concurrent items share a
// chunk's nodekey slice in L2).  Per stage t (one s_barrier each):
//   loader waves (kLoadW)  write item t+1 into LDS buffer (t+1)&1 from the
//                          registers filled earlier, then issue the gathers of
//                          item t+2 (node keys, records, zero case), the assign
//                          loads of item t+3 and the image pod ids of item t+4;
//   scorer waves (kScoreW) score item t from buffer t&1 and store its targets.
// Loaders never store and scorers never load from global memory, so neither
// kind waits on the other's vector-memory traffic (vmcnt retires in issue
// order): a loader's waits are exactly the loads it issued one stage earlier,
// and a scorer never waits on its stores.  Out-of-range items are clamped to
// a valid one (their loads are harmless repeats; nothing is scored).
// ---------------------------------------------------------------------------
constexpr int kPipeSL = 32, kPipeLsl = 5;
constexpr int kLoadW = 4, kScoreW = 8;
constexpr int kPipeThreads = (kLoadW + kScoreW) * 64;
constexpr int kLdThreads = kLoadW * 64;
constexpr int kLdSlots = (kTileRows * (kPipeSL / 4) + kLdThreads - 1) / kLdThreads;  // int4 image slots per loader
constexpr int kLdRec = (kTileOwners * 12 / 4 + kLdThreads - 1) / kLdThreads;         // int4 record slots per loader
constexpr int kBufHead = 80;                                                          // meta[12], zt[32], zs[32], pad
constexpr int kBufInts = kBufHead + kTileRows * kPipeSL * 2 + kTileOwners * 12;

struct PipeArgs {
    TileArgs t;
    int items;  // T * chunks
};

struct LdA {  // assign slices of one item (this loader thread's slots)
    int4 v[kLdSlots];
};
struct LdK {  // node keys of one item + its records + zero case
    int k[kLdSlots][4];
    int4 rec[kLdRec];
    int zt, zs;
};
struct LdP {
    int pod[kLdSlots];
};

__device__ __forceinline__ int pipe_item(const PipeArgs &a, int j) {
    // j-th item of this workgroup, clamped into [first, last] of its own items
    const int n = (a.items - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    j = min(max(j, 0), n - 1);
    return (int)blockIdx.x + j * (int)gridDim.x;
}

// Tile meta read through the constant address space: the plan never changes
// during a launch, so these become scalar loads (lgkmcnt) instead of vector
// loads that would queue behind the loaders' in-flight gathers.
typedef const __attribute__((address_space(4))) int *cint_ptr;
__device__ __forceinline__ cint_ptr const_ptr(const int *p) { return (cint_ptr)(uintptr_t)p; }

struct ItemGeo {
    int tile, s0, img_off, total, rec_off, rec_ints;
    cint_ptr meta;
};
__device__ __forceinline__ ItemGeo pipe_geo(const PipeArgs &a, int item) {
    ItemGeo g;
    g.tile = item % a.t.T;
    g.s0 = (item / a.t.T) * kPipeSL;
    g.meta = const_ptr(a.t.meta) + (size_t)g.tile * kMetaW;
    g.img_off = g.meta[0];
    g.total = g.meta[1] << 3;  // 8 int4 slots per row
    g.rec_off = g.meta[2];
    g.rec_ints = g.meta[3];
    return g;
}

__device__ __forceinline__ int ld_slot(int u, int lt, int total) { return min(u * kLdThreads + lt, max(total - 1, 0)); }

__device__ __forceinline__ void ld_issue_p(const PipeArgs &a, int item, int lt, LdP &p) {
    const ItemGeo g = pipe_geo(a, item);
#pragma unroll
    for (int u = 0; u < kLdSlots; ++u)
        p.pod[u] = a.t.img_pods[RSK_BOUND(g.img_off + (ld_slot(u, lt, g.total) >> 3), a.t.n_pods, 2u)];
}

template <bool kOff32>
__device__ __forceinline__ void ld_issue_a(const PipeArgs &a, int item, int lt, const LdP &p, LdA &A) {
    const ItemGeo g = pipe_geo(a, item);
    const unsigned S = (unsigned)a.t.S;
    const char *asg = reinterpret_cast<const char *>(a.t.assign);
#pragma unroll
    for (int u = 0; u < kLdSlots; ++u) {
        const int e = ld_slot(u, lt, g.total);
        const unsigned s = (unsigned)min(g.s0 + ((e & 7) << 2), (int)S - 4);
#ifdef RSK_DEBUG_BOUNDS
        if ((size_t)(unsigned)p.pod[u] * S + s + 3 >= a.t.n_assign) { atomicOr(&rsk_dbg_flags, 4u); A.v[u] = make_int4(0, 0, 0, 0); continue; }
#endif
        A.v[u] = *reinterpret_cast<const int4 *>(asg + cell<kOff32>((unsigned)p.pod[u], S, s));
    }
}

__device__ __forceinline__ void ld_issue_k(const PipeArgs &a, int item, int lt, const LdA &A, LdK &K, bool keys) {
    const ItemGeo g = pipe_geo(a, item);
    const int S = a.t.S;
    const unsigned N = (unsigned)a.t.N;
#pragma unroll
    for (int u = 0; keys && u < kLdSlots; ++u) {
        const int e = ld_slot(u, lt, g.total);
        const int s = g.s0 + ((e & 7) << 2);
        const int nn[4] = {A.v[u].x, A.v[u].y, A.v[u].z, A.v[u].w};
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            const bool ok = (unsigned)nn[x] < N && s + x < S;
            const int key = ld32(a.t.nodekey, RSK_BOUND(ok ? (unsigned)nn[x] * (unsigned)S + (unsigned)(s + x) : 0u, a.t.n_key, 8u));
            K.k[u][x] = ok ? key : kKeyHaz;
        }
    }
#pragma unroll
    for (int u = 0; u < kLdRec; ++u) {
        const int i = min(4 * (u * kLdThreads + lt), g.rec_ints - 4);
        K.rec[u] = *reinterpret_cast<const int4 *>(a.t.recs + RSK_BOUND(g.rec_off + i + 3, a.t.n_recs, 16u) - 3);
    }
    const int s = min(g.s0 + (lt & (kPipeSL - 1)), S - 1);
    int zs;
    K.zt = zero_target(load_zc(a.t.zc_cnt, a.t.zc_key, s), zs);
    K.zs = zs;
}

__device__ __forceinline__ void ld_write(const PipeArgs &a, int item, int lt, const LdA &A, const LdK &K, int *buf) {
    const ItemGeo g = pipe_geo(a, item);
    int2 *img = reinterpret_cast<int2 *>(buf + kBufHead);
    int *rec = buf + kBufHead + kTileRows * kPipeSL * 2;
#pragma unroll
    for (int u = 0; u < kLdSlots; ++u) {
        const int e = ld_slot(u, lt, g.total);
        int4 *dst = reinterpret_cast<int4 *>(img + ((e >> 3) << kPipeLsl) + ((e & 7) << 2));
        dst[0] = make_int4(A.v[u].x, K.k[u][0], A.v[u].y, K.k[u][1]);
        dst[1] = make_int4(A.v[u].z, K.k[u][2], A.v[u].w, K.k[u][3]);
    }
#pragma unroll
    for (int u = 0; u < kLdRec; ++u) {
        const int i = min(4 * (u * kLdThreads + lt), g.rec_ints - 4);
        *reinterpret_cast<int4 *>(rec + i) = K.rec[u];
    }
    if (lt == 0) {
#pragma unroll
        for (int i = 0; i < kMetaW; ++i) buf[i] = g.meta[i];
    }
    if (lt < kPipeSL) {
        buf[kMetaW + lt] = K.zt;
        buf[kMetaW + kPipeSL + lt] = K.zs;
    }
}

__device__ __forceinline__ void pipe_barrier() {
    // LDS writes / reads of this stage complete, then the workgroup barrier;
    // never a vmcnt wait (loads and stores stay in flight across stages)
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One loader stage t, register sets named by role.
template <bool kOff32>
__device__ __forceinline__ void ld_stage(const PipeArgs &a, int t, int lt, int *bufs, LdA &A1, LdK &K1, LdA &A2,
                                         LdK &K2, LdA &A3, LdP &P3, LdP &P4) {
    // compiler fences keep the issue order = the order the next stage waits in
    ld_write(a, pipe_item(a, t + 1), lt, A1, K1, bufs + ((t + 1) & 1) * kBufInts);
    asm volatile("" ::: "memory");
    ld_issue_k(a, pipe_item(a, t + 2), lt, A2, K2, !(a.t.ablate & 1));
    asm volatile("" ::: "memory");
    if (!(a.t.ablate & 1)) ld_issue_a<kOff32>(a, pipe_item(a, t + 3), lt, P3, A3);
    asm volatile("" ::: "memory");
    ld_issue_p(a, pipe_item(a, t + 4), lt, P4);
    pipe_barrier();
}

template <bool kScore, bool kOff32>
__device__ __forceinline__ void sc_stage(const PipeArgs &a, int t, int n_items, int sw, int lane, int *bufs) {
    if (t >= 0 && t < n_items && !(a.t.ablate & 2)) {
        const int *buf = bufs + (t & 1) * kBufInts;
        const int2 *img = reinterpret_cast<const int2 *>(buf + kBufHead);
        const int *rec = buf + kBufHead + kTileRows * kPipeSL * 2;
        const int item = pipe_item(a, t);
        const int s0 = (item / a.t.T) * kPipeSL;
        TileLane L;
        L.PS = 64 / kPipeSL;
        L.slot = lane >> kPipeLsl;
        L.s = min(s0 + (lane & (kPipeSL - 1)), a.t.S - 1);
        L.col = L.s - s0;
        L.zt = buf[kMetaW + L.col];
        L.zs = buf[kMetaW + kPipeSL + L.col];
        const int n1 = buf[4], n2 = buf[5], n4 = buf[6], n8 = buf[7], n16 = buf[8];
        const int o4 = buf[9], o8 = buf[10], o16 = buf[11];
        if (n1) tile_d1<4, kScore, kOff32, kScoreW>(a.t, img, rec, n1, L, sw);
        if (n2) tile_d2<2, kScore, kOff32, kScoreW>(a.t, img, rec + 2 * n1, n2, L, sw);
        if (n4) tile_dn<4, 4, kScore, kOff32, kScoreW>(a.t, img, rec + o4, n4, L, sw);
        if (n8) tile_dn<8, 8, kScore, kOff32, kScoreW>(a.t, img, rec + o8, n8, L, sw);
        if (n16) tile_dn<16, 12, kScore, kOff32, kScoreW>(a.t, img, rec + o16, n16, L, sw);
    }
    pipe_barrier();
}

template <bool kScore, bool kOff32>
__global__ __launch_bounds__(kPipeThreads) void car_tile_pipe_kernel(PipeArgs a) {
    extern __shared__ __attribute__((aligned(16))) int lds[];  // 2 item buffers of kBufInts
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int n = (a.items - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    // stages t = -4 .. n-1, padded to a multiple of 6 (the loaders' register
    // rotation period); padding stages touch only clamped items
    const int t_end = -4 + ((n + 4 + 5) / 6) * 6;
    if (wave < kLoadW) {
        const int lt = threadIdx.x;
        // zero-initialised: the prologue stages consume sets no stage has
        // filled yet (their loads must still hit valid addresses: pod 0)
        LdA A0 = {}, A1 = {}, A2 = {};
        LdK K0 = {}, K1 = {};
        LdP P0 = {}, P1 = {};
        for (int t = -4; t < t_end; t += 6) {
            // roles per stage: write (A,K) of t+1, K-issue from A of t+2, A-issue of t+3, P-issue of t+4
            ld_stage<kOff32>(a, t + 0, lt, lds, A0, K1, A1, K0, A2, P1, P0);
            ld_stage<kOff32>(a, t + 1, lt, lds, A1, K0, A2, K1, A0, P0, P1);
            ld_stage<kOff32>(a, t + 2, lt, lds, A2, K1, A0, K0, A1, P1, P0);
            ld_stage<kOff32>(a, t + 3, lt, lds, A0, K0, A1, K1, A2, P0, P1);
            ld_stage<kOff32>(a, t + 4, lt, lds, A1, K1, A2, K0, A0, P1, P0);
            ld_stage<kOff32>(a, t + 5, lt, lds, A2, K0, A0, K1, A1, P0, P1);
        }
    } else {
        const int sw = wave - kLoadW;
        for (int t = -4; t < t_end; ++t) sc_stage<kScore, kOff32>(a, t, n, sw, lane, lds);
    }
}

// ---------------------------------------------------------------------------
// Shared by the mid and heavy kernels.
struct ScoreCtx {
    const int *nodekey;
    const int *zc_cnt;
    const unsigned long long *zc_key;
    int *out_target;
    int *out_score;
    int S, N, PS;
};

// ---------------------------------------------------------------------------
// K2: mid rows (17 <= deg <= 64), one wave per (row, 64-scenario chunk),
// lane = scenario.  Each lane loads its deg node ids (coalesced 256-B rows),
// sorts them with a bitonic network in registers (min/max only: no compare
// masks, no memory), then scans the sorted runs once, gathering nodekey words
// 32 at a time: best packed candidate and the number of best-count runs.
// ---------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ void bitonic_sort(int (&v)[D]) {
#pragma unroll
    for (int k = 2; k <= D; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < D; ++i) {
                const int l = i ^ j;
                if (l > i) {
                    const int lo = min(v[i], v[l]), hi = max(v[i], v[l]);
                    if ((i & k) == 0) { v[i] = lo; v[l] = hi; }
                    else { v[i] = hi; v[l] = lo; }
                }
            }
}

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
    // record: [oi, d, nb[0..D-1], pad]; neighbour ids read 4 at a time
    int v[D];
#pragma unroll
    for (int w = 0; w < W / 4; ++w) {
        const int4 x = r4[w];
        const int q[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = 4 * w + t - 2;
            if (j >= 0 && j < D) v[j] = ld32(a.assign, (unsigned)q[t] * (unsigned)S + (unsigned)s_ld);
        }
    }
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = (j < d && (unsigned)v[j] < (unsigned)a.sc.N) ? v[j] : INT_MAX;
    bitonic_sort<D>(v);
    // one pass over the sorted ids: runs = distinct nodes; keys gathered kC at a time
    constexpr int kC = 32;
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
    // a wave scores PS rows of one bucket, lanes split into PS slots of SL scenarios
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
// K3: hub rows (deg > 64).  Workgroup (4 waves) = (row, group of G scenarios).
//   stage  col[si][j] = {node, key} of neighbour j in scenario s0+si: each
//          neighbour row's G consecutive scenarios in one coalesced segment, its
//          node keys gathered right away (hazard / unscheduled -> KEY_HAZ);
//   score  wave w takes scenarios si = w, w+4, ...; lanes = neighbours:
//          A count every candidate entry into the wave's own LDS table
//          B max count M (wave max)
//          C best (remaining CPU, -node) among the entries with count M, and
//            their number nm = M * |best| (wave reductions)
//          D clear the table for the next scenario.
// Tables: two u16 counters per word indexed by node id when N <= 16384, else
// an open-addressing hash (keys + counts) of next_pow2(2 * deg) slots.
// ---------------------------------------------------------------------------
struct HeavyItem {
    int oi, rb, d, pad;
};

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = __shfl_xor(v, o, 64);
        v = w > v ? w : v;
    }
    return v;
}

// (remaining CPU, -node) as one u64, 0 = none (node < 2^25)
__device__ __forceinline__ unsigned long long pack_rn(int rem, int n) {
    return ((unsigned long long)((unsigned)rem ^ 0x80000000u) << kNodeBits) | (unsigned long long)(kNodeMask - (unsigned)n);
}

template <bool kDirect>
struct HubTable {
    unsigned *keys, *cnts;  // direct: cnts only (2 x u16 per word); hash: keys[H] + cnts[H]
    unsigned mask;
    __device__ __forceinline__ unsigned slot(int n) const {  // hash: the slot holding n (inserted)
        const unsigned k = (unsigned)n + 1u;
        unsigned h = (k * 2654435761u) & mask;
        while (keys[h] != k) h = (h + 1u) & mask;
        return h;
    }
    __device__ __forceinline__ void add(int n) const {
        if (kDirect) {
            atomicAdd(&cnts[n >> 1], 1u << ((n & 1) << 4));
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
        if (kDirect) return (int)((cnts[n >> 1] >> ((n & 1) << 4)) & 0xffffu);
        return (int)cnts[slot(n)];
    }
    __device__ __forceinline__ void clear(int n) const { cnts[n >> 1] = 0u; }  // direct tables only
};

template <bool kDirect>
__global__ __launch_bounds__(256) void car_hub_kernel(const HeavyItem *__restrict__ items, int n_items,
                                                      const int *__restrict__ hcol, const int *__restrict__ assign,
                                                      const int *__restrict__ nodekey, int S, int N, int lg, int dpad,
                                                      int H, const int *__restrict__ zc_cnt,
                                                      const unsigned long long *__restrict__ zc_key,
                                                      int *__restrict__ out_target, int *__restrict__ out_score) {
    extern __shared__ __attribute__((aligned(16))) int lds[];
    const int G = 1 << lg;
    const int grp = blockIdx.x / n_items;
    const HeavyItem it = items[blockIdx.x % n_items];
    const int s0 = grp * G;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int2 *col = reinterpret_cast<int2 *>(lds);                       // [G][dpad]
    unsigned *tabs = reinterpret_cast<unsigned *>(col + G * dpad);   // [4][H] (x2 for the hash)
    const int d = it.d;
    const int total = d << lg;
    // stage: element e -> (neighbour j = e >> lg, scenario si = e & (G-1)); loads
    // unconditional (clamped), duplicates rewrite identical values
    constexpr int kB = 8;
    for (int e0 = 0; e0 < total; e0 += 256 * kB) {
        int e[kB], q[kB], n[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            e[u] = min(e0 + u * 256 + tid, total - 1);
            q[u] = hcol[it.rb + (e[u] >> lg)];
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) n[u] = assign[(size_t)q[u] * S + min(s0 + (e[u] & (G - 1)), S - 1)];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            const int si = e[u] & (G - 1), s = s0 + si;
            const bool ok = (unsigned)n[u] < (unsigned)N && s < S;
            const int key = ld32(nodekey, ok ? (unsigned)n[u] * (unsigned)S + (unsigned)s : 0u);
            col[si * dpad + (e[u] >> lg)] = make_int2(n[u], ok ? key : kKeyHaz);
        }
    }
    const int Hw = kDirect ? H : 2 * H;  // words per wave table
    for (int k = tid; k < 4 * Hw; k += 256) tabs[k] = 0u;
    __syncthreads();
    HubTable<kDirect> tb;
    tb.cnts = tabs + wave * Hw + (kDirect ? 0 : H);
    tb.keys = tabs + wave * Hw;
    tb.mask = (unsigned)H - 1u;
    for (int si = wave; si < G && s0 + si < S; si += 4) {
        const int2 *c = col + si * dpad;
        for (int j = lane; j < d; j += 64) {
            const int2 x = c[j];
            if (x.y != kKeyHaz) tb.add(x.x);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        int M = 0;
        for (int j = lane; j < d; j += 64) {
            const int2 x = c[j];
            if (x.y != kKeyHaz) M = max(M, tb.get(x.x));
        }
        M = wave_max_i(M);
        unsigned long long best = 0;
        int nm = 0;
        for (int j = lane; j < d && M > 0; j += 64) {
            const int2 x = c[j];
            if (x.y != kKeyHaz && tb.get(x.x) == M) {
                ++nm;
                const unsigned long long k = pack_rn(x.y, x.x);
                best = k > best ? k : best;
            }
        }
        best = wave_max_u64(best);
        nm = wave_sum_i(nm);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (kDirect) {
            for (int j = lane; j < d; j += 64) {
                const int2 x = c[j];
                if (x.y != kKeyHaz) tb.clear(x.x);
            }
        } else {  // a probe may still need a slot another lane cleared: wipe the whole table
            for (int k = lane; k < Hw; k += 64) tb.keys[k] = 0u;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (lane == 0) {
            const int s = s0 + si;
            int sc, t;
            if (M == 0) {
                t = zero_target(load_zc(zc_cnt, zc_key, s), sc);
            } else {
                sc = M;
                const int rem = (int)((unsigned)(best >> kNodeBits) ^ 0x80000000u);
                const int bn = (int)(kNodeMask - (unsigned)(best & kNodeMask));
                t = nm == M ? bn : (rem >= 0 ? bn : RSK_TARGET_NONE);
            }
            const size_t o = (size_t)it.oi * S + s;
            out_target[o] = t;
            if (out_score) out_score[o] = sc;
        }
    }
}

}  // namespace rsk

using namespace rsk;

struct rsk_car_plan {
    rsk_ctx *ctx = nullptr;
    int P = 0, Q = 0, max_deg = 0;
    // light rows (deg <= 16) in LDS tiles
    int T = 0, rmax = 0, recmax = 0, n_tile_rows = 0;
    int owners_cap = 128, rows_cap = 160;  // tile limits (RSK_TILE_OWNERS / RSK_TILE_ROWS)
    int64_t img_rows_total = 0, img_pods_distinct = 0, n_img_pods = 0, n_recs = 0;
    DevBuf img_pods, meta, recs;
    // mid rows (17..64)
    int n_mid[kNumMid] = {0, 0};
    DevBuf mid[kNumMid];
    // heavy rows (> 64)
    int n_heavy[kNumHeavy] = {0, 0, 0};
    int heavy_dmax[kNumHeavy] = {0, 0, 0};
    DevBuf heavy_items[kNumHeavy];
    DevBuf hcol;
    // per-execute workspace
    DevBuf nodekey, zc;
    ~rsk_car_plan() {
        img_pods.release();
        meta.release();
        recs.release();
        for (auto &b : mid) b.release();
        for (auto &b : heavy_items) b.release();
        hcol.release();
        nodekey.release();
        zc.release();
    }
};

namespace {

int heavy_class(int d) {
    for (int c = 0; c < kNumHeavy; ++c)
        if (d <= kHeavyMax[c]) return c;
    return -1;
}

int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

struct HeavyGeom {
    int lg, dpad, H;
    bool direct;
    size_t lds;
};

constexpr int kDirectMaxN = 16384;  // direct count tables up to 32 KiB per wave

HeavyGeom heavy_geometry(int dmax, int S, int N) {
    // Largest scenario group G = 2^lg (<= 64, <= next_pow2(S)) whose staged
    // columns + 4 wave tables fit 80 KiB (2 workgroups per CU), else 160 KiB.
    HeavyGeom g;
    g.dpad = dmax | 1;
    g.direct = N <= kDirectMaxN;
    g.H = g.direct ? (N + 1) / 2 : next_pow2(2 * dmax);
    const size_t tab = (size_t)4 * (g.direct ? g.H : 2 * g.H) * 4;
    const int gmax = std::min(64, next_pow2(S));
    for (size_t lim : {(size_t)80 * 1024, (size_t)160 * 1024})
        for (int G = gmax; G >= 1; G >>= 1) {
            g.lds = (size_t)G * g.dpad * 8 + tab;
            g.lg = 0;
            while ((1 << g.lg) < G) ++g.lg;
            if (g.lds <= lim) return g;
        }
    return g;
}

// Locality order of the pods: DFS over the (deduplicated) relation graph, each
// node's DFS-tree children visited smallest subtree first, roots in pod order.
// Consecutive runs of CP pods of this order become tiles.
std::vector<int> locality_order(int P, const std::vector<int> &rp, const std::vector<int> &ci) {
    std::vector<int> parent(P, -1), pre;
    std::vector<char> seen(P, 0);
    pre.reserve(P);
    std::vector<std::pair<int, int>> st;  // (node, next edge)
    for (int r = 0; r < P; ++r) {
        if (seen[r]) continue;
        seen[r] = 1;
        pre.push_back(r);
        st.push_back({r, rp[r]});
        while (!st.empty()) {
            auto &top = st.back();
            const int u = top.first;
            if (top.second >= rp[u + 1]) { st.pop_back(); continue; }
            const int v = ci[top.second++];
            if (seen[v]) continue;
            seen[v] = 1;
            parent[v] = u;
            pre.push_back(v);
            st.push_back({v, rp[v]});
        }
    }
    std::vector<int> size(P, 1);
    for (int k = P - 1; k >= 0; --k) {
        const int v = pre[k];
        if (parent[v] >= 0) size[parent[v]] += size[v];
    }
    std::vector<int> cptr(P + 1, 0), kids(P > 0 ? P : 1);
    for (int v = 0; v < P; ++v) if (parent[v] >= 0) ++cptr[parent[v] + 1];
    for (int v = 0; v < P; ++v) cptr[v + 1] += cptr[v];
    {
        std::vector<int> fill(cptr.begin(), cptr.end() - 1);
        for (int k = 0; k < P; ++k) {
            const int v = pre[k];
            if (parent[v] >= 0) kids[fill[parent[v]]++] = v;
        }
    }
    for (int u = 0; u < P; ++u)
        std::stable_sort(kids.begin() + cptr[u], kids.begin() + cptr[u + 1],
                         [&](int a, int b) { return size[a] < size[b]; });
    std::vector<int> order;
    order.reserve(P);
    std::vector<int> stack;
    for (int r = 0; r < P; ++r) {
        if (parent[r] >= 0) continue;
        stack.push_back(r);
        while (!stack.empty()) {
            const int u = stack.back();
            stack.pop_back();
            order.push_back(u);
            for (int k = cptr[u + 1] - 1; k >= cptr[u]; --k) stack.push_back(kids[k]);
        }
    }
    return order;
}

int upload(DevBuf &buf, const void *src, size_t bytes) {
    if (!bytes) return RSK_OK;
    RSK_TRY(buf.reserve(bytes));
    RSK_HIP(hipMemcpy(buf.ptr, src, bytes, hipMemcpyHostToDevice));
    return RSK_OK;
}

int light_class(int d) {  // d = 0 rows go to the generic class: all entries masked -> zero case
    if (d == 1) return 0;
    if (d == 2) return 1;
    if (d <= 4) return 2;
    if (d <= 8) return 3;
    return 4;
}

// Light-row tiles: rows in DFS order are packed greedily into tiles of at most
// kTileOwners rows whose distinct neighbours (the image rows) number at most
// kTileRows.  On a relation tree in DFS order a tile's image is essentially its
// own 128 pods plus ~5 external neighbours.
struct TileBuilder {
    std::vector<int> img_pods, meta, recs;
    std::vector<int> cur_pods;
    std::unordered_map<int, int> cur_slot;
    std::vector<int> cur_rec[kNumCls];
    int cur_rows = 0, T = 0, rmax = 0, recmax = 0;
    int owners_cap = kTileOwners, rows_cap = kTileRows;
    int64_t img_total = 0;

    bool fits(const int *nb, int d) const {
        if (cur_rows >= owners_cap) return false;
        int fresh = 0;
        for (int j = 0; j < d; ++j) {
            if (cur_slot.count(nb[j])) continue;
            bool dup = false;
            for (int i = 0; i < j; ++i) dup |= nb[i] == nb[j];
            fresh += !dup;
        }
        return (int)cur_pods.size() + fresh <= rows_cap;
    }
    void add(int oi, const int *nb, int d) {
        int lr[kLightMax];
        for (int j = 0; j < d; ++j) {
            auto it = cur_slot.find(nb[j]);
            if (it == cur_slot.end()) {
                it = cur_slot.emplace(nb[j], (int)cur_pods.size()).first;
                cur_pods.push_back(nb[j]);
            }
            lr[j] = it->second;
        }
        const int c = light_class(d);
        auto &e = cur_rec[c];
        const size_t o = e.size();
        e.resize(o + kClsW[c], 0);
        e[o] = oi;
        if (c == 0) {
            e[o + 1] = lr[0];
        } else if (c == 1) {
            e[o + 1] = lr[0] | (lr[1] << 16);
        } else {
            e[o + 1] = d;
            for (int j = 0; j < d; ++j) e[o + 2 + j / 2] |= lr[j] << ((j & 1) * 16);
        }
        ++cur_rows;
    }
    void close() {
        if (!cur_rows) return;
        // every tile stages >= 1 image row (a tile of deg-0 rows stages pod 0,
        // which no record reads): the loaders never see an empty image
        if (cur_pods.empty()) cur_pods.push_back(0);
        const int rec_off = (int)recs.size();
        int n[kNumCls], off[kNumCls];
        for (int c = 0; c < kNumCls; ++c) {
            if (c == 2) while ((recs.size() - rec_off) % 4) recs.push_back(0);  // int4 records from here on
            off[c] = (int)recs.size() - rec_off;
            n[c] = (int)cur_rec[c].size() / kClsW[c];
            recs.insert(recs.end(), cur_rec[c].begin(), cur_rec[c].end());
            cur_rec[c].clear();
        }
        while ((recs.size() - rec_off) % 4) recs.push_back(0);
        const int rec_ints = (int)recs.size() - rec_off;
        const int m[kMetaW] = {(int)img_pods.size(), (int)cur_pods.size(), rec_off, rec_ints,
                               n[0], n[1], n[2], n[3], n[4], off[2], off[3], off[4]};
        meta.insert(meta.end(), m, m + kMetaW);
        img_pods.insert(img_pods.end(), cur_pods.begin(), cur_pods.end());
        img_total += (int64_t)cur_pods.size();
        rmax = std::max(rmax, (int)cur_pods.size());
        recmax = std::max(recmax, rec_ints);
        ++T;
        cur_pods.clear();
        cur_slot.clear();
        cur_rows = 0;
    }
};

int build_plan(rsk_car_plan *plan, const int32_t *row_ptr, const int32_t *col_idx, int32_t P, const int32_t *rows,
               int32_t Q) {
    // deduplicated adjacency without self edges (the evicted pod is off the cluster)
    std::vector<int> rp(P + 1, 0), ci;
    ci.reserve(P ? row_ptr[P] : 0);
    std::vector<int> nb;
    for (int p = 0; p < P; ++p) {
        nb.assign(col_idx + row_ptr[p], col_idx + row_ptr[p + 1]);
        std::sort(nb.begin(), nb.end());
        nb.erase(std::unique(nb.begin(), nb.end()), nb.end());
        nb.erase(std::remove(nb.begin(), nb.end(), p), nb.end());
        ci.insert(ci.end(), nb.begin(), nb.end());
        rp[p + 1] = (int)ci.size();
    }
    const std::vector<int> order = locality_order(P, rp, ci);
    std::vector<int> pos(P);
    for (int k = 0; k < P; ++k) pos[order[k]] = k;

    std::vector<int> light;  // row indices i with deg <= 16, to be tiled in DFS order
    std::vector<std::vector<int>> midr(kNumMid);
    std::vector<std::vector<HeavyItem>> hitems(kNumHeavy);
    std::vector<int> hcol;
    for (int i = 0; i < Q; ++i) {
        const int p = rows ? rows[i] : i;
        const int d = rp[p + 1] - rp[p];
        plan->max_deg = std::max(plan->max_deg, d);
        RSK_CHECK(d <= kMaxDegree, "a row has degree %d > %d (unsupported)", d, kMaxDegree);
        const int *nbp = ci.data() + rp[p];
        if (d <= kLightMax) {
            light.push_back(i);
        } else if (d <= kMidMax) {
            const int b = d <= 32 ? 0 : 1;
            auto &e = midr[b];
            const size_t o = e.size();
            e.resize(o + kMidW[b], 0);
            e[o] = i;
            e[o + 1] = d;
            for (int j = 0; j < d; ++j) e[o + 2 + j] = nbp[j];
            plan->n_mid[b] += 1;
        } else {
            const int c = heavy_class(d);
            hitems[c].push_back({i, (int)hcol.size(), d, 0});
            hcol.insert(hcol.end(), nbp, nbp + d);
            plan->n_heavy[c] += 1;
            plan->heavy_dmax[c] = std::max(plan->heavy_dmax[c], d);
        }
    }
    std::stable_sort(light.begin(), light.end(), [&](int x, int y) {
        return pos[rows ? rows[x] : x] < pos[rows ? rows[y] : y];
    });
    TileBuilder tb;
    tb.owners_cap = plan->owners_cap;
    tb.rows_cap = plan->rows_cap;
    for (int i : light) {
        const int p = rows ? rows[i] : i;
        const int d = rp[p + 1] - rp[p];
        const int *nbp = ci.data() + rp[p];
        if (!tb.fits(nbp, d)) tb.close();
        tb.add(i, nbp, d);
    }
    tb.close();
    plan->T = tb.T;
    plan->rmax = std::max(1, tb.rmax);
    plan->recmax = tb.recmax;
    plan->n_tile_rows = (int)light.size();
    plan->img_rows_total = tb.img_total;
    {
        std::vector<char> seen(P, 0);
        for (int q : tb.img_pods) seen[q] = 1;
        plan->img_pods_distinct = std::count(seen.begin(), seen.end(), 1);
    }
    plan->n_img_pods = (int64_t)tb.img_pods.size();
    plan->n_recs = std::max<int64_t>(4, (int64_t)tb.recs.size());
    if (tb.T > 0) {
        RSK_TRY(upload(plan->img_pods, tb.img_pods.data(), tb.img_pods.size() * 4));
        RSK_TRY(upload(plan->meta, tb.meta.data(), tb.meta.size() * 4));
        if (tb.recs.empty()) tb.recs.assign(4, 0);
        RSK_TRY(upload(plan->recs, tb.recs.data(), tb.recs.size() * 4));
    }
    for (int b = 0; b < kNumMid; ++b) RSK_TRY(upload(plan->mid[b], midr[b].data(), midr[b].size() * 4));
    for (int c = 0; c < kNumHeavy; ++c)
        RSK_TRY(upload(plan->heavy_items[c], hitems[c].data(), hitems[c].size() * sizeof(HeavyItem)));
    RSK_TRY(upload(plan->hcol, hcol.data(), hcol.size() * 4));
    return RSK_OK;
}

int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return e ? atoi(e) : dflt;
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
    auto plan = new rsk_car_plan();
    plan->ctx = ctx;
    plan->owners_cap = std::min(kTileOwners, std::max(8, env_int("RSK_TILE_OWNERS", 128)));
    plan->rows_cap = std::min(kTileRows, std::max(kLightMax, env_int("RSK_TILE_ROWS", plan->owners_cap + 32)));
    plan->P = P;
    plan->Q = Q;
    const int rc = build_plan(plan, row_ptr, col_idx, P, rows, Q);
    if (rc != RSK_OK) {
        std::string keep = last_error();
        delete plan;
        set_error("%s", keep.c_str());
        return rc;
    }
    *out = plan;
    return RSK_OK;
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
    const int64_t v[14] = {plan->n_tile_rows, 0, mid, heavy, plan->T, plan->rmax, plan->owners_cap,
                           tile_bytes, 0, mid_bytes, heavy_bytes, plan->max_deg, plan->img_rows_total,
                           plan->img_pods_distinct};
    const int m = n < 14 ? n : 14;
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

    RSK_TRY(plan->nodekey.reserve(NS * 4));
    RSK_TRY(plan->zc.reserve((size_t)S * 12 + 16));
    int *d_key = plan->nodekey.as<int>();
    unsigned long long *d_zkey = plan->zc.as<unsigned long long>();
    int *d_zcnt = reinterpret_cast<int *>(d_zkey + S);
    RSK_HIP(hipMemsetAsync(plan->zc.ptr, 0, (size_t)S * 12, ctx->stream));

    {   // K0
        const int target_threads = 256 * 2048;
        int npb = (int)std::max<int64_t>(1, ceil_div((int64_t)N * S, target_threads));
        const int64_t chunks = ceil_div(N, npb);
        const unsigned total = (unsigned)(chunks * S);
        ScopedTimer tm(ctx, "car_prep");
        car_prep_kernel<<<dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, ctx->stream>>>(
            d_cap, d_use, d_haz, N, S, npb, total, d_key, d_zcnt, d_zkey);
        RSK_HIP(hipGetLastError());
    }
    if (plan->T > 0) {   // K1 light-row tiles
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
        a.n_meta = (unsigned)plan->T * kMetaW;
        static const int sl_max = [] { int v = env_int("RSK_TILE_SL", 32); return v >= 1 && v <= 64 ? v : 32; }();
        int SL = std::min(next_pow2(S), next_pow2(sl_max));
        a.lsl = 0;
        while ((1 << a.lsl) < SL) ++a.lsl;
        static const int ablate = env_int("RSK_ABLATE_TILE", 0);
        static const int order = env_int("RSK_TILE_ORDER", 0);
        a.order = order;
        a.ablate = ablate;
        const bool vec = SL >= 4 && S % 4 == 0;
        const bool off32 = (int64_t)std::max(plan->P, plan->Q) * S * 4 < ((int64_t)1 << 32);
        const size_t lds = ((((size_t)2 * plan->rmax * SL + 3) & ~(size_t)3) + plan->recmax) * 4;
        RSK_CHECK(lds <= 160 * 1024, "tile image needs %zu B of LDS", lds);
        const int64_t blocks = ceil_div(S, SL) * plan->T;
        RSK_CHECK(blocks < INT32_MAX, "tile grid too large");
        using TileKern = void (*)(TileArgs);
#define RSK_TK(NT) {&car_tile_kernel<false, false, false, NT>, &car_tile_kernel<false, false, true, NT>, \
                    &car_tile_kernel<false, true, false, NT>,  &car_tile_kernel<false, true, true, NT>,  \
                    &car_tile_kernel<true, false, false, NT>,  &car_tile_kernel<true, false, true, NT>,  \
                    &car_tile_kernel<true, true, false, NT>,   &car_tile_kernel<true, true, true, NT>}
        static const TileKern kerns[2][8] = {RSK_TK(128), RSK_TK(256)};
#undef RSK_TK
        static const int nt_env = env_int("RSK_TILE_NT", 0);
        int nt = nt_env == 128 || nt_env == 256 ? nt_env : (plan->owners_cap >= 64 ? 256 : 128);
        if (nt * 8 < plan->recmax) nt = 256;
        RSK_CHECK(nt * 8 >= plan->recmax, "tile records (%d ints) exceed the copy width", plan->recmax);
        const TileKern kern = kerns[nt == 256][(vec ? 4 : 0) + (d_score ? 2 : 0) + (off32 ? 1 : 0)];
        if (lds > 64 * 1024)
            RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        static const int pipe_env = env_int("RSK_TILE_PIPE", 0);
        if (pipe_env && vec && SL == kPipeSL) {
            PipeArgs pa;
            pa.t = a;
            pa.items = (int)blocks;
            int cus = 0;
            RSK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
            const size_t plds = (size_t)2 * kBufInts * 4;
            using PipeKern = void (*)(PipeArgs);
            static const PipeKern pk[4] = {&car_tile_pipe_kernel<false, false>, &car_tile_pipe_kernel<false, true>,
                                           &car_tile_pipe_kernel<true, false>, &car_tile_pipe_kernel<true, true>};
            const PipeKern pkern = pk[(d_score ? 2 : 0) + (off32 ? 1 : 0)];
            RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(pkern),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)plds));
            const int grid = (int)std::min<int64_t>(blocks, (int64_t)cus * std::max(1, env_int("RSK_PIPE_PER_CU", 1)));
            ScopedTimer tm(ctx, "car_tile");
            pkern<<<dim3((unsigned)grid), dim3(kPipeThreads), plds, ctx->stream>>>(pa);
            RSK_HIP(hipGetLastError());
        } else {
            ScopedTimer tm(ctx, "car_tile");
            kern<<<dim3((unsigned)blocks), dim3(nt), lds, ctx->stream>>>(a);
            RSK_HIP(hipGetLastError());
        }
    }
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
    {   // K2 mid rows
        MidArgs a;
        std::memset(&a, 0, sizeof(a));
        a.sc = sc;
        a.SL = SL;
        a.prefix[0] = 0;
        for (int b = 0; b < kNumMid; ++b) {
            a.rec[b] = plan->mid[b].as<int>();
            a.n_items[b] = plan->n_mid[b];
            a.prefix[b + 1] = a.prefix[b] + (int)ceil_div(plan->n_mid[b], sc.PS);
        }
        a.assign = d_assign;
        const int waves = a.prefix[kNumMid];
        if (waves > 0) {
            a.blocks_per_chunk = (int)ceil_div(waves, 4);
            const int64_t blocks = chunks * a.blocks_per_chunk;
            RSK_CHECK(blocks < INT32_MAX, "mid grid too large");
            ScopedTimer tm(ctx, "car_mid");
            car_mid_kernel<<<dim3((unsigned)blocks), dim3(256), 0, ctx->stream>>>(a);
            RSK_HIP(hipGetLastError());
        }
    }
    for (int c = 0; c < kNumHeavy; ++c) {   // K3 hub rows
        const int n = plan->n_heavy[c];
        if (!n) continue;
        const HeavyGeom g = heavy_geometry(plan->heavy_dmax[c], S, N);
        RSK_CHECK(g.lds <= 160 * 1024, "hub class %d needs %zu B of LDS", c, g.lds);
        const int64_t groups = ceil_div(S, 1 << g.lg);
        RSK_CHECK(groups * n < INT32_MAX, "hub grid too large");
        auto kern = g.direct ? &car_hub_kernel<true> : &car_hub_kernel<false>;
        if (g.lds > 64 * 1024)
            RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)g.lds));
        ScopedTimer tm(ctx, "car_heavy");
        kern<<<dim3((unsigned)(groups * n)), dim3(256), g.lds, ctx->stream>>>(
            plan->heavy_items[c].as<HeavyItem>(), n, plan->hcol.as<int>(), d_assign, d_key, S, N, g.lg, g.dpad,
            g.H, d_zcnt, d_zkey, d_target, d_score);
        RSK_HIP(hipGetLastError());
    }
#ifdef RSK_DEBUG_BOUNDS
    {
        unsigned flags_h = 0, zero = 0;
        RSK_HIP(hipStreamSynchronize(ctx->stream));
        RSK_HIP(hipMemcpyFromSymbol(&flags_h, HIP_SYMBOL(rsk_dbg_flags), 4));
        RSK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(rsk_dbg_flags), &zero, 4));
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
