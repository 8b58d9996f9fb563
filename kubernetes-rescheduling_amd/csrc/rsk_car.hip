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
//   * max score M > 0: the winner is among the neighbour nodes.  With the
//     lexicographic key (count, remaining CPU, -node) the argmax is the
//     reference's choice; |best| == 1 iff exactly M neighbour entries reach M.
//   * M == 0: every non-hazard node ties at 0 -> a per-scenario constant
//     ("zero case"), computed once by car_prep_kernel.
//
// Kernels (one HIP stream, all integer, no atomics on the decision path):
//   car_prep_kernel   nodekey[n*S+s] = hazard ? KEY_HAZ : cap[n]-use[n*S+s] (one
//                     gather word per node later) + the zero case per scenario.
//   car_tile_kernel   deg <= 16 rows of dense tiles: LDS image of the tile's
//                     assign rows (each row read from HBM once per chunk),
//                     per-lane register histograms (lane = scenario).
//   car_light_kernel  deg <= 16 rows of sparse tiles: same scorer, neighbour
//                     rows gathered from global.
//   car_mid_kernel    17 <= deg <= 128: per-lane bitonic sort of the neighbour
//                     node ids in registers + run-length scan.
//   car_heavy_kernel  deg > 128: node ids staged in LDS, per-wave LDS count
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

constexpr int kKeyHaz = INT_MIN;
constexpr int kMaxDegree = 4096;
constexpr int kLightMax = 16;                      // register-histogram rows: deg <= 16
constexpr int kNumLight = 4;                       // buckets D = 16, 8, 4, 2
constexpr int kLightW[kNumLight] = {20, 12, 8, 4};  // record ints: oi, d, nb[D], pad to x4
constexpr int kLightPK[kNumLight] = {1, 2, 4, 4};  // direct kernel: records per lane per step
constexpr int kMidMax = 128;                       // sorted-register rows: 17 <= deg <= 128
constexpr int kNumMid = 3;                         // buckets D = 32, 64, 128
constexpr int kMidW[kNumMid] = {36, 68, 132};
constexpr int kNumHeavy = 3;                       // (128,512] (512,2048] (2048,4096]
constexpr int kHeavyMax[kNumHeavy] = {512, 2048, 4096};
constexpr int kTileCP = 256;                       // pods per tile
constexpr int kTileXCap = 64;                      // max external rows appended to a tile image
constexpr int kTileWaves = 8;                      // waves per tile workgroup
constexpr int kTileBatch = 12;                     // rows per wave per load batch (register path)

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

// Candidate key of the register scorers: lexicographic (count, remaining CPU,
// -node) as one u64 — count 7 bits (<= 64), remaining CPU 32 bits (sign
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

// rescheduling.py:199-214 applied to the reduced state.
__device__ __forceinline__ int car_finalize(const CarState &st, const ZeroCase &z, int &score) {
    if (st.bc == 0) {
        if (z.cnt == 0) { score = -1; return RSK_TARGET_NO_CANDIDATE; }
        const int n = (int)(~(unsigned)(z.key & 0xffffffffull));
        const int rem = (int)((unsigned)(z.key >> 32) ^ 0x80000000u);
        score = 0;
        if (z.cnt == 1) return n;
        return rem >= 0 ? n : RSK_TARGET_NONE;
    }
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
// Register scorer for deg <= 16 rows.  A record is
//   [out_row, deg, nb[0..D-1], pad]   (W ints, W % 4 == 0, int4-loadable)
// and `fetch(nb)` returns the neighbour's node id in this lane's scenario
// (padding entries encode a valid source).  Each lane counts equal node ids
// pairwise in registers, gathers one nodekey word per neighbour and keeps the
// max packed candidate key.
//
// Every load is issued unconditionally from a clamped, always-valid address
// and the result selected afterwards: hipcc otherwise branches around each
// guarded load and waits vmcnt(0) per element, serialising the gather.
// ---------------------------------------------------------------------------
struct ScoreCtx {
    const int *nodekey;
    const int *zc_cnt;
    const unsigned long long *zc_key;
    int *out_target;
    int *out_score;
    int S, N, PS;
};

template <int D>
__device__ __forceinline__ CarState reduce_entries(const int (&nd)[D], const int (&ky)[D]) {
    int cnt[D];
#pragma unroll
    for (int j = 0; j < D; ++j) cnt[j] = 1;
#pragma unroll
    for (int j = 1; j < D; ++j)
#pragma unroll
        for (int jj = 0; jj < j; ++jj) {
            const int e = 1 - (int)min((unsigned)(nd[j] ^ nd[jj]), 1u);
            cnt[j] += e;
            cnt[jj] += e;
        }
    unsigned long long best = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const unsigned long long key = ky[j] == kKeyHaz ? 0ull : pack_cand(cnt[j], ky[j], nd[j]);
        best = key > best ? key : best;
    }
    const int M = cand_count(best);
    int nm = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) nm += (ky[j] != kKeyHaz) & (cnt[j] == M);
    return cand_state(best, nm);
}

template <int D, int PK, int W, class Fetch>
__device__ __forceinline__ void score_records(const ScoreCtx &a, const int *__restrict__ recs, int item0,
                                              int item_end, int slot, int s, bool lane_ok, Fetch fetch) {
    const int S = a.S;
    const int s_ld = min(s, S - 1);  // loads of inactive lanes stay in bounds
    const int step = PK * a.PS;
    const ZeroCase z = load_zc(a.zc_cnt, a.zc_key, s_ld);
    for (int base = item0; base < item_end; base += step) {
        int oi[PK], dg[PK], nd[PK][D], ky[PK][D];
        bool v[PK];
#pragma unroll
        for (int k = 0; k < PK; ++k) {
            const int it = base + k * a.PS + slot;
            v[k] = lane_ok && it < item_end;
            const int4 *rec = reinterpret_cast<const int4 *>(recs + (size_t)(v[k] ? it : item0) * W);
            int r[W];
#pragma unroll
            for (int w = 0; w < W / 4; ++w) {
                const int4 x = rec[w];
                r[4 * w] = x.x; r[4 * w + 1] = x.y; r[4 * w + 2] = x.z; r[4 * w + 3] = x.w;
            }
            oi[k] = r[0];
            dg[k] = v[k] ? r[1] : 0;
#pragma unroll
            for (int j = 0; j < D; ++j) nd[k][j] = fetch(r[2 + j]);
        }
#pragma unroll
        for (int k = 0; k < PK; ++k)
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const int n = j < dg[k] ? nd[k][j] : -1;
                const bool ok = (unsigned)n < (unsigned)a.N;
                const int key = ld32(a.nodekey, (unsigned)(ok ? n : 0) * (unsigned)S + (unsigned)s_ld);
                ky[k][j] = ok ? key : kKeyHaz;
                nd[k][j] = ok ? n : -1 - j;  // never equal to another entry
            }
#pragma unroll
        for (int k = 0; k < PK; ++k) {
            const CarState st = reduce_entries<D>(nd[k], ky[k]);
            if (v[k]) {
                int sc;
                const int t = car_finalize(st, z, sc);
                const size_t o = (size_t)oi[k] * S + s;
                a.out_target[o] = t;
                if (a.out_score) a.out_score[o] = sc;
            }
        }
    }
}

// K1a: direct rows (deg <= 16, owners of sparse tiles): records whose
// neighbours are global pod ids (padding = pod 0); each neighbour row is one
// coalesced 256-B gather.
struct LightArgs {
    ScoreCtx sc;
    const int *ell[kNumLight];
    int n_items[kNumLight];
    int task_items[kNumLight];   // items per wave task
    int task_prefix[kNumLight + 1];
    const int *assign;
    int SL, blocks_per_chunk;
};

__global__ __launch_bounds__(256) void car_light_kernel(LightArgs a) {
    const int chunk = blockIdx.x / a.blocks_per_chunk;
    const int wave = (blockIdx.x % a.blocks_per_chunk) * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (wave >= a.task_prefix[kNumLight]) return;
    const int slot = lane / a.SL;
    const int s = chunk * a.SL + lane % a.SL;
    const bool lane_ok = slot < a.sc.PS && s < a.sc.S;
    int b = 0;
    while (wave >= a.task_prefix[b + 1]) ++b;
    const int lt = wave - a.task_prefix[b];
    const int item0 = lt * a.task_items[b];
    const int item_end = min(a.n_items[b], item0 + a.task_items[b]);
    const int *__restrict__ assign = a.assign;
    const size_t S = (size_t)a.sc.S;
    const int s_ld = min(s, a.sc.S - 1);
    auto fetch = [=](int q) { return assign[(size_t)q * S + s_ld]; };
    switch (b) {
        case 0: score_records<16, 1, 20>(a.sc, a.ell[0], item0, item_end, slot, s, lane_ok, fetch); break;
        case 1: score_records<8, 2, 12>(a.sc, a.ell[1], item0, item_end, slot, s, lane_ok, fetch); break;
        case 2: score_records<4, 4, 8>(a.sc, a.ell[2], item0, item_end, slot, s, lane_ok, fetch); break;
        default: score_records<2, 4, 4>(a.sc, a.ell[3], item0, item_end, slot, s, lane_ok, fetch); break;
    }
}

// K1b: tiled rows (deg <= 16).  The plan orders pods by a DFS of the relation
// graph (small subtrees first) and cuts the order into tiles of CP pods; ~96%
// of a light row's neighbours share its tile (100k/5k PA tree, CP=256) and the
// rest (a handful per tile) are appended to the tile image as extra rows.
// Workgroup (8 waves) = (tile, chunk of SL <= 64 scenarios):
//   phase 1  the tile's image rows (members + externals), SL scenarios each ->
//            LDS image[row][SL] — each assign row leaves HBM once per chunk as
//            one 256-B LDS-DMA (global_load_lds_dword) per row when SL = 64 —
//            and the tile's owner records (one contiguous blob) -> LDS.
//   phase 2  owner records score from LDS; only each neighbour's nodekey word
//            comes from L2; one 256-B target store per record.
struct TileArgs {
    ScoreCtx sc;
    const int *members;       // [T][RS] pod ids (pad = pod 0, never referenced)
    const int *nrows;         // [T] image rows of each tile (<= RS)
    const int *blob;          // per-tile record blobs, concatenated
    const int *blob_off;      // [T][kNumLight + 1] ints: blob start + bucket starts (absolute)
    const int *assign;
    int SL, RS, T, blob_max;  // blob_max: largest blob (ints, multiple of 4)
    int ablate;               // profiling only (RSK_ABLATE_TILE): 1 skip image load, 2 skip scoring
};

template <int D, int PK, int W>
__device__ __forceinline__ void tile_bucket(const TileArgs &a, const int *img, const int *recs, int nrec, int wave,
                                            int slot, int sl, int s, bool lane_ok) {
    const int per = PK * a.sc.PS;
    const int SL = a.SL;
    auto fetch = [=](int row) { return img[row * SL + sl]; };
    for (int g0 = wave * per; g0 < nrec; g0 += kTileWaves * per)
        score_records<D, PK, W>(a.sc, recs, g0, min(nrec, g0 + per), slot, s, lane_ok, fetch);
}

__global__ __launch_bounds__(kTileWaves * 64) void car_tile_kernel(TileArgs a) {
    extern __shared__ __attribute__((aligned(16))) int lds[];  // image [RS][SL] then records [blob_max]
    const int chunk = blockIdx.x / a.T, tile = blockIdx.x % a.T;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int SL = a.SL, PS = a.sc.PS;
    const int slot = lane / SL, sl = lane % SL;
    const int s = chunk * SL + sl;
    const bool lane_ok = slot < PS && s < a.sc.S;
    const int *__restrict__ mem = a.members + (size_t)tile * a.RS;
    const int *__restrict__ assign = a.assign;
    const size_t S = (size_t)a.sc.S;
    const int s_ld = min(s, a.sc.S - 1);
    const int nr = a.nrows[tile];
    int *img = lds;
    int *recs = lds + a.RS * SL;

    // phase 1a: owner record blob -> LDS (int4 copies, issued first: no dependency)
    const int *bo = a.blob_off + (size_t)tile * (kNumLight + 2);
    const int b0 = bo[0], b1 = bo[kNumLight + 1];
    for (int i = threadIdx.x * 4; i < b1 - b0; i += kTileWaves * 64 * 4)
        *reinterpret_cast<int4 *>(recs + i) = *reinterpret_cast<const int4 *>(a.blob + b0 + i);
    // phase 1b: image rows
    if (a.ablate & 1) {
        // profiling ablation: no image load (results are wrong)
    } else if (PS == 1) {
        // one LDS-DMA wave instruction per row: lane l loads scenario chunk*64+l
        // No branch between the DMAs (a per-row `if` splits basic blocks and the
        // waitcnt pass then drains vmcnt(0) before every DMA): rows past the
        // image's end re-load its last row into the same LDS row (same bytes).
        // Row ids are wave-uniform: readfirstlane makes the member loads scalar
        // (lgkmcnt), so they never share the vector-memory counter with the DMAs.
        constexpr int kMaxRowsPerWave = (kTileCP + kTileXCap + kTileWaves - 1) / kTileWaves;
        const int wu = __builtin_amdgcn_readfirstlane(wave);
        int q[kMaxRowsPerWave];
#pragma unroll
        for (int k = 0; k < kMaxRowsPerWave; ++k) q[k] = mem[min(wu + k * kTileWaves, nr - 1)];
#pragma unroll
        for (int k = 0; k < kMaxRowsPerWave; ++k) {
            const int r = min(wu + k * kTileWaves, nr - 1);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(assign + (size_t)q[k] * S + s_ld),
                (__attribute__((address_space(3))) void *)(img + r * SL), 4, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        for (int r0 = wave * PS; r0 < nr; r0 += kTileWaves * PS * kTileBatch) {
            int q[kTileBatch], v[kTileBatch];
#pragma unroll
            for (int k = 0; k < kTileBatch; ++k) q[k] = mem[min(r0 + k * kTileWaves * PS + slot, a.RS - 1)];
#pragma unroll
            for (int k = 0; k < kTileBatch; ++k) v[k] = assign[(size_t)q[k] * S + s_ld];
#pragma unroll
            for (int k = 0; k < kTileBatch; ++k) {
                const int r = r0 + k * kTileWaves * PS + slot;
                if (slot < PS && r < nr) img[r * SL + sl] = v[k];
            }
        }
    }
    __syncthreads();
    if (a.ablate & 2) return;  // profiling ablation: no scoring (results are wrong)
    tile_bucket<16, 1, 20>(a, img, recs + (bo[1] - b0), (bo[2] - bo[1]) / 20, wave, slot, sl, s, lane_ok);
    tile_bucket<8, 2, 12>(a, img, recs + (bo[2] - b0), (bo[3] - bo[2]) / 12, wave, slot, sl, s, lane_ok);
    tile_bucket<4, 4, 8>(a, img, recs + (bo[3] - b0), (bo[4] - bo[3]) / 8, wave, slot, sl, s, lane_ok);
    tile_bucket<2, 8, 4>(a, img, recs + (bo[4] - b0), (bo[5] - bo[4]) / 4, wave, slot, sl, s, lane_ok);
}

// ---------------------------------------------------------------------------
// K1c: mid rows (17 <= deg <= 128), one wave per (row, 64-scenario chunk),
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

// kWide = false: buckets D = 32, 64; kWide = true: bucket D = 128 (its own
// launch, so the 256-VGPR D=128 body does not lower the occupancy of the others)
template <bool kWide>
__global__ __launch_bounds__(256) void car_mid_kernel(MidArgs a) {
    const int chunk = blockIdx.x / a.blocks_per_chunk;
    const int wave = (blockIdx.x % a.blocks_per_chunk) * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int b_lo = kWide ? 2 : 0, b_hi = kWide ? 3 : 2;
    if (wave >= a.prefix[b_hi] - a.prefix[b_lo]) return;
    // a wave scores PS rows of one bucket, lanes split into PS slots of SL scenarios
    const int slot = lane / a.SL;
    const int s = chunk * a.SL + lane % a.SL;
    int b = b_lo;
    while (wave >= a.prefix[b + 1] - a.prefix[b_lo]) ++b;
    const int item = (wave - (a.prefix[b] - a.prefix[b_lo])) * a.sc.PS + slot;
    const bool lane_ok = slot < a.sc.PS && s < a.sc.S && item < a.n_items[b];
    const int it = min(item, a.n_items[b] - 1);
    if (kWide) {
        mid_row<128, 132>(a, a.rec[2] + (size_t)it * 132, slot, s, lane_ok);
    } else if (b == 0) {
        mid_row<32, 36>(a, a.rec[0] + (size_t)it * 36, slot, s, lane_ok);
    } else {
        mid_row<64, 68>(a, a.rec[1] + (size_t)it * 68, slot, s, lane_ok);
    }
}

// ---------------------------------------------------------------------------
// K2: heavy rows (deg > 128).  Workgroup = (row, group of G scenarios).
//   phase 0  stage node ids ntile[si][j] (G-scenario row segments per neighbour)
//   phase A  wave w < NT hashes scenario si's d node ids into its LDS table
//   phase B  counts back into ctile[si][j]; table cleared for the next scenario
//   phase C  thread -> (si = tid % G, j = tid / G + k*256/G): nodekey gathers are
//            G consecutive scenarios of one node (coalesced), then a shuffle /
//            LDS reduction of CarState per scenario.
// ---------------------------------------------------------------------------
struct HeavyItem {
    int oi, rb, d, pad;
};

__device__ __forceinline__ int hash_insert(unsigned *keys, unsigned *cnts, unsigned mask, int n) {
    const unsigned k = (unsigned)n + 1u;
    unsigned h = (k * 2654435761u) & mask;
    while (true) {
        const unsigned prev = atomicCAS(&keys[h], 0u, k);
        if (prev == 0u || prev == k) {
            atomicAdd(&cnts[h], 1u);
            return (int)h;
        }
        h = (h + 1u) & mask;
    }
}

template <bool kDirect>
__global__ __launch_bounds__(256) void car_heavy_kernel(const HeavyItem *__restrict__ items, int n_items,
                                                        const int *__restrict__ hcol,
                                                        const int *__restrict__ assign,
                                                        const int *__restrict__ nodekey, int S, int N, int G,
                                                        int dpad, int H, int NT, const int *__restrict__ zc_cnt,
                                                        const unsigned long long *__restrict__ zc_key,
                                                        int *__restrict__ out_target, int *__restrict__ out_score) {
    extern __shared__ __attribute__((aligned(16))) int lds[];
    const int g = blockIdx.x / n_items;
    const HeavyItem it = items[blockIdx.x % n_items];
    const int s0 = g * G;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // kDirect: per-wave count table over node ids, two u16 counters per word
    // (H = ceil(N/2) words); otherwise an open-addressing hash of H slots.
    int *ntile = lds;                                       // [G][dpad]
    int *ctile = ntile + G * dpad;                          // [G][dpad]
    unsigned *tkey = reinterpret_cast<unsigned *>(ctile + G * dpad);  // [NT][H] (hash only)
    unsigned *tcnt = kDirect ? tkey : tkey + NT * H;        // [NT][H]
    CarState *red = reinterpret_cast<CarState *>(tcnt + NT * H);      // [4][G]

    const int d = it.d;
    // stage: G consecutive scenarios of each neighbour row; loads unconditional
    // (clamped) and batched so they are all in flight before the LDS writes
    constexpr int kB = 4;
    for (int idx0 = tid; idx0 < d * G; idx0 += 256 * kB) {
        int v[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const int idx = min(idx0 + k * 256, d * G - 1);
            const int j = idx / G, si = idx - j * G;
            v[k] = assign[(size_t)hcol[it.rb + j] * S + min(s0 + si, S - 1)];
        }
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const int idx = idx0 + k * 256;
            if (idx < d * G) {
                const int j = idx / G, si = idx - j * G;
                ntile[si * dpad + j] = (s0 + si < S && (unsigned)v[k] < (unsigned)N) ? v[k] : -1;
            }
        }
    }
    for (int k = tid; k < NT * H; k += 256) { tkey[k] = 0u; tcnt[k] = 0u; }
    __syncthreads();

    if (kDirect && wave < NT) {
        unsigned *cnts = tcnt + wave * H;
        for (int si = wave; si < G; si += NT) {
            const int *nrow = ntile + si * dpad;
            int *crow = ctile + si * dpad;
            for (int j = lane; j < d; j += 64) {
                const int n = nrow[j];
                if (n >= 0) atomicAdd(&cnts[n >> 1], 1u << ((n & 1) << 4));
            }
            __builtin_amdgcn_wave_barrier();
            for (int j = lane; j < d; j += 64) {
                const int n = nrow[j];
                crow[j] = n >= 0 ? (int)((cnts[n >> 1] >> ((n & 1) << 4)) & 0xffffu) : 0;
            }
            __builtin_amdgcn_wave_barrier();
            for (int j = lane; j < d; j += 64) {
                const int n = nrow[j];
                if (n >= 0) cnts[n >> 1] = 0u;
            }
            __builtin_amdgcn_wave_barrier();
        }
    } else if (!kDirect && wave < NT) {
        unsigned *keys = tkey + wave * H, *cnts = tcnt + wave * H;
        const unsigned mask = (unsigned)H - 1u;
        for (int si = wave; si < G; si += NT) {
            int *nrow = ntile + si * dpad, *crow = ctile + si * dpad;
            for (int j = lane; j < d; j += 64) {
                const int n = nrow[j];
                crow[j] = n >= 0 ? hash_insert(keys, cnts, mask, n) : -1;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            for (int j = lane; j < d; j += 64) {
                const int slot = crow[j];
                crow[j] = slot >= 0 ? (int)cnts[slot] : 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            for (int k = lane; k < H; k += 64) { keys[k] = 0u; cnts[k] = 0u; }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        }
    }
    __syncthreads();

    const int si = tid % G, jstep = 256 / G;
    const int s = s0 + si;
    CarState st;
    st_init(st);
    {
        // batches of kC independent gathers (a load-then-use loop body would
        // serialise one L2 round trip per neighbour)
        constexpr int kC = 8;
        const int *nrow = ntile + si * dpad, *crow = ctile + si * dpad;
        const unsigned s_ld = (unsigned)min(s, S - 1);
        for (int j0 = tid / G; j0 < d; j0 += jstep * kC) {
            int n[kC], key[kC];
#pragma unroll
            for (int k = 0; k < kC; ++k) {
                const int j = min(j0 + k * jstep, d - 1);
                n[k] = nrow[j];
                key[k] = ld32(nodekey, (unsigned)max(n[k], 0) * (unsigned)S + s_ld);
            }
#pragma unroll
            for (int k = 0; k < kC; ++k) {
                const int j = j0 + k * jstep;
                if (j < d && s < S && n[k] >= 0 && key[k] != kKeyHaz) st_add(st, crow[j], key[k], n[k]);
            }
        }
    }
    for (int off = G; off < 64; off <<= 1) st = st_combine(st, st_shfl_xor(st, off));
    if (lane < G) red[wave * G + lane] = st;
    __syncthreads();
    if (tid < G && s < S) {
        CarState r = red[tid];
        for (int w = 1; w < 4; ++w) r = st_combine(r, red[w * G + tid]);
        int sc;
        const int t = car_finalize(r, load_zc(zc_cnt, zc_key, s), sc);
        const size_t o = (size_t)it.oi * S + s;
        out_target[o] = t;
        if (out_score) out_score[o] = sc;
    }
}

}  // namespace rsk

using namespace rsk;

struct rsk_car_plan {
    rsk_ctx *ctx = nullptr;
    int P = 0, Q = 0, max_deg = 0;
    // tiled rows (deg <= 16 in dense tiles)
    int CP = kTileCP, RS = kTileCP, T = 0, n_tile_owners = 0, blob_max = 0;
    DevBuf members, nrows, blob, blob_off;
    // direct rows (deg <= 16 in sparse tiles)
    int n_light[kNumLight] = {0, 0, 0, 0};
    DevBuf ell[kNumLight];
    // mid rows (17..64)
    int n_mid[kNumMid] = {0, 0, 0};
    DevBuf mid[kNumMid];
    // heavy rows (> 64)
    int n_heavy[kNumHeavy] = {0, 0, 0};
    int heavy_dmax[kNumHeavy] = {0, 0, 0};
    DevBuf heavy_items[kNumHeavy];
    DevBuf hcol;
    // per-execute workspace
    DevBuf nodekey, zc;
    ~rsk_car_plan() {
        members.release();
        nrows.release();
        blob.release();
        blob_off.release();
        for (auto &b : ell) b.release();
        for (auto &b : mid) b.release();
        for (auto &b : heavy_items) b.release();
        hcol.release();
        nodekey.release();
        zc.release();
    }
};

namespace {

int light_bucket(int d) {
    if (d <= 2) return 3;
    if (d <= 4) return 2;
    if (d <= 8) return 1;
    return 0;
}


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
    int G, dpad, H, NT;
    bool direct;
    size_t lds;
};

constexpr int kDirectMaxN = 16384;  // direct count tables up to 32 KiB per wave

HeavyGeom heavy_geometry(int dmax, int S, int N) {
    // Largest scenario group G (<= 64, <= S rounded up to a power of two) and
    // hash-table count NT that fit 64 KiB of LDS (2 workgroups per CU); failing
    // that, anything up to the 160 KiB a single workgroup may declare.
    HeavyGeom g;
    g.dpad = dmax | 1;  // odd row pitch: scenario rows start on different banks
    g.direct = N <= kDirectMaxN;
    g.H = g.direct ? (N + 1) / 2 : next_pow2(2 * dmax);
    const size_t slot_bytes = g.direct ? 4 : 8;
    const int gmax = std::min(64, next_pow2(S));
    const size_t limits[2] = {64 * 1024, 160 * 1024};
    for (size_t lim : limits)
        for (g.G = gmax; g.G >= 1; g.G >>= 1)
            for (g.NT = 4; g.NT >= 1; g.NT >>= 1) {
                g.lds = (size_t)2 * g.G * g.dpad * 4 + (size_t)g.NT * g.H * slot_bytes +
                        (size_t)4 * g.G * sizeof(CarState);
                if (g.lds <= lim) return g;
            }
    g.G = 1;
    g.NT = 1;
    g.lds = (size_t)2 * g.dpad * 4 + (size_t)g.H * slot_bytes + 4 * sizeof(CarState);
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
    const int CP = plan->CP;
    const std::vector<int> order = locality_order(P, rp, ci);
    std::vector<int> pos(P);
    for (int k = 0; k < P; ++k) pos[order[k]] = k;
    const int ntiles = (P + CP - 1) / CP;

    // owners per tile (rows with deg <= kLightMax)
    std::vector<int> owners_in(ntiles, 0);
    for (int i = 0; i < Q; ++i) {
        const int p = rows ? rows[i] : i;
        const int d = rp[p + 1] - rp[p];
        plan->max_deg = std::max(plan->max_deg, d);
        if (d <= kLightMax) ++owners_in[pos[p] / CP];
    }
    RSK_CHECK(plan->max_deg <= kMaxDegree, "a row has degree %d > %d (unsupported)", plan->max_deg, kMaxDegree);
    const int min_owners = std::max(1, CP / 16);  // sparser tiles use the direct path
    std::vector<int> tile_id(ntiles, -1);
    int T = 0;
    for (int t = 0; t < ntiles; ++t)
        if (owners_in[t] >= min_owners) tile_id[t] = T++;

    std::vector<std::vector<std::vector<int>>> trec(kNumLight, std::vector<std::vector<int>>(T));
    std::vector<std::vector<int>> ext_rows(T);             // external pods appended to each tile image
    std::vector<std::unordered_map<int, int>> ext_slot(T);  // pod -> image row
    std::vector<std::vector<int>> ell(kNumLight), midr(kNumMid);
    std::vector<std::vector<HeavyItem>> hitems(kNumHeavy);
    std::vector<int> hcol;
    std::vector<int> fresh;
    for (int i = 0; i < Q; ++i) {
        const int p = rows ? rows[i] : i;
        const int d = rp[p + 1] - rp[p];
        const int *nbp = ci.data() + rp[p];
        const int tile = pos[p] / CP;
        const int tid = tile_id[tile];
        bool tiled = d <= kLightMax && tid >= 0;
        if (tiled) {  // externals of this row must fit the tile image
            fresh.clear();
            for (int j = 0; j < d; ++j) {
                const int q = nbp[j];
                if (pos[q] / CP != tile && !ext_slot[tid].count(q) &&
                    std::find(fresh.begin(), fresh.end(), q) == fresh.end())
                    fresh.push_back(q);
            }
            tiled = (int)(ext_rows[tid].size() + fresh.size()) <= kTileXCap;
            if (tiled)
                for (int q : fresh) {
                    ext_slot[tid][q] = CP + (int)ext_rows[tid].size();
                    ext_rows[tid].push_back(q);
                }
        }
        if (tiled) {
            const int b = light_bucket(d);
            auto &e = trec[b][tid];
            const size_t o = e.size();
            e.resize(o + kLightW[b], 0);
            e[o] = i;
            e[o + 1] = d;
            for (int j = 0; j < d; ++j) {
                const int q = nbp[j];
                e[o + 2 + j] = pos[q] / CP == tile ? pos[q] % CP : ext_slot[tid][q];
            }
            plan->n_tile_owners += 1;
        } else if (d <= kLightMax) {
            const int b = light_bucket(d);
            auto &e = ell[b];
            const size_t o = e.size();
            e.resize(o + kLightW[b], 0);
            e[o] = i;
            e[o + 1] = d;
            for (int j = 0; j < d; ++j) e[o + 2 + j] = nbp[j];
            plan->n_light[b] += 1;
        } else if (d <= kMidMax) {
            const int b = d <= 32 ? 0 : (d <= 64 ? 1 : 2);
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
    plan->T = T;
    if (T > 0) {
        size_t xm = 0;
        for (auto &e : ext_rows) xm = std::max(xm, e.size());
        const int RS = CP + (int)((xm + 7) / 8 * 8);
        plan->RS = RS;
        std::vector<int> mem((size_t)T * RS, 0), nr(T, 0);
        for (int t = 0; t < ntiles; ++t) {
            const int id = tile_id[t];
            if (id < 0) continue;
            for (int k = 0; k < CP && t * CP + k < P; ++k) mem[(size_t)id * RS + k] = order[t * CP + k];
            for (size_t x = 0; x < ext_rows[id].size(); ++x) mem[(size_t)id * RS + CP + x] = ext_rows[id][x];
            nr[id] = CP + (int)ext_rows[id].size();  // short last tile: rows past its members are never read
        }
        RSK_TRY(upload(plan->members, mem.data(), mem.size() * 4));
        RSK_TRY(upload(plan->nrows, nr.data(), nr.size() * 4));
        // per-tile record blob: buckets D = 16, 8, 4, 2 back to back, padded to 4 ints
        std::vector<int> blob, boff((size_t)T * (kNumLight + 2));
        for (int t = 0; t < T; ++t) {
            int *bo = boff.data() + (size_t)t * (kNumLight + 2);
            bo[0] = (int)blob.size();
            for (int b = 0; b < kNumLight; ++b) {
                bo[1 + b] = (int)blob.size();
                blob.insert(blob.end(), trec[b][t].begin(), trec[b][t].end());
            }
            bo[kNumLight + 1] = (int)blob.size();
            plan->blob_max = std::max(plan->blob_max, bo[kNumLight + 1] - bo[0]);
        }
        if (blob.empty()) blob.assign(4, 0);
        RSK_TRY(upload(plan->blob, blob.data(), blob.size() * 4));
        RSK_TRY(upload(plan->blob_off, boff.data(), boff.size() * 4));
    }
    for (int b = 0; b < kNumMid; ++b) RSK_TRY(upload(plan->mid[b], midr[b].data(), midr[b].size() * 4));
    for (int b = 0; b < kNumLight; ++b) RSK_TRY(upload(plan->ell[b], ell[b].data(), ell[b].size() * 4));
    for (int c = 0; c < kNumHeavy; ++c)
        RSK_TRY(upload(plan->heavy_items[c], hitems[c].data(), hitems[c].size() * sizeof(HeavyItem)));
    RSK_TRY(upload(plan->hcol, hcol.data(), hcol.size() * 4));
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
    auto plan = new rsk_car_plan();
    plan->ctx = ctx;
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
    int64_t light = 0, mid = 0, heavy = 0, tile_bytes = 0, ell_bytes = 0, mid_bytes = 0;
    int64_t heavy_bytes = (int64_t)plan->hcol.bytes;
    for (int b = 0; b < kNumLight; ++b) {
        light += plan->n_light[b];
        ell_bytes += (int64_t)plan->n_light[b] * kLightW[b] * 4;
    }
    for (int b = 0; b < kNumMid; ++b) {
        mid += plan->n_mid[b];
        mid_bytes += (int64_t)plan->n_mid[b] * kMidW[b] * 4;
    }
    for (int c = 0; c < kNumHeavy; ++c) {
        heavy += plan->n_heavy[c];
        heavy_bytes += (int64_t)plan->n_heavy[c] * (int64_t)sizeof(HeavyItem);
    }
    if (plan->T > 0)
        tile_bytes = (int64_t)plan->T * plan->RS * 4 + (int64_t)plan->T * 4 * (kNumLight + 3) +
                     (int64_t)plan->blob.bytes;
    const int64_t v[12] = {plan->n_tile_owners, light, mid, heavy, plan->T, plan->RS, plan->CP,
                           tile_bytes, ell_bytes, mid_bytes, heavy_bytes, plan->max_deg};
    const int m = n < 12 ? n : 12;
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
    if (plan->T > 0) {   // K1b tiles
        TileArgs a;
        std::memset(&a, 0, sizeof(a));
        a.sc = sc;
        a.members = plan->members.as<int>();
        a.nrows = plan->nrows.as<int>();
        a.blob = plan->blob.as<int>();
        a.blob_off = plan->blob_off.as<int>();
        a.assign = d_assign;
        a.SL = SL;
        a.RS = plan->RS;
        a.T = plan->T;
        a.blob_max = plan->blob_max;
        static const int ablate = [] { const char *e = getenv("RSK_ABLATE_TILE"); return e ? atoi(e) : 0; }();
        a.ablate = ablate;
        const size_t lds = (size_t)plan->RS * SL * 4 + (size_t)plan->blob_max * 4;
        RSK_CHECK(lds <= 160 * 1024, "tile image needs %zu B of LDS", lds);
        const int64_t blocks = chunks * plan->T;
        RSK_CHECK(blocks < INT32_MAX, "tile grid too large");
        if (lds > 64 * 1024)
            RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&car_tile_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        ScopedTimer tm(ctx, "car_tile");
        car_tile_kernel<<<dim3((unsigned)blocks), dim3(kTileWaves * 64), lds, ctx->stream>>>(a);
        RSK_HIP(hipGetLastError());
    }
    {   // K1a direct light rows
        LightArgs a;
        std::memset(&a, 0, sizeof(a));
        a.sc = sc;
        a.SL = SL;
        const int iters = 2;
        a.task_prefix[0] = 0;
        for (int b = 0; b < kNumLight; ++b) {
            a.ell[b] = plan->ell[b].as<int>();
            a.n_items[b] = plan->n_light[b];
            a.task_items[b] = kLightPK[b] * sc.PS * iters;
            a.task_prefix[b + 1] = a.task_prefix[b] + (int)ceil_div(plan->n_light[b], a.task_items[b]);
        }
        const int tasks = a.task_prefix[kNumLight];
        if (tasks > 0) {
            a.assign = d_assign;
            a.blocks_per_chunk = (int)ceil_div(tasks, 4);
            const int64_t blocks = chunks * a.blocks_per_chunk;
            RSK_CHECK(blocks < INT32_MAX, "light grid too large");
            ScopedTimer tm(ctx, "car_light");
            car_light_kernel<<<dim3((unsigned)blocks), dim3(256), 0, ctx->stream>>>(a);
            RSK_HIP(hipGetLastError());
        }
    }
    {   // K1c mid rows
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
        for (int wide = 0; wide < 2; ++wide) {
            const int waves = wide ? a.prefix[3] - a.prefix[2] : a.prefix[2] - a.prefix[0];
            if (waves <= 0) continue;
            a.blocks_per_chunk = (int)ceil_div(waves, 4);
            const int64_t blocks = chunks * a.blocks_per_chunk;
            RSK_CHECK(blocks < INT32_MAX, "mid grid too large");
            ScopedTimer tm(ctx, "car_mid");
            if (wide) car_mid_kernel<true><<<dim3((unsigned)blocks), dim3(256), 0, ctx->stream>>>(a);
            else car_mid_kernel<false><<<dim3((unsigned)blocks), dim3(256), 0, ctx->stream>>>(a);
            RSK_HIP(hipGetLastError());
        }
    }
    for (int c = 0; c < kNumHeavy; ++c) {   // K2
        const int n = plan->n_heavy[c];
        if (!n) continue;
        const HeavyGeom g = heavy_geometry(plan->heavy_dmax[c], S, N);
        RSK_CHECK(g.lds <= 160 * 1024, "heavy class %d needs %zu B of LDS", c, g.lds);
        const int64_t groups = ceil_div(S, g.G);
        RSK_CHECK(groups * n < INT32_MAX, "heavy grid too large");
        auto kern = g.direct ? &car_heavy_kernel<true> : &car_heavy_kernel<false>;
        if (g.lds > 64 * 1024)
            RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)g.lds));
        ScopedTimer tm(ctx, "car_heavy");
        kern<<<dim3((unsigned)(groups * n)), dim3(256), g.lds, ctx->stream>>>(
            plan->heavy_items[c].as<HeavyItem>(), n, plan->hcol.as<int>(), d_assign, d_key, S, N, g.G, g.dpad,
            g.H, g.NT, d_zcnt, d_zkey, d_target, d_score);
        RSK_HIP(hipGetLastError());
    }
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
