// rsk_car16.hip — the compact CAR path for N <= 65535 nodes (gfx950).
//
// Reference: the score loop + argmax of `communication`,
// rescheduling.py:183-214 (see rsk_car.hip for the full statement).
//
// car_prep_kernel  one pass over the node state per (node, scenario):
//                  code16[n*S+s] (rsk_car.h: 0 hazard, 1 rem < 0, 2+f(rem)
//                  monotone), optionally the exact nodekey[n*S+s] for the wide
//                  kernels, and the per-scenario zero case.
// car_tile16       rows of degree <= 32 in LDS tiles, like the wide tile
//                  kernel, but the image cell is ONE 32-bit word
//                  (code << 16 | node) and a workgroup covers 64 scenarios:
//                  per image row a wave-instruction reads 256 contiguous
//                  bytes of assign and gathers 128 contiguous bytes of codes
//                  (the wide kernel: 128 B + 128 B of 32-bit keys per 32
//                  scenarios) — a third fewer cache lines through the vector
//                  memory path, which bounds the kernel.  Ties decided by
//                  codes alone except equal codes >= 2 on distinct nodes,
//                  resolved exactly from cap / use (rare: the code spacing is
//                  1 below 16384 millicores and 2..32 up to 2^19).
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "rsk_side16.h"

namespace rsk {

#ifdef RSK_DEBUG_BOUNDS
static __device__ unsigned rsk_dbg16;
__device__ __forceinline__ unsigned dbg16(unsigned idx, unsigned lim, unsigned code) {
    if (idx < lim) return idx;
    atomicOr(&rsk_dbg16, code);
    return 0u;
}
#define RSK_B16(idx, lim, code) dbg16((unsigned)(idx), (unsigned)(lim), (code))
#else
#define RSK_B16(idx, lim, code) (idx)
#endif

// ---------------------------------------------------------------------------
// node state
// ---------------------------------------------------------------------------
template <int V>
struct VecT;
template <> struct VecT<1> { typedef int I; typedef uint8_t H; typedef unsigned short C; };
template <> struct VecT<4> { typedef int4 I; typedef uchar4 H; typedef ushort4 C; };

__device__ __forceinline__ void vec_get(const int &v, int (&o)[1]) { o[0] = v; }
__device__ __forceinline__ void vec_get(const int4 &v, int (&o)[4]) { o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w; }
__device__ __forceinline__ void vec_get(const uint8_t &v, int (&o)[1]) { o[0] = v; }
__device__ __forceinline__ void vec_get(const uchar4 &v, int (&o)[4]) { o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w; }
__device__ __forceinline__ int vec_make(const int (&k)[1]) { return k[0]; }
__device__ __forceinline__ int4 vec_make(const int (&k)[4]) { return make_int4(k[0], k[1], k[2], k[3]); }
__device__ __forceinline__ unsigned short cvec_make(const unsigned (&k)[1]) { return (unsigned short)k[0]; }
__device__ __forceinline__ ushort4 cvec_make(const unsigned (&k)[4]) {
    return make_ushort4((unsigned short)k[0], (unsigned short)k[1], (unsigned short)k[2], (unsigned short)k[3]);
}

// Small batches (N * S <= kPrepSmallCells, S <= kPrepSmallS; config 2 is
// 64 cells): max(cap) and the prep pass in one workgroup.
constexpr int kPrep0Threads = 1024;
constexpr int kPrepSmallCells = 32768, kPrepSmallS = 256;
__global__ __launch_bounds__(kPrep0Threads) void car_prep_small_kernel(const int *__restrict__ cap,
                                                                      const int *__restrict__ use,
                                                                      const uint8_t *__restrict__ haz, int N, int S,
                                                                      unsigned short *__restrict__ code,
                                                                      int *__restrict__ nodekey,
                                                                      int *__restrict__ zc_cnt,
                                                                      unsigned long long *__restrict__ zc_key,
                                                                      unsigned *__restrict__ zc_clear,
                                                                      int clear_words) {
    __shared__ int red[kPrep0Threads / 64];
    __shared__ int lcnt[kPrepSmallS];
    __shared__ unsigned long long lkey[kPrepSmallS];
    const int t = (int)threadIdx.x;
    int mc = 0;
    for (int n = t; n < N; n += kPrep0Threads) mc = max(mc, cap[n]);
    mc = dpp_max(mc);
    if ((t & 63) == 0) red[t >> 6] = mc;
    for (int i = t; i < S; i += kPrep0Threads) {
        lcnt[i] = 0;
        lkey[i] = 0ull;
    }
    __syncthreads();
    mc = red[0];
    for (int w = 1; w < kPrep0Threads / 64; ++w) mc = max(mc, red[w]);
    const int B = max(0, mc - 32766);  // the exact code window (rsk_car.h)
    for (int i = t; i < clear_words; i += kPrep0Threads) zc_clear[i] = 0u;  // the next execute's half
    if (code)
        for (int i = t; i < S; i += kPrep0Threads) code[(size_t)N * S + i] = 0;  // row N: no candidate
    for (int i = t; i < N * S; i += kPrep0Threads) {
        const int n = i / S, sc = i - n * S;
        const int rem = cap[n] - use[i];
        const bool h = haz[i] != 0;
        if (code) code[i] = (unsigned short)code16(rem, h, B);
        if (nodekey) nodekey[i] = h ? kKeyHaz : rem;
        if (!h) {
            atomicAdd(&lcnt[sc], 1);
            atomicMax(&lkey[sc], zc_pack(rem, n));
        }
    }
    __syncthreads();
    for (int i = t; i < S; i += kPrep0Threads) {
        zc_cnt[i] = lcnt[i];
        zc_key[i] = lkey[i];
    }
}

// Thread t -> (V consecutive scenarios, node chunk): V-wide loads of use /
// hazard per node.  Every workgroup first reduces max(cap) itself (the exact
// code window B = max(0, max(cap) - 32766), the same in every workgroup), so
// no launch precedes this one; workgroup 0 clears the other half of the
// double-buffered zero-case words for the next execute.  The zero case
// (non-hazard count, packed max of (rem, ~node)) is reduced in LDS per
// workgroup first — threads of one workgroup that share a scenario meet in one
// LDS slot — so a scenario receives one global atomic per workgroup.
// kGrp (kBlock 256, SV % 64 == 0): a workgroup takes 64 vector slots x 4 node
// chunks instead of 256 slots x 1 chunk, so its LDS reduction folds 4 chunks
// and a scenario's zero-case words receive 4x fewer global atomics (the
// slots' loads stay 64 consecutive 16-B words per wave).
template <int V, bool kCode, bool kKey, int kBlock = 256, bool kGrp = false>
__global__ __launch_bounds__(kBlock) void car_prep_kernel(const int *__restrict__ cap, const typename VecT<V>::I *__restrict__ use,
                                                       const typename VecT<V>::H *__restrict__ haz, int N, int SV,
                                                       int npb, unsigned total, typename VecT<V>::C *__restrict__ code,
                                                       typename VecT<V>::I *__restrict__ nodekey,
                                                       int *__restrict__ zc_cnt, unsigned long long *__restrict__ zc_key,
                                                       unsigned *__restrict__ zc_clear, int clear_words) {
    // kBlock 1024 only with SV <= 256: the slots never exceed 256
    static_assert(!kGrp || kBlock == 256, "grouped prep: 4 waves = 4 chunks");
    __shared__ int lcnt[256 * V];
    __shared__ unsigned long long lkey[256 * V];
    const unsigned t = blockIdx.x * (unsigned)kBlock + threadIdx.x;
    // vt: the thread's (chunk * SV + slot) work index; base: the vector slot of its LDS slot 0
    const unsigned gpr = kGrp ? (unsigned)SV / 64u : 1u;
    const unsigned vt = kGrp ? ((blockIdx.x / gpr) * 4u + (threadIdx.x >> 6)) * (unsigned)SV +
                                   (blockIdx.x % gpr) * 64u + (threadIdx.x & 63u)
                             : t;
    const unsigned base = kGrp ? (blockIdx.x % gpr) * 64u : (blockIdx.x * (unsigned)kBlock) % (unsigned)SV;
    const int nslot = kGrp ? 64 : min(256, SV);
    for (int i = threadIdx.x; i < nslot * V; i += kBlock) { lcnt[i] = 0; lkey[i] = 0ull; }
    __syncthreads();
    __shared__ int red[kBlock / 64];
    const int B = kCode ? max(0, block_capmax<kBlock>(cap, N, red) - 32766) : 0;  // the exact code window
    if (blockIdx.x == 0)  // the other half of the zero-case words, for the next execute
        for (int i = (int)threadIdx.x; i < clear_words; i += kBlock) zc_clear[i] = 0u;
    if (kCode && t < (unsigned)SV) {  // code row N: code 0 for every scenario (clamped invalid assignments)
        const unsigned z[V] = {};
        code[(size_t)N * SV + t] = cvec_make(z);
    }
    if (vt < total) {
        const int sv = (int)(vt % (unsigned)SV);
        const int n0 = (int)(vt / (unsigned)SV) * npb;
        const int n1 = min(N, n0 + npb);
        int cnt[V];
        unsigned long long best[V];
#pragma unroll
        for (int x = 0; x < V; ++x) { cnt[x] = 0; best[x] = 0ull; }
#pragma unroll 4
        for (int n = n0; n < n1; ++n) {
            const size_t idx = (size_t)n * SV + sv;
            int uu[V], hh[V], k[V];
            unsigned cd[V];
            vec_get(use[idx], uu);
            vec_get(haz[idx], hh);
            const int c = cap[n];
#pragma unroll
            for (int x = 0; x < V; ++x) {
                const int rem = c - uu[x];
                k[x] = hh[x] ? kKeyHaz : rem;
                cd[x] = code16(rem, hh[x] != 0, B);
                cnt[x] += hh[x] ? 0 : 1;
                const unsigned long long pk = hh[x] ? 0ull : zc_pack(rem, n);
                best[x] = pk > best[x] ? pk : best[x];
            }
            if (kKey) nodekey[idx] = vec_make(k);
            if (kCode) code[idx] = cvec_make(cd);
        }
        const int slot = (int)(((unsigned)sv + (unsigned)SV - base) % (unsigned)SV);  // < nslot
#pragma unroll
        for (int x = 0; x < V; ++x)
            if (cnt[x]) {
                atomicAdd(&lcnt[slot * V + x], cnt[x]);
                atomicMax(&lkey[slot * V + x], best[x]);
            }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nslot * V; i += kBlock)
        if (lcnt[i]) {
            const int s = (int)(((base + (unsigned)(i / V)) % (unsigned)SV) * V + (unsigned)(i % V));
            atomicAdd(&zc_cnt[s], lcnt[i]);
            atomicMax(&zc_key[s], lkey[i]);
        }
}

template <int V, int kBlock = 256, bool kGrp = false>
static int prep_launch(hipStream_t stream, const Prep16Args &a, int SV, int npb, unsigned total) {
    typedef typename VecT<V>::I I;
    typedef typename VecT<V>::H H;
    typedef typename VecT<V>::C C;
    // kGrp: (SV / 64) workgroups per 4 node chunks
    const dim3 grid(kGrp ? (unsigned)(SV / 64 * ceil_div(ceil_div(total, SV), 4)) : (unsigned)ceil_div(total, kBlock)),
        block(kBlock);
    const I *use = reinterpret_cast<const I *>(a.use);
    const H *haz = reinterpret_cast<const H *>(a.haz);
    C *code = reinterpret_cast<C *>(a.code);
    I *key = reinterpret_cast<I *>(a.nodekey);
    if (a.code && a.nodekey)
        car_prep_kernel<V, true, true, kBlock, kGrp><<<grid, block, 0, stream>>>(a.cap, use, haz, a.N, SV, npb, total, code, key, a.zc_cnt, a.zc_key,
                                                                 a.zc_clear, a.clear_words);
    else if (a.code)
        car_prep_kernel<V, true, false, kBlock, kGrp><<<grid, block, 0, stream>>>(a.cap, use, haz, a.N, SV, npb, total, code, key, a.zc_cnt, a.zc_key,
                                                                 a.zc_clear, a.clear_words);
    else
        car_prep_kernel<V, false, true, kBlock, kGrp><<<grid, block, 0, stream>>>(a.cap, use, haz, a.N, SV, npb, total, code, key, a.zc_cnt, a.zc_key,
                                                                 a.zc_clear, a.clear_words);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

static int launch_prep_main(hipStream_t stream, const Prep16Args &a);

int launch_prep(hipStream_t stream, const Prep16Args &a) {
    RSK_CHECK(a.code || a.nodekey, "prep: nothing to write");
    if ((int64_t)a.N * a.S <= kPrepSmallCells && a.S <= kPrepSmallS) {
        car_prep_small_kernel<<<1, kPrep0Threads, 0, stream>>>(a.cap, a.use, a.haz, a.N, a.S, a.code, a.nodekey,
                                                               a.zc_cnt, a.zc_key, a.zc_clear, a.clear_words);
        RSK_HIP(hipGetLastError());
        return RSK_OK;
    }
    return launch_prep_main(stream, a);
}

static int launch_prep_main(hipStream_t stream, const Prep16Args &a) {
    // 4 scenarios per thread when S % 4 == 0 (16-B use / key words, 8-B codes)
    const bool v4 = a.S % 4 == 0 && ((uintptr_t)a.use % 16) == 0 && ((uintptr_t)a.haz % 4) == 0;
    const int SV = v4 ? a.S / 4 : a.S;
    // Threads: more cost zero-case atomics, fewer cost bandwidth.  A scenario's
    // slot receives one atomic per workgroup over its node chunks — threads /
    // SV of them when SV >= 256, threads / 256 below — so aim at ~256 per slot:
    // 256 * max(SV, 256) threads within [2^16, 2^18] (config 3, SV = 1024:
    // 2^18; config 4, SV = 16: 2^16, prep 0.029 -> 0.024 ms).
    // Few scenarios (SV <= 64, e.g. config 4: SV = 16): workgroups of 1024
    // threads, 4 nodes per thread — a scenario's slot still takes one atomic per
    // workgroup (N * SV / 4096 of them), with 4x the loads in flight of 256-thread
    // workgroups at 13 nodes per thread (prep 17 us at 50k nodes x 64).
    if (v4 && SV <= 64) {
        // (2 or 1 nodes per thread, or 256-thread workgroups: 0.0186-0.070 against 0.0162 ms, profiles/r06g)
        const int npb = 4;
        const unsigned total = (unsigned)(ceil_div(a.N, npb) * SV);
        return prep_launch<4, 1024>(stream, a, SV, npb, total);
    }
    const int target_threads = (int)std::min<int64_t>(256 * 1024, std::max<int64_t>(65536, 256LL * std::max(SV, 256)));
    const int npb = (int)std::max<int64_t>(1, ceil_div((int64_t)a.N * SV, target_threads));
    const int64_t chunks = ceil_div(a.N, npb);
    const unsigned total = (unsigned)(chunks * SV);
    if (SV % 64 == 0)
        return v4 ? prep_launch<4, 256, true>(stream, a, SV, npb, total) : prep_launch<1, 256, true>(stream, a, SV, npb, total);
    return v4 ? prep_launch<4>(stream, a, SV, npb, total) : prep_launch<1>(stream, a, SV, npb, total);
}

// ---------------------------------------------------------------------------
// car_tile16: rows with deg <= 32 in LDS tiles (plan: rsk_car.hip TileBuilder).
//
// Workgroup = (tile, chunk of SL = 2^lsl scenarios), 4 waves; SL = 64 when
// S >= 64 (kL64: lane = scenario throughout, every record wave-uniform).
//   phase 1  image row r, scenario column c -> LDS cell
//              (code16[node, s] << 16) | node        node = assign[pod_r, s]
//            or kCellPad (code 0 = no candidate, node 0xffff = no real node)
//            when the assignment is outside [0, N).
//   phase 2  per record the degree-class scorer reads its cells from LDS,
//            stores one target word per lane.
// Every global access is issued from a clamped, always-valid index and never
// guarded by a lane-divergent branch (hipcc otherwise waits vmcnt(0) per
// element), except the exact tie resolution, which is rare.
// ---------------------------------------------------------------------------

// Image rows per tile the compact kernel is compiled for (the plan's rows_cap)
// and workgroups per CU it is register-sized for.
// 80 rows x 64 scenarios x 4 B = 20 KiB of LDS and <= 64 VGPRs: eight
// workgroups (32 waves) per CU, the occupancy that hides the load phase of one
// workgroup behind the store phase of others (measured: 144 rows / 4 per CU
// 0.84 ms, 96 / 6 0.75, 88 / 7 0.72, 80 / 8 0.715, 64 / 8 0.76 at config 3).
#ifndef RSK_TILE16_ROWS
#define RSK_TILE16_ROWS 80
#endif
#ifndef RSK_TILE16_WGS
#define RSK_TILE16_WGS 8
#endif
#ifndef RSK_TILE16_WGS_GENERIC
#define RSK_TILE16_WGS_GENERIC 6  // the generic (S < 64) tiles: records and a work counter in LDS too
#endif
constexpr int kT16Rows = RSK_TILE16_ROWS;
static_assert(kT16Rows % 4 == 0 && kT16Rows <= kTileRows, "bad RSK_TILE16_ROWS");

#ifndef RSK_TILE_NT
#define RSK_TILE_NT 3  // streamed image loads / target stores non-temporal (codes stay in L2)
#endif

struct Lane16 {
    int col;    // image column of the lane's (clamped) scenario
    int s;      // clamped scenario
    int slot, PS;
    int zt, zs; // zero-case target / score
};

template <bool kOff32>
__device__ __forceinline__ size_t cell_off(unsigned i, unsigned S, unsigned s) {
    if (kOff32) return (size_t)((i * S + s) << 2);
    return ((size_t)i * S + s) << 2;
}

template <bool kScore, bool kOff32>
__device__ __forceinline__ void emit16(const Tile16Args &a, int oi, const Lane16 &L, int t, int sc) {
#ifdef RSK_DEBUG_BOUNDS
    if ((size_t)(unsigned)oi * a.S + L.s >= a.n_out || oi < 0) { atomicOr(&rsk_dbg16, 1u); return; }
#endif
    int *p = reinterpret_cast<int *>(reinterpret_cast<char *>(a.out_target) + cell_off<kOff32>((unsigned)oi, a.S, L.s));
    if (RSK_TILE_NT & 2) __builtin_nontemporal_store(t, p);
    else *p = t;
    if (kScore) {
        int *q = reinterpret_cast<int *>(reinterpret_cast<char *>(a.out_score) + cell_off<kOff32>((unsigned)oi, a.S, L.s));
        if (RSK_TILE_NT & 2) __builtin_nontemporal_store(sc, q);
        else *q = sc;
    }
}

// Exact remaining CPU of node n in scenario s (a code >= 2: not hazard).
__device__ __forceinline__ int exact_rem(const Tile16Args &a, int n, int s) {
    return a.cap[n] - ld32(a.use, (unsigned)n * (unsigned)a.S + (unsigned)s);
}

struct Img16 {
    const unsigned *w;
    int lsl;
    __device__ __forceinline__ unsigned at(int row, int col) const { return w[(row << lsl) + col]; }
};

// d == 1: the neighbour's node unless it is no candidate (zero case).
template <int U, bool kScore, bool kOff32>
__device__ __forceinline__ void t16_d1(const Tile16Args &a, const Img16 &img, const int *rec, int n, const Lane16 &L,
                                       int p0) {
    const int2 *r2 = reinterpret_cast<const int2 *>(rec);
    int2 r[U];
    unsigned c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = r2[min((p0 + u) * L.PS + L.slot, n - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = img.at(r[u].y, L.col);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const bool z = cell_code(c[u]) == kCodeHaz;
        emit16<kScore, kOff32>(a, r[u].x, L, z ? L.zt : cell_node(c[u]), z ? L.zs : 1);
    }
}

// d == 2: same node -> score 2; one no-candidate -> the other; two distinct
// candidates -> a tie of two: larger remaining CPU, then lower index, None
// when that remaining CPU is < 0.
template <int U, bool kScore, bool kOff32>
__device__ __forceinline__ void t16_d2(const Tile16Args &a, const Img16 &img, const int *rec, int n, const Lane16 &L,
                                       int p0) {
    const int2 *r2 = reinterpret_cast<const int2 *>(rec);
    int2 r[U];
    unsigned c0[U], c1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = r2[min((p0 + u) * L.PS + L.slot, n - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        c0[u] = img.at(r[u].y & 0xffff, L.col);
        c1[u] = img.at((int)((unsigned)r[u].y >> 16), L.col);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const unsigned k0 = cell_code(c0[u]), k1 = cell_code(c1[u]);
        const unsigned w0 = k0 ? cell_cand(c0[u]) : 0u, w1 = k1 ? cell_cand(c1[u]) : 0u;
        const unsigned best = max(w0, w1);
        const bool same = c0[u] == c1[u];
        const bool single = w0 == 0u || w1 == 0u || same;
        int t = cand_node(best);
        if (!single && cell_code(best) < 2u) t = RSK_TARGET_NONE;
        if (!single && k0 == k1 && code_inexact(k0)) {  // equal inexact codes: exact remaining CPU (rare)
            const int n0 = cell_node(c0[u]), n1 = cell_node(c1[u]);
            const int e0 = exact_rem(a, n0, L.s), e1 = exact_rem(a, n1, L.s);
            t = (e0 > e1 || (e0 == e1 && n0 < n1)) ? n0 : n1;
        }
        const bool zero = best == 0u;
        emit16<kScore, kOff32>(a, r[u].x, L, zero ? L.zt : t, zero ? L.zs : (same ? 2 : 1));
    }
}

template <int W>
__device__ __forceinline__ void load_rec16(const int *rec, int (&r)[W]) {
    const int4 *r4 = reinterpret_cast<const int4 *>(rec);
#pragma unroll
    for (int w = 0; w < W / 4; ++w) {
        const int4 x = r4[w];
        r[4 * w] = x.x; r[4 * w + 1] = x.y; r[4 * w + 2] = x.z; r[4 * w + 3] = x.w;
    }
}

// Exact resolution among candidates whose word's code equals `bk`: max exact
// remaining CPU, then the lower node.
template <int D>
__device__ __forceinline__ int exact_among(const Tile16Args &a, const unsigned (&w)[D], unsigned bk, int s) {
    int br = INT_MIN, bn = INT_MAX;
#pragma unroll
    for (int j = 0; j < D; ++j)
        if (cell_code(w[j]) == bk) {
            const int nd = cand_node(w[j]);
            const int e = exact_rem(a, nd, s);
            if (e > br || (e == br && nd < bn)) { br = e; bn = nd; }
        }
    return bn;
}

// 0 or 3 <= d <= D (D = 4, 8, 16): pairwise equality counts of the cells in
// registers — equal cells are the same node (in one scenario a node has one
// code) — c[j] = #{i < j : cell i == cell j}, so a node's last entry holds its
// count - 1 and the entries at the maximum are exactly one per maximal node.
template <int D, int W, int kR0, bool kScore, bool kOff32>
__device__ __forceinline__ void t16_dn(const Tile16Args &a, const Img16 &img, const int *rec, int n, const Lane16 &L,
                                       int p0) {
    int r[W];
    load_rec16<W>(rec + min(p0 * L.PS + L.slot, n - 1) * W, r);
    const int d = r[1];
    unsigned x[D];
    int c[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const unsigned pr = (unsigned)r[kR0 + j / 2];
        const int row = (j & 1) ? (int)(pr >> 16) : (int)(pr & 0xffffu);
        const unsigned e = img.at(row, L.col);  // padding entries read row 0
        x[j] = j < d ? e : kCellPad;
        c[j] = 0;
    }
#pragma unroll
    for (int j = 1; j < D; ++j)
#pragma unroll
        for (int i = 0; i < j; ++i) c[j] += x[j] == x[i];
    int M1 = -1;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        c[j] = cell_code(x[j]) == kCodeHaz ? -1 : c[j];
        M1 = max(M1, c[j]);
    }
    unsigned w[D], best = 0u;
    int nm = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const bool m = c[j] == M1;
        w[j] = m ? cell_cand(x[j]) : 0u;
        best = max(best, w[j]);
        nm += m;
    }
    const unsigned bk = cell_code(best);
    int t = nm == 1 ? cand_node(best) : (bk >= 2u ? cand_node(best) : RSK_TARGET_NONE);
    if (nm > 1 && code_inexact(bk)) {
        int namb = 0;
#pragma unroll
        for (int j = 0; j < D; ++j) namb += cell_code(w[j]) == bk;
        if (namb > 1) t = exact_among<D>(a, w, bk, L.s);
    }
    emit16<kScore, kOff32>(a, r[0], L, M1 < 0 ? L.zt : t, M1 < 0 ? L.zs : M1 + 1);
}

// Decision over sorted cells (equal nodes in runs): two walks — the maximal
// run length M over candidate nodes and how many runs reach it, then the best
// (code, -node) word among those runs and how many share its code.  Returns
// INT_MIN when no neighbour node is a candidate (M = 0: the caller applies the
// zero case); `need` when equal codes >= 2 tie (exact resolution required).
template <int D>
__device__ __forceinline__ int sorted_runs_decide(const unsigned (&x)[D], int &score, unsigned &bk_out, bool &need) {
    int M = 0, Rn = 0, namb = 0;
    unsigned bw = 0u;
    int c = 0;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        c = (i > 0 && x[i] == x[i > 0 ? i - 1 : 0]) ? c + 1 : 1;
        const bool end = i == D - 1 || x[i < D - 1 ? i + 1 : i] != x[i];
        const bool cand = end && cell_code(x[i]) != kCodeHaz;
        const bool gt = cand && c > M, eq = cand && c == M;
        Rn = gt ? 1 : (eq ? Rn + 1 : Rn);
        M = gt ? c : M;
    }
    c = 0;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        c = (i > 0 && x[i] == x[i > 0 ? i - 1 : 0]) ? c + 1 : 1;
        const bool end = i == D - 1 || x[i < D - 1 ? i + 1 : i] != x[i];
        const bool cand = end && c == M && cell_code(x[i]) != kCodeHaz;
        const unsigned wv = cand ? cell_cand(x[i]) : 0u;
        const unsigned kw = cell_code(wv), kb = cell_code(bw);
        namb = kw > kb ? 1 : (cand && kw == kb ? namb + 1 : namb);
        bw = max(bw, wv);
    }
    score = M;
    const unsigned bk = cell_code(bw);
    bk_out = bk;
    need = M > 0 && Rn > 1 && code_inexact(bk) && namb > 1;
    if (M == 0) return INT_MIN;
    return Rn == 1 ? cand_node(bw) : (bk >= 2u ? cand_node(bw) : RSK_TARGET_NONE);
}

// The same decision in one walk: the two largest (run length, code, -node)
// keys over the runs of candidate nodes.  The second key tells whether
// another node reaches the maximal count (a tie) and, being the best of the
// others, whether one of them shares the best code (exact resolution).
template <int D>
__device__ __forceinline__ int sorted_runs_top2(const unsigned (&x)[D], int &score, unsigned &bk_out, bool &need) {
    unsigned long long k1 = 0ull, k2 = 0ull;
    int c = 0;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        c = (i > 0 && x[i] == x[i > 0 ? i - 1 : 0]) ? c + 1 : 1;
        const bool end = i == D - 1 || x[i < D - 1 ? i + 1 : i] != x[i];
        const bool cand = end && cell_code(x[i]) != kCodeHaz;
        const unsigned long long k = cand ? ((unsigned long long)c << 32) | cell_cand(x[i]) : 0ull;
        const bool g1 = k > k1;
        k2 = g1 ? k1 : (k > k2 ? k : k2);
        k1 = g1 ? k : k1;
    }
    const int M = (int)(k1 >> 32);
    const unsigned bw = (unsigned)k1, bk = cell_code(bw);
    const bool tie = (int)(k2 >> 32) == M;
    score = M;
    bk_out = bk;
    need = M > 0 && tie && code_inexact(bk) && cell_code((unsigned)k2) == bk;
    if (M == 0) return INT_MIN;
    return !tie ? cand_node(bw) : (bk >= 2u ? cand_node(bw) : RSK_TARGET_NONE);
}

#ifndef RSK_RUNS_TOP2
#define RSK_RUNS_TOP2 1
#endif
template <int D>
__device__ __forceinline__ int sorted_runs(const unsigned (&x)[D], int &score, unsigned &bk_out, bool &need) {
    if (RSK_RUNS_TOP2) return sorted_runs_top2<D>(x, score, bk_out, need);
    return sorted_runs_decide<D>(x, score, bk_out, need);
}

// Exact tie resolution straight from the LDS image (rare path, kept free of
// register arrays): among the row's distinct nodes with code bk and count M,
// the largest exact remaining CPU, then the lower node.
__device__ __forceinline__ int t16_exact_scan(const Tile16Args &a, const Img16 &img, const int *rows, int d, int col, int M,
                                           unsigned bk, int s) {
    int br = INT_MIN, bn = INT_MAX;
#pragma unroll 1
    for (int j = 0; j < d; ++j) {
        const unsigned cj = img.at((int)(((unsigned)rows[j >> 1] >> ((j & 1) * 16)) & 0xffffu), col);
        if (cell_code(cj) != bk) continue;
        int cnt = 0;
#pragma unroll 1
        for (int i = 0; i < d; ++i)
            cnt += img.at((int)(((unsigned)rows[i >> 1] >> ((i & 1) * 16)) & 0xffffu), col) == cj;
        if (cnt != M) continue;
        const int nd = cell_node(cj);
        const int e = exact_rem(a, nd, s);
        if (e > br || (e == br && nd < bn)) { br = e; bn = nd; }
    }
    return bn;
}

// kL64 phase 1 of one wave: image rows [r0, rend), at most kB of them, lane =
// scenario.  Rows past rend re-read row rend - 1 (same lines, no LDS write).
// An assignment outside [0, N) is clamped to node N, whose code row the prep
// kernel zeroes (code 0: never a candidate), so the cell needs no validity
// select; the code offset is one 24-bit multiply-add (N <= 65535, 2S < 2^24:
// rsk_car.hip routes larger S to the wide path).  Lanes past S load scenario
// S - 1 into columns no scorer reads (W64 columns are clamped).
template <int kB, bool kOff32>
__device__ __forceinline__ void t16_rows64(const Tile16Args &a, unsigned *img, int img_off, int r0, int rend, int s0) {
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    const char *__restrict__ asg = reinterpret_cast<const char *>(a.assign);
    const char *__restrict__ codeb = reinterpret_cast<const char *>(a.code);
    const int lane = threadIdx.x & 63;
    const int s = s0 + lane;
    const unsigned sl = (unsigned)min(s, (int)S - 1);
    const unsigned S2 = 2u * S, sl2 = 2u * sl;
    const cint_ptr pods = const_ptr(a.img_pods) + img_off + r0;
    const int nr = rend - r0;  // >= 1 except for waves past the image
    if (nr <= 0) return;
    int v[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) {
        const int ur = u < nr ? u : nr - 1;
        const unsigned qd = (unsigned)pods[ur];
#ifdef RSK_DEBUG_BOUNDS
        if (img_off + r0 + ur >= (int)a.n_pods) atomicOr(&rsk_dbg16, 2u);
        if ((size_t)qd * S + sl >= a.n_assign) atomicOr(&rsk_dbg16, 4u);
#endif
        const int *pa = reinterpret_cast<const int *>(asg + cell_off<kOff32>(RSK_B16(qd, a.n_assign / S, 4u), S, sl));
        v[u] = (RSK_TILE_NT & 1) ? __builtin_nontemporal_load(pa) : *pa;
    }
    unsigned cd[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) {
        v[u] = (int)min((unsigned)v[u], N);
        // (profiling ablation 8: every code gather from node 0's line — the code-line traffic by difference)
        const unsigned off = (RSK_ABL(a) & 8) ? sl2 : __umul24((unsigned)v[u], S2) + sl2;
#ifdef RSK_DEBUG_BOUNDS
        if (off / 2u >= a.n_key + S) atomicOr(&rsk_dbg16, 8u);
#endif
        cd[u] = *reinterpret_cast<const unsigned short *>(codeb + off);
    }
    unsigned *dst = img + (r0 << 6) + lane;
#pragma unroll
    for (int u = 0; u < kB; ++u)
        if (u < nr) dst[u << 6] = (cd[u] << 16) | (unsigned)v[u];
}

// Phase 1.  kL64 (t16_rows64): the pod index is wave-uniform (scalar load),
// the assign slice one 256-B row, the code gather one 128-B line whenever the
// row's pod sits on one node in all 64 scenarios.
// Generic (SL < 64): lanes = (row, scenario) pairs as in the wide kernel.
template <bool kL64, bool kOff32>
__device__ __forceinline__ void t16_load_image(const Tile16Args &a, unsigned *img, int img_off, int nrows, int s0) {
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    const char *__restrict__ asg = reinterpret_cast<const char *>(a.assign);
    const unsigned short *__restrict__ code = a.code;
    if (kL64) {
        // wave w loads image rows [w*q, w*q + q), q = ceil(nrows / 4): the pod
        // list is read with wide scalar loads, all q rows in flight at once
        const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
        const int q = (nrows + 3) >> 2;
        const int r0 = wave * q;
        const int rend = min(r0 + q, nrows);
        if (q <= 8) t16_rows64<8, kOff32>(a, img, img_off, r0, rend, s0);
        else if (q <= 16) t16_rows64<16, kOff32>(a, img, img_off, r0, rend, s0);
        else if (q <= 24 || kT16Rows <= 96) t16_rows64<kT16Rows <= 96 ? kT16Rows / 4 : 24, kOff32>(a, img, img_off, r0, rend, s0);
        else if (q <= 28) t16_rows64<28, kOff32>(a, img, img_off, r0, rend, s0);
        else if (q <= 32) t16_rows64<32, kOff32>(a, img, img_off, r0, rend, s0);
        else t16_rows64<kT16Rows / 4, kOff32>(a, img, img_off, r0, rend, s0);
    } else {
        const int *__restrict__ pods = a.img_pods + img_off;
        constexpr int kE = kTileRows * 32 / kTileThreads;
        const int total = nrows << a.lsl;
        const int msk = (1 << a.lsl) - 1;
        for (int b = 0; b < total; b += kTileThreads * kE) {
            int e[kE], v[kE];
#pragma unroll
            for (int u = 0; u < kE; ++u) {
                e[u] = min(b + u * kTileThreads + (int)threadIdx.x, total - 1);
                const unsigned q = (unsigned)pods[RSK_B16(e[u] >> a.lsl, a.n_pods - img_off, 2u)];
                const unsigned s = (unsigned)min(s0 + (e[u] & msk), (int)S - 1);
                const int *pa = reinterpret_cast<const int *>(asg + cell_off<kOff32>(RSK_B16(q, a.n_assign / S, 4u), S, s));
                v[u] = *pa;
            }
            unsigned cd[kE];
#pragma unroll
            for (int u = 0; u < kE; ++u) {
                const int s = s0 + (e[u] & msk);
                const bool ok = (unsigned)v[u] < N && s < (int)S;
                cd[u] = ld16(code, RSK_B16(ok ? (unsigned)v[u] * S + (unsigned)s : 0u, a.n_key, 8u));
            }
#pragma unroll
            for (int u = 0; u < kE; ++u) {
                const int s = s0 + (e[u] & msk);
                const bool ok = (unsigned)v[u] < N && s < (int)S;
                img[e[u]] = ok ? ((cd[u] << 16) | (unsigned)v[u]) : kCellPad;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// kL64 scoring (S >= 64): lane = scenario column, every record wave-uniform.
// Wave w takes the records of each class in blocks round-robin over the four
// waves; records are read through the scalar cache straight from the plan
// (no LDS copy, no work-unit atomics), so per record a wave issues its cell
// reads (one ds_read_b32 per neighbour), the scorer's VALU and one 256-B
// target store whose address is a scalar base + the lane's column.
// ---------------------------------------------------------------------------
struct W64 {
    const char *img;  // LDS image, rows of 256 B
    unsigned col4;    // lane's (clamped) column * 4
    int s;            // lane's clamped scenario
    int zt, zs;       // zero-case target / score
    __device__ __forceinline__ unsigned cell(int row) const {
        return *reinterpret_cast<const unsigned *>(img + ((unsigned)row << 8) + col4);
    }
};

template <bool kScore, bool kOff32>
__device__ __forceinline__ void emit64(const Tile16Args &a, int oi, int s0, const W64 &w, int t, int sc) {
#ifdef RSK_DEBUG_BOUNDS
    if ((size_t)(unsigned)oi * a.S + w.s >= a.n_out || oi < 0) { atomicOr(&rsk_dbg16, 1u); return; }
#endif
    const size_t row = kOff32 ? (size_t)(((unsigned)oi * (unsigned)a.S + (unsigned)s0) << 2)
                              : ((size_t)(unsigned)oi * (unsigned)a.S + (unsigned)s0) << 2;
    int *p = reinterpret_cast<int *>(reinterpret_cast<char *>(a.out_target) + row + w.col4);
    if (RSK_TILE_NT & 2) __builtin_nontemporal_store(t, p);
    else *p = t;
    if (kScore) {
        int *q = reinterpret_cast<int *>(reinterpret_cast<char *>(a.out_score) + row + w.col4);
        if (RSK_TILE_NT & 2) __builtin_nontemporal_store(sc, q);
        else *q = sc;
    }
}

// Record blocks through the scalar cache: U two-int records from index k as
// U/2 unconditional 16-B scalar loads (the plan pads the blobs, so a block
// may run past its class; those records are masked, never stored).
template <int U>
__device__ __forceinline__ void rec_pairs(cint_ptr R, int k, int (&x)[U], int (&y)[U]) {
    const cint_ptr p = R + 2 * k;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        x[u] = p[2 * u];
        y[u] = p[2 * u + 1];
    }
}

// d == 1, U records from index k: {oi, row}
template <int U, bool kScore, bool kOff32>
__device__ __forceinline__ void w64_d1(const Tile16Args &a, const W64 &w, cint_ptr R, int n, int k, int s0) {
    int oi[U], row[U];
    unsigned c[U];
    rec_pairs<U>(R, k, oi, row);
#pragma unroll
    for (int u = 0; u < U; ++u) c[u] = w.cell(k + u < n ? row[u] : 0);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (k + u < n) {
            const bool z = cell_code(c[u]) == kCodeHaz;
            emit64<kScore, kOff32>(a, oi[u], s0, w, z ? w.zt : cell_node(c[u]), z ? w.zs : 1);
        }
}

// d == 2, U records from index k: {oi, row0 | row1 << 16}
template <int U, bool kScore, bool kOff32>
__device__ __forceinline__ void w64_d2(const Tile16Args &a, const W64 &w, cint_ptr R, int n, int k, int s0) {
    int oi[U], rr[U];
    unsigned c0[U], c1[U];
    rec_pairs<U>(R, k, oi, rr);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const unsigned pr = k + u < n ? (unsigned)rr[u] : 0u;
        c0[u] = w.cell((int)(pr & 0xffffu));
        c1[u] = w.cell((int)(pr >> 16));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (k + u >= n) continue;
        const unsigned k0 = cell_code(c0[u]), k1 = cell_code(c1[u]);
        const unsigned w0 = k0 ? cell_cand(c0[u]) : 0u, w1 = k1 ? cell_cand(c1[u]) : 0u;
        const unsigned best = max(w0, w1);
        const bool same = c0[u] == c1[u];
        const bool single = w0 == 0u || w1 == 0u || same;
        int t = cand_node(best);
        if (!single && cell_code(best) < 2u) t = RSK_TARGET_NONE;
        if (!single && k0 == k1 && code_inexact(k0)) {  // equal inexact codes: exact remaining CPU (rare)
            const int n0 = cell_node(c0[u]), n1 = cell_node(c1[u]);
            const int e0 = exact_rem(a, n0, w.s), e1 = exact_rem(a, n1, w.s);
            t = (e0 > e1 || (e0 == e1 && n0 < n1)) ? n0 : n1;
        }
        const bool zero = best == 0u;
        emit64<kScore, kOff32>(a, oi[u], s0, w, zero ? w.zt : t, zero ? w.zs : (same ? 2 : 1));
    }
}

// 0 or 3 <= d <= D (D = 4, 8, 16, 32), record j at R[W * j]: [oi, d, rows
// from int kR0].  One pass over the cells, registers only for the D cells:
// entry e's count c = #{earlier entries equal to it} (equal cells are the same
// node: in one scenario a node has one code), so a node with k entries shows
// c = 0 .. k-1 and the entries at the running maximum c = M are exactly one
// per node with M + 1 entries.  Running over candidates (code != 0): M, R =
// nodes at M, the best (code, -node) word among them and how many of them
// share its code (> 1 with a code >= 2: the rare exact resolution).
//
// Fast path first: when no lane of the wave holds two equal cells (distinct
// pads: kCellPad - i, code 0), every candidate node has count 1, so the answer
// is the largest candidate word, score 1; only a best code of 1 (None unless a
// single candidate) or an inexact best code shared by another entry needs a
// second look (rare, wave-uniform).  The pair tests cost one compare each
// (lane masks OR-ed on the scalar unit) against compare + add + the running
// state per entry of the counting walk below.
template <int D, int W, int kR0, bool kScore, bool kOff32>
__device__ __forceinline__ void w64_dm(const Tile16Args &a, const W64 &w, cint_ptr R, int j, int s0) {
    const cint_ptr r = R + W * j;
    const int d = r[1];
    unsigned x[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        const unsigned pr = (unsigned)r[kR0 + i / 2];
        const int row = (i & 1) ? (int)(pr >> 16) : (int)(pr & 0xffffu);
        x[i] = i < d ? w.cell(row) : kCellPad - (unsigned)i;
    }
    bool dup = false;
#pragma unroll
    for (int e = 1; e < D; ++e)
#pragma unroll
        for (int h = 0; h < e; ++h) dup |= x[h] == x[e];
    if (!__builtin_amdgcn_ballot_w64(dup)) {
        unsigned bw = 0u;
#pragma unroll
        for (int e = 0; e < D; ++e) bw = max(bw, cell_cand(x[e]));  // code 0 words stay below every candidate
        const unsigned bk = cell_code(bw);
        int t = cand_node(bw);
        if (__builtin_amdgcn_ballot_w64(bk == kCodeNeg || code_inexact(bk))) {  // rare: wave-uniform branch
            int rn = 0, nb = 0;
#pragma unroll
            for (int e = 0; e < D; ++e) {
                rn += cell_code(x[e]) != kCodeHaz;
                nb += cell_code(x[e]) == bk;
            }
            if (bk == kCodeNeg && rn > 1) t = RSK_TARGET_NONE;
            const bool need = code_inexact(bk) && nb > 1;
            if (__builtin_amdgcn_ballot_w64(need)) {
                Img16 im;
                im.w = reinterpret_cast<const unsigned *>(w.img);
                im.lsl = 6;
                const int te = t16_exact_scan(a, im, (const int *)(uintptr_t)(r + kR0), d, (int)(w.col4 >> 2), 1, bk, w.s);
                t = need ? te : t;
            }
        }
        emit64<kScore, kOff32>(a, r[0], s0, w, bk == kCodeHaz ? w.zt : t, bk == kCodeHaz ? w.zs : 1);
        return;
    }
#pragma unroll
    for (int i = 0; i < D; ++i) asm volatile("" : "+v"(x[i]));  // the walk recomputes its compares (no pair masks kept live)
    int M = -1, Rn = 0, namb = 0;
    unsigned bw = 0u;
#pragma unroll
    for (int e = 0; e < D; ++e) {
        if (D >= 16 && e % 8 == 0) __builtin_amdgcn_sched_barrier(0);  // bounds live registers
        int c = 0;
#pragma unroll
        for (int h = 0; h < e; ++h) c += x[h] == x[e];
        const bool cand = cell_code(x[e]) != kCodeHaz;
        const unsigned wv = cell_cand(x[e]);
        const bool gt = cand && c > M, eq = cand && c == M;
        const unsigned kw = cell_code(wv), kb = cell_code(bw);
        namb = gt ? 1 : (eq ? (kw > kb ? 1 : (kw == kb ? namb + 1 : namb)) : namb);
        bw = gt ? wv : (eq ? max(bw, wv) : bw);
        Rn = gt ? 1 : (eq ? Rn + 1 : Rn);
        M = gt ? c : M;
    }
    const unsigned bk = cell_code(bw);
    int t = Rn == 1 ? cand_node(bw) : (bk >= 2u ? cand_node(bw) : RSK_TARGET_NONE);
    const bool need = Rn > 1 && code_inexact(bk) && namb > 1;
    if (__builtin_amdgcn_ballot_w64(need)) {  // rare: wave-uniform branch
        Img16 im;
        im.w = reinterpret_cast<const unsigned *>(w.img);
        im.lsl = 6;
        const int te = t16_exact_scan(a, im, (const int *)(uintptr_t)(r + kR0), d, (int)(w.col4 >> 2), M + 1, bk, w.s);
        t = need ? te : t;
    }
    emit64<kScore, kOff32>(a, r[0], s0, w, M < 0 ? w.zt : t, M < 0 ? w.zs : M + 1);
}

// 17 <= d <= 32, record j at R[20 * j] ([oi, d, -, -, rows from int 4]): the
// counting walk of w64_dm with only the first 16 cells in registers.  Entry
// e's count c = #{earlier entries equal to it}: for e < 16 against the
// registers; for e >= 16 (cell read from the LDS image) against the 16
// registers plus the earlier entries >= 16, re-read from the LDS one at a time
// (<= 120 extra ds_read_b32 per record).  About 30 VGPRs, so the class fits
// the tile kernel's 64 and runs at 8 workgroups per CU (round 3's separate
// heavy-tile launch sorted all 32 cells in registers at 6 per CU: slower).
template <bool kScore, bool kOff32>
__device__ __forceinline__ void w64_ds_lean(const Tile16Args &a, const W64 &w, cint_ptr R, int j, int s0) {
    const cint_ptr r = R + 20 * j;
    const int d = r[1];
    auto row_of = [&](int i) -> int {
        const unsigned pr = (unsigned)r[4 + i / 2];
        return (i & 1) ? (int)(pr >> 16) : (int)(pr & 0xffffu);
    };
    unsigned x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = w.cell(row_of(i));  // d >= 17: all real cells
    int M = -1, Rn = 0, namb = 0;
    unsigned bw = 0u;
    auto put = [&](unsigned xe, int c) {
        const bool cand = cell_code(xe) != kCodeHaz;
        const unsigned wv = cell_cand(xe);
        const bool gt = cand && c > M, eq = cand && c == M;
        const unsigned kw = cell_code(wv), kb = cell_code(bw);
        namb = gt ? 1 : (eq ? (kw > kb ? 1 : (kw == kb ? namb + 1 : namb)) : namb);
        bw = gt ? wv : (eq ? max(bw, wv) : bw);
        Rn = gt ? 1 : (eq ? Rn + 1 : Rn);
        M = gt ? c : M;
    };
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        if (e % 8 == 0) __builtin_amdgcn_sched_barrier(0);
        int c = 0;
#pragma unroll
        for (int h = 0; h < e; ++h) c += x[h] == x[e];
        put(x[e], c);
    }
#pragma unroll 1
    for (int e = 16; e < d; ++e) {  // wave-uniform bound
        const unsigned xe = w.cell(row_of(e));
        int c = 0;
#pragma unroll
        for (int h = 0; h < 16; ++h) c += x[h] == xe;
#pragma unroll 1
        for (int h = 16; h < e; ++h) c += w.cell(row_of(h)) == xe;
        put(xe, c);
    }
    const unsigned bk = cell_code(bw);
    int t = Rn == 1 ? cand_node(bw) : (bk >= 2u ? cand_node(bw) : RSK_TARGET_NONE);
    const bool need = Rn > 1 && code_inexact(bk) && namb > 1;
    if (__builtin_amdgcn_ballot_w64(need)) {  // rare: wave-uniform branch
        Img16 im;
        im.w = reinterpret_cast<const unsigned *>(w.img);
        im.lsl = 6;
        const int te = t16_exact_scan(a, im, (const int *)(uintptr_t)(r + 4), d, (int)(w.col4 >> 2), M + 1, bk, w.s);
        t = need ? te : t;
    }
    emit64<kScore, kOff32>(a, r[0], s0, w, M < 0 ? w.zt : t, M < 0 ? w.zs : M + 1);
}

// kL64 phase 2, part 1: the multi-neighbour classes (d >= 3), most expensive
// first.  Record j of a class goes to wave (rot + j) % 4, rot carried from
// class to class (and into part 2), so a tile's few records of each class do
// not all start on wave 0.
template <bool kScore, bool kOff32>
__device__ __forceinline__ int w64_score_multi(const Tile16Args &a, const W64 &w, cint_ptr m, cint_ptr R, int wave,
                                               int s0) {
    int rot = 0;
    {   // d = 17..32: the register-light counting walk
        const cint_ptr Rc = R + m[15];
        for (int j = (wave - rot) & 3; j < m[9]; j += 4) w64_ds_lean<kScore, kOff32>(a, w, Rc, j, s0);
        rot = (rot + m[9]) & 3;
    }
    {
        const cint_ptr Rc = R + m[14];
        for (int j = (wave - rot) & 3; j < m[8]; j += 4) w64_dm<16, 12, 2, kScore, kOff32>(a, w, Rc, j, s0);
        rot = (rot + m[8]) & 3;
    }
    {
        const cint_ptr Rc = R + m[13];
        for (int j = (wave - rot) & 3; j < m[7]; j += 4) w64_dm<8, 8, 2, kScore, kOff32>(a, w, Rc, j, s0);
        rot = (rot + m[7]) & 3;
    }
    {
        const cint_ptr Rc = R + m[12];
        for (int j = (wave - rot) & 3; j < m[6]; j += 4) w64_dm<4, 4, 2, kScore, kOff32>(a, w, Rc, j, s0);
        rot = (rot + m[6]) & 3;
    }
    return rot;
}

// kL64 phase 2, part 2: d = 2 and d = 1 records in blocks of 8 (block b to
// wave (rot + b) % 4).
template <bool kScore, bool kOff32>
__device__ __forceinline__ void w64_score_light(const Tile16Args &a, const W64 &w, cint_ptr m, cint_ptr R, int wave,
                                                int s0, int rot) {
    constexpr int U = 8;
    {
        const cint_ptr Rc = R + m[11];
        const int n = m[5];
        for (int k = ((wave - rot) & 3) * U; k < n; k += 4 * U) w64_d2<U, kScore, kOff32>(a, w, Rc, n, k, s0);
        rot = (rot + (n + U - 1) / U) & 3;
    }
    {
        const cint_ptr Rc = R + m[10];
        const int n = m[4];
        for (int k = ((wave - rot) & 3) * U; k < n; k += 4 * U) w64_d1<U, kScore, kOff32>(a, w, Rc, n, k, s0);
    }
}

// kL64 phase 2: the records of each class, spread over the 4 waves.
template <bool kScore, bool kOff32>
__device__ __forceinline__ void w64_score(const Tile16Args &a, const W64 &w, cint_ptr m, cint_ptr R, int wave, int s0) {
    if (RSK_ABL(a) & 4) {  // profiling: the target stores alone (every record, zero-case value, no LDS reads)
        for (int c = 0; c < kNumCls; ++c) {
            const cint_ptr Rc = R + m[10 + c];
            for (int j = wave; j < m[4 + c]; j += 4) emit64<kScore, kOff32>(a, Rc[kClsW[c] * j], s0, w, w.zt, w.zs);
        }
        return;
    }
    const int rot = w64_score_multi<kScore, kOff32>(a, w, m, R, wave, s0);
    w64_score_light<kScore, kOff32>(a, w, m, R, wave, s0, rot);
}

// One tile workgroup; bid plays blockIdx.x (the fused kernel below maps its
// own blocks onto tile blocks and side blocks).
template <bool kScore, bool kOff32, bool kL64>
__device__ __forceinline__ void tile16_block(const Tile16Args &a, unsigned bid) {
    extern __shared__ __attribute__((aligned(16))) int lds[];  // img cells [rmax][SL] (+ records, unit counter: !kL64)
    const int lsl = kL64 ? 6 : a.lsl;
    const int SL = 1 << lsl;
    const int nchunk = (a.S + SL - 1) >> lsl;
    // XCD-contiguous units: blocks b and b + 8 share an XCD, so XCD x walks
    // units [x * xcd_per, (x + 1) * xcd_per)
    const int unit = (int)(bid & 7u) * a.xcd_per + (int)(bid >> 3);
    if (unit >= nchunk * a.T) return;  // whole workgroup, before any barrier
    // ... in groups of kTileGroup chunks, each group walked tile-major: the
    // workgroups an XCD runs together read adjacent 256-B segments of the same
    // pod rows while a group's code slices stay in its L2
    int tile, chunk;
    {
        const int G = kTileGroup, full = nchunk / G;
        if (unit < full * a.T * G) {
            const int cg = unit / (a.T * G), r = unit - cg * a.T * G;
            tile = r / G;
            chunk = cg * G + (r - tile * G);
        } else {
            const int g = nchunk - full * G, r = unit - full * a.T * G;
            tile = r / g;
            chunk = full * G + (r - tile * g);
        }
    }
    const int lane = threadIdx.x & 63;
    const int s0 = chunk * SL;
    unsigned *img = reinterpret_cast<unsigned *>(lds);
    const cint_ptr m = const_ptr(a.meta) + (size_t)tile * kMetaW;
    const int img_off = m[0], nrows = m[1], rec_off = m[2], rec_ints = m[3];
    if (kL64) {
        if (!(RSK_ABL(a) & 1)) t16_load_image<true, kOff32>(a, img, img_off, nrows, s0);
        else for (int i = threadIdx.x; i < nrows * 64; i += kTileThreads) img[i] = kCellPad;  // ablation: no loads, no garbage
        W64 w;
        w.img = reinterpret_cast<const char *>(lds);
        w.s = min(s0 + lane, a.S - 1);
        w.col4 = (unsigned)(w.s - s0) << 2;
        {
            int zs;
            w.zt = zero_target(load_zc(a.zc_cnt, a.zc_key, w.s), zs);
            w.zs = zs;
        }
        __syncthreads();
        if (RSK_ABL(a) & 2) return;  // profiling ablation: no scoring (results are wrong)
        const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
        w64_score<kScore, kOff32>(a, w, m, const_ptr(a.recs) + RSK_B16(rec_off, a.n_recs, 16u), wave, s0);
        return;
    }
    int *rec = lds + a.img_cells;  // 16-B aligned (img_cells % 4 == 0) for the int4 record reads
    {   // records -> LDS: one int4 per thread, clamped
        const int i = min((int)threadIdx.x * 4, rec_ints - 4);
        *reinterpret_cast<int4 *>(rec + i) =
            *reinterpret_cast<const int4 *>(a.recs + RSK_B16(rec_off + i + 3, a.n_recs, 16u) - 3);
    }
    if (!(RSK_ABL(a) & 1)) t16_load_image<false, kOff32>(a, img, img_off, nrows, s0);
    else for (int i = threadIdx.x; i < (nrows << lsl); i += kTileThreads) img[i] = kCellPad;

    Lane16 L;
    L.PS = 64 >> lsl;
    L.slot = lane >> lsl;
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
    Img16 im;
    im.w = img;
    im.lsl = lsl;
    // Work units (PS records each: d1 4 x PS, d2 2 x PS, the rest PS), most
    // expensive class first, handed out by an LDS counter.
    const int n0 = m[4], n1 = m[5], n2 = m[6], n3 = m[7], n4 = m[8], n5 = m[9];
    const int lp = 6 - lsl;  // log2(PS)
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
            t16_dn<32, 20, 4, kScore, kOff32>(a, im, rec + m[15], n5, L, u);
        } else if ((u -= u5) < u4) {
            t16_dn<16, 12, 2, kScore, kOff32>(a, im, rec + m[14], n4, L, u);
        } else if ((u -= u4) < u3) {
            t16_dn<8, 8, 2, kScore, kOff32>(a, im, rec + m[13], n3, L, u);
        } else if ((u -= u3) < u2) {
            t16_dn<4, 4, 2, kScore, kOff32>(a, im, rec + m[12], n2, L, u);
        } else if ((u -= u2) < u1) {
            t16_d2<2, kScore, kOff32>(a, im, rec + m[11], n1, L, 2 * u);
        } else {
            t16_d1<4, kScore, kOff32>(a, im, rec + m[10], n0, L, 4 * (u - u1));
        }
        k = kn;
    }
}

template <bool kScore, bool kOff32, bool kL64>
__global__ __launch_bounds__(kTileThreads, kL64 ? RSK_TILE16_WGS : RSK_TILE16_WGS_GENERIC) void car_tile16_kernel(
    Tile16Args a) {
    tile16_block<kScore, kOff32, kL64>(a, blockIdx.x);
}

// Lean tiles and side rows (rsk_side16.h) in one grid, so the latency- and
// VALU-bound side work shares each CU with the memory-bound tile workgroups
// instead of running alone before them:
//   blocks [0, big_blocks)  one 4-wave side team each (the rows above 128
//                           neighbours): dispatched first, they run the
//                           longest;
//   then rows of 8 blocks (one block per XCD): in the first K1 periods of R
//   rows, the last row holds 4 single-wave side items per block (33..128
//   neighbours) and the other R - 1 are tile rows; then the remaining tile
//   rows; then the remaining side rows (when side rows outnumber the tile
//   rows the periods can hold).
// Every side workgroup fits the tile's footprint (4 waves, <= 64 VGPRs, its
// LDS within the tile's).
// (the side items keep their next assign rows in flight while a batch is scored)
//
// direct16_block: one (row, scenario) cell of the rows above the side classes
// (DirectArgs, targets only), in the front of the fused grid: the neighbours'
// nodes (hazard nodes skipped) counted in an LDS hash of packed words
// ((node + 1) << 16 | count: N <= 65535, degree < 65536), then the exact
// (cap - use, -node) maximum over the nodes at the max count, or the
// scenario's zero case from the prep kernel — rescheduling.py:183-214 on the
// deduplicated row without its self edge, as car_direct_kernel.
__device__ __forceinline__ void direct16_block(const DirectArgs &a, const Tile16Args &ta, int cell) {
    extern __shared__ __attribute__((aligned(16))) unsigned dtab[];
    const int H = a.H, S = a.S, N = a.N, t = (int)threadIdx.x;
    unsigned *red = dtab + H;                                                   // M, nbest
    unsigned long long *best64 = reinterpret_cast<unsigned long long *>(dtab + H + 2);  // (H even: 8-B aligned)
    const int k = cell / S, s = cell - k * S;
    const int i = a.items[(size_t)k * a.istride];
    const int p = a.rows ? a.rows[i] : i;
    const int b = a.rp[p], d = a.rp[p + 1] - b;
    for (int h = t; h < H + 4; h += kTileThreads) dtab[h] = 0u;
    __syncthreads();
    const unsigned mask = (unsigned)H - 1u;
    constexpr int kU = 4;  // neighbours in flight per thread (clamped, always-valid addresses)
    for (int j0 = t; j0 < d; j0 += kTileThreads * kU) {
        int q[kU], x[kU];
        uint8_t hz[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) q[u] = a.ci[b + min(j0 + u * kTileThreads, d - 1)];
#pragma unroll
        for (int u = 0; u < kU; ++u) x[u] = a.assign[(size_t)q[u] * S + s];
#pragma unroll
        for (int u = 0; u < kU; ++u) hz[u] = a.haz[(size_t)min((unsigned)x[u], (unsigned)N - 1u) * S + s];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            if (j0 + u * kTileThreads >= d || (unsigned)x[u] >= (unsigned)N || hz[u]) continue;
            const unsigned key = (unsigned)x[u] + 1u;
            unsigned h = (key * 2654435761u) & mask;
            while (true) {
                const unsigned prev = atomicCAS(&dtab[h], 0u, (key << 16) | 1u);
                if (prev == 0u) break;
                if ((prev >> 16) == key) { atomicAdd(&dtab[h], 1u); break; }
                h = (h + 1u) & mask;
            }
        }
    }
    __syncthreads();
    int m = 0;
    for (int h = t; h < H; h += kTileThreads) m = max(m, (int)(dtab[h] & 0xffffu));
    m = dpp_max(m);
    if ((t & 63) == 0 && m) atomicMax(&red[0], (unsigned)m);
    __syncthreads();
    const unsigned M = red[0];
    if (M > 0) {
        unsigned long long bk = 0;
        unsigned nb = 0;
        for (int h = t; h < H; h += kTileThreads) {
            const unsigned w = dtab[h];
            if ((w & 0xffffu) != M) continue;
            const int n = (int)(w >> 16) - 1;
            ++nb;
            const unsigned long long kk = pack_rn(a.cap[n] - a.use[(size_t)n * S + s], n);
            bk = kk > bk ? kk : bk;
        }
        if (nb) {
            atomicAdd(&red[1], nb);
            atomicMax(best64, bk);
        }
    }
    __syncthreads();
    if (t == 0) {
        int score, tg;
        if (M == 0) {
            tg = zero_target(load_zc(ta.zc_cnt, ta.zc_key, s), score);
        } else {
            CarState st;
            st.bc = (int)M;
            st.nm = red[1] == 1u ? (int)M : 0;  // one node at the max count: it, even if overloaded
            st.br = (int)((unsigned)(*best64 >> kNodeBits) ^ 0x80000000u);
            st.bn = (int)(kNodeMask - (unsigned)(*best64 & kNodeMask));
            tg = car_finalize(st, ZeroCase{}, score);
        }
        a.out_target[(size_t)i * S + s] = tg;
    }
}

template <bool kScore, bool kOff32, bool kDirect>
__global__ __launch_bounds__(kTileThreads, RSK_TILE16_WGS) void car_fused16_kernel(Tile16Args ta, SideArgs sa,
                                                                                  SideArgs ba, DirectArgs da,
                                                                                  FuseMap f) {
    if (kDirect && blockIdx.x < (unsigned)f.direct_blocks) {
        if ((int)blockIdx.x < da.Q * da.S) direct16_block(da, ta, (int)blockIdx.x);
        return;
    }
    const unsigned v0 = blockIdx.x - (unsigned)f.direct_blocks;
    if (v0 < (unsigned)f.big_blocks) {  // (XCD x: the x-th eighth of the chunk-major team items)
        side16_block<4, 4, 16, kOff32, true>(ba, (int)((v0 & 7u) * ((unsigned)f.big_blocks >> 3) + (v0 >> 3)));
        return;
    }
    const unsigned v = v0 - (unsigned)f.big_blocks, row = v >> 3, x = v & 7u;
    const unsigned R = (unsigned)f.R, K1 = (unsigned)f.k1, P1 = K1 * R;
    unsigned side = 0xffffffffu, tile;
    if (row < P1) {
        const unsigned k = row / R, m = row - k * R;
        if (m == R - 1u) side = k;
        tile = k * (R - 1u) + m;
    } else {
        const unsigned t_rem = (unsigned)f.tile_rows - K1 * (R - 1u);
        tile = K1 * (R - 1u) + (row - P1);
        if (row - P1 >= t_rem) side = K1 + (row - P1 - t_rem);
    }
    if (side != 0xffffffffu) {  // XCD x: the x-th eighth of the chunk-major items (its tiles' chunks)
        side16_block<4, 1, 16, kOff32, true>(sa, (int)(x * (unsigned)f.side_rows + side));
        return;
    }
    tile16_block<kScore, kOff32, true>(ta, (tile << 3) | x);
}

int launch_tile16(hipStream_t stream, const Tile16Args &a, bool score, bool off32, unsigned blocks, size_t lds) {
    using K = void (*)(Tile16Args);
    // [l64][score][off32]; the generic (S < 64) kernel scores every class
    static const K kerns[8] = {
        &car_tile16_kernel<false, false, false>, &car_tile16_kernel<false, true, false>,
        &car_tile16_kernel<true, false, false>,  &car_tile16_kernel<true, true, false>,
        &car_tile16_kernel<false, false, true>,  &car_tile16_kernel<false, true, true>,
        &car_tile16_kernel<true, false, true>,   &car_tile16_kernel<true, true, true>};
    const bool l64 = a.lsl == 6;
    RSK_CHECK(!l64 || (size_t)a.img_cells * 4 <= (size_t)kT16Rows * 256,
              "tile image exceeds the %d rows the kernel was built for", kT16Rows);
    const K kern = kerns[(l64 ? 4 : 0) + (score ? 2 : 0) + (off32 ? 1 : 0)];
    RSK_CHECK(lds <= 160 * 1024, "tile image needs %zu B of LDS", lds);
    if (lds > 64 * 1024)
        RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
    kern<<<dim3(blocks), dim3(kTileThreads), lds, stream>>>(a);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int direct16_table(int dmax, int N, size_t lds) {
    const int distinct = std::min(dmax, N);
    if (N > 65535 || dmax >= 65536) return 0;  // the packed (node + 1, count) words
    int H = 2;
    while (H < 2 * distinct) H <<= 1;          // load factor <= 1/2
    while (H > 2 && (size_t)(H + 4) * 4 > lds) H >>= 1;
    return H > distinct && (size_t)(H + 4) * 4 <= lds ? H : 0;
}

int launch_fused16(hipStream_t stream, const Tile16Args &a, const SideArgs &sa, int side_blocks, const SideArgs &ba,
                   const DirectArgs &da, bool score, bool off32, unsigned tile_blocks, size_t lds) {
    RSK_CHECK(a.lsl == 6 && (size_t)a.img_cells * 4 <= (size_t)kT16Rows * 256 && tile_blocks % 8 == 0,
              "fused launch needs 64-scenario tiles");
    const int64_t cells = (int64_t)da.Q * da.S;
    RSK_CHECK(cells == 0 || (!score && da.H > 0 && (size_t)(da.H + 4) * 4 <= lds && cells < INT32_MAX),
              "direct cells in the fused grid: targets only, a table within the tile's LDS");
#ifndef RSK_FUSE_SPREAD
#define RSK_FUSE_SPREAD 2
#endif
    constexpr int spread = RSK_FUSE_SPREAD;  // side rows over the first half of the tile rows (1 / 4 of them: slower)
    FuseMap f;
    f.direct_blocks = (int)(8 * ceil_div(cells, 8));  // (XCD alignment of the blocks after them)
    f.big_blocks = (int)(8 * ceil_div((int64_t)ba.n_rows * ba.nchunk, 8));
    // (side_blocks = ceil(items / 4): XCD x takes blocks [x * side_rows, (x + 1) * side_rows), chunk-major
    // items, so its side items read the code and assign columns of its own tiles' chunks)
    f.side_rows = (int)ceil_div(side_blocks, 8);
    f.tile_rows = (int)(tile_blocks / 8);
    // one side row every R rows over the first 1 / spread of the tile rows; the
    // side rows the periods cannot hold go after the tiles
    f.R = std::max(2, f.tile_rows / std::max(1, f.side_rows * spread));
    f.k1 = std::min(f.side_rows, f.tile_rows / (f.R - 1));
    const int64_t blocks = (int64_t)f.direct_blocks + f.big_blocks + tile_blocks + 8LL * f.side_rows;
    RSK_CHECK(blocks < INT32_MAX, "fused grid too large");
    using K = void (*)(Tile16Args, SideArgs, SideArgs, DirectArgs, FuseMap);
    // [direct][score][off32]; direct cells only without scores
    static const K kerns[6] = {&car_fused16_kernel<false, false, false>, &car_fused16_kernel<false, true, false>,
                               &car_fused16_kernel<true, false, false>,  &car_fused16_kernel<true, true, false>,
                               &car_fused16_kernel<false, false, true>,  &car_fused16_kernel<false, true, true>};
    const K kern = kerns[(cells ? 4 : 0) + (score ? 2 : 0) + (off32 ? 1 : 0)];
    RSK_CHECK(lds <= 160 * 1024, "fused tile needs %zu B of LDS", lds);
    if (lds > 64 * 1024)
        RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
    kern<<<dim3((unsigned)blocks), dim3(kTileThreads), lds, stream>>>(a, sa, ba, da, f);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

size_t tile16_lds_bytes(int rmax, int lsl, int rec_cap) {
    if (lsl == 6) return (size_t)rmax * 64 * 4;  // kL64: records are read from the plan, not LDS
    return ((((size_t)rmax << lsl) + 3) / 4 * 4 + (size_t)rec_cap + 4) * 4;
}

int tile16_rows_built() { return kT16Rows; }

unsigned tile16_debug_take() {
#ifdef RSK_DEBUG_BOUNDS
    unsigned f = 0, zero = 0;
    if (hipDeviceSynchronize() != hipSuccess) return 0x80000000u;
    if (hipMemcpyFromSymbol(&f, HIP_SYMBOL(rsk_dbg16), 4) != hipSuccess) return 0x80000000u;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(rsk_dbg16), &zero, 4);
    return f;
#else
    return 0u;
#endif
}

}  // namespace rsk
