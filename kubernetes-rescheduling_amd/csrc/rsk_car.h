// rsk_car.h — internals shared by the CAR sources of librsk.so:
//   rsk_car.hip    plan building, execute, the wide tile path (N > 65535),
//                  mid / hub rows for the wide path;
//   rsk_car16.hip  the compact path (N <= 65535): node-state prep, tiles with
//                  32-bit {code, node} cells;
//   rsk_side16.hip the compact path's side rows (degree above the tiles).
// Reference semantics: rescheduling.py:183-214 (see rsk_car.hip's header).
#pragma once

#include <climits>
#include <cstdint>

#include "rsk_common.h"
#include "rsk_plan.h"
#include "rsk_wave.h"

namespace rsk {

constexpr int kKeyHaz = INT_MIN;  // cap - use never reaches INT_MIN (both in [0, 2^31))
struct CarState {
    int bc;  // best count (max score); 0 = no non-hazard neighbour node
    int br;  // remaining CPU of the best node
    int bn;  // best node index
    int nm;  // neighbour entries whose count == bc  (= bc * |best|)
};

// Candidate key of the sorted scorers: lexicographic (count, remaining CPU,
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

// (remaining CPU, -node) as one u64, 0 = none (node < 2^25)
__device__ __forceinline__ unsigned long long pack_rn(int rem, int n) {
    return ((unsigned long long)((unsigned)rem ^ 0x80000000u) << kNodeBits) | (unsigned long long)(kNodeMask - (unsigned)n);
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
// in-flight load.  Callers guarantee index * sizeof(T) < 2^32.
__device__ __forceinline__ int ld32(const int *__restrict__ base, unsigned idx) {
    return *reinterpret_cast<const int *>(reinterpret_cast<const char *>(base) + (idx << 2));
}
__device__ __forceinline__ unsigned ld16(const unsigned short *__restrict__ base, unsigned idx) {
    return *reinterpret_cast<const unsigned short *>(reinterpret_cast<const char *>(base) + (idx << 1));
}

// Plan data read through the constant address space: it never changes during a
// launch, so wave-uniform reads become scalar loads (lgkmcnt) instead of vector
// loads queued behind in-flight gathers.
typedef const __attribute__((address_space(4))) int *cint_ptr;
__device__ __forceinline__ cint_ptr const_ptr(const int *p) { return (cint_ptr)(uintptr_t)p; }

template <int D, class T>
__device__ __forceinline__ void bitonic_sort(T (&v)[D]) {
#pragma unroll
    for (int k = 2; k <= D; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (int i = 0; i < D; ++i) {
                const int l = i ^ j;
                if (l > i) {
                    const T lo = min(v[i], v[l]), hi = max(v[i], v[l]);
                    if ((i & k) == 0) { v[i] = lo; v[l] = hi; }
                    else { v[i] = hi; v[l] = lo; }
                }
            }
            // one network stage at a time: the scheduler would otherwise
            // interleave stages and hold both halves of every exchange
            if (D >= 32) __builtin_amdgcn_sched_barrier(0);
        }
}

// Batcher's odd-even merge sort, ascending: the same register-only
// compare-exchanges as bitonic_sort but fewer of them (D = 32: 191 instead of
// 240; D = 64: 543 instead of 672).
template <int D, class T>
__device__ __forceinline__ void oem_sort(T (&v)[D]) {
#pragma unroll
    for (int p = 1; p < D; p += p)
#pragma unroll
        for (int k = p; k >= 1; k >>= 1) {
#pragma unroll
            for (int j = k % p; j + k < D; j += 2 * k)
#pragma unroll
                for (int i = 0; i < k; ++i)
                    if (i + j + k < D && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
                        const T lo = min(v[i + j], v[i + j + k]), hi = max(v[i + j], v[i + j + k]);
                        v[i + j] = lo;
                        v[i + j + k] = hi;
                    }
            if (D >= 32) __builtin_amdgcn_sched_barrier(0);
        }
}

#ifndef RSK_OEM_SORT
#define RSK_OEM_SORT 1
#endif
template <int D, class T>
__device__ __forceinline__ void sort_cells(T (&v)[D]) {
    if (RSK_OEM_SORT) oem_sort<D, T>(v);
    else bitonic_sort<D, T>(v);
}

// Next work unit of the wave: lane 0 bumps the workgroup's LDS counter.
__device__ __forceinline__ int grab(int *ctr, int lane) {
    int k = 0;
    if (lane == 0) k = atomicAdd(ctr, 1);
    return __builtin_amdgcn_readfirstlane(k);
}

// ---------------------------------------------------------------------------
// Compact path (rsk_car16.hip), N <= 65535.
//
// Node state per (node, scenario) as a 16-bit code, monotone in the remaining
// CPU rem = cap - use:
//   0                hazard (never a candidate)
//   1                rem < 0 (any negative value: a tie whose best rem is < 0 is
//                    None whichever node wins it, rescheduling.py:203-212)
//   2 .. 8193        rem in [0, 8192) exactly, while rem < B
//   8194 .. 32768    rem in [8192, B): 12 mantissa bits per power of two (inexact)
//   32769 .. 65534   rem in [B, B + 32766) exactly
//   65535            rem beyond that (inexact)
// with B = max(0, max(cap) - 32766): every rem within 32766 millicores of the
// largest capacity has its own code, so ties on the top nodes are decided by
// the code word alone.  A code comparison decides every tie except between
// distinct nodes with the same inexact code; those few are resolved exactly
// from cap / use.
// A cell: (code << 16) | node; kCellPad = code 0 (no candidate), node 0xffff
// (never a node: N <= 65535) for padding and assignments outside [0, N).
constexpr unsigned kCellPad = 0x0000ffffu;
__device__ __forceinline__ unsigned cell_code(unsigned c) { return c >> 16; }
__device__ __forceinline__ int cell_node(unsigned c) { return (int)(c & 0xffffu); }
// candidate word: larger code first, then the lower node (the reference's
// `rem > r` keeps the first node in nodes_name order on equal rem)
__device__ __forceinline__ unsigned cell_cand(unsigned c) { return c ^ 0xffffu; }
__device__ __forceinline__ int cand_node(unsigned w) { return (int)((w & 0xffffu) ^ 0xffffu); }
// equal codes >= 2 that do NOT imply equal remaining CPU (exact resolution needed)
__device__ __forceinline__ bool code_inexact(unsigned c) { return (c >= 8194u && c <= 32768u) || c == 65535u; }

constexpr unsigned kCodeHaz = 0u;
constexpr unsigned kCodeNeg = 1u;

// The code of remaining CPU rem (hazard: 0) with the exact window at B (above).
__device__ __forceinline__ unsigned code16(int rem, bool haz, int B) {
    if (haz) return kCodeHaz;
    if (rem < 0) return kCodeNeg;
    if (rem >= B) return 32769u + (unsigned)min(rem - B, 32766);
    const unsigned x = (unsigned)rem;
    if (x < 8192u) return 2u + x;
    const int e = 31 - __clz((int)x);  // 13..30
    if (e > 18) return 32768u;          // one bucket from 2^19 to B (exact ties resolve it)
    return 2u + 8192u + (unsigned)(e - 13) * 4096u + ((x >> (e - 12)) & 0xfffu);
}

constexpr int kMaxNodes16 = 65535;  // node ids fit 16 bits, 0xffff stays free as the pad node

struct Prep16Args {
    const int *cap, *use;
    const uint8_t *haz;
    int N, S;
    unsigned short *code;        // [N*S] or null
    int *nodekey;                // [N*S] (hazard ? KEY_HAZ : cap - use) or null
    int *zc_cnt;                 // [S] (zero on entry: the previous execute's prep cleared this half)
    unsigned long long *zc_key;  // [S]
    unsigned *zc_clear;          // the other half of the double-buffered zero-case words, cleared
    int clear_words;             // by the prep kernel for the next execute
};

// max(cap[0..N)) by the whole workgroup of kT threads, returned to every
// thread (every workgroup reads the same caps: the same exact code window B
// everywhere, without a launch of its own).  red: kT / 64 ints of LDS.
template <int kT>
__device__ __forceinline__ int block_capmax(const int *__restrict__ cap, int N, int *red) {
    const int t = (int)threadIdx.x;
    int mc = 0;
    const int N4 = ((uintptr_t)cap % 16) == 0 ? N / 4 : 0;
    const int4 *cap4 = reinterpret_cast<const int4 *>(cap);
    constexpr int kU = 8;  // 16-B loads in flight per thread (clamped: a repeated word does not change a max)
    for (int i0 = t; i0 < N4; i0 += kT * kU) {
        int4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) v[u] = cap4[min(i0 + u * kT, N4 - 1)];
#pragma unroll
        for (int u = 0; u < kU; ++u) mc = max(mc, max(max(v[u].x, v[u].y), max(v[u].z, v[u].w)));
    }
    for (int n = 4 * N4 + t; n < N; n += kT) mc = max(mc, cap[n]);
    mc = dpp_max(mc);
    if ((t & 63) == 0) red[t >> 6] = mc;
    __syncthreads();
    mc = red[0];
#pragma unroll
    for (int w = 1; w < kT / 64; ++w) mc = max(mc, red[w]);
    __syncthreads();  // red free again
    return mc;
}

// chunks per group in the tile grid order (each group walked tile-major inside
// its XCD's run): round 5's interleaved A/B at config 3 gave 0.8167 / 0.8170 ms
// for 4, 0.8196 / 0.8188 for 2, 0.8198 / 0.8196 for 1, with the same reads
// (2.14-2.17 GB): the group does not move the code lines' L2 misses)
constexpr int kTileGroup = 4;

struct Tile16Args {
    const int *img_pods;   // concatenated per-tile image pod lists
    const int *meta;       // [T][kMetaW]
    const int *recs;       // concatenated per-tile record blobs (16-B aligned)
    const int *assign;
    const unsigned short *code;
    const int *cap, *use;  // exact tie resolution between equal codes
    const int *zc_cnt;
    const unsigned long long *zc_key;
    int *out_target;
    int *out_score;
    int S, N, T, lsl;      // SL = 1 << lsl scenarios per workgroup (64 when S >= 64); T tiles from tile0
    int tile0;
    int img_cells;         // LDS cells of the largest image (rmax * SL); the records follow
    int rec_cap;           // record ints reserved in LDS; the unit counter follows
    int xcd_per;           // tile units per XCD (the XCD-contiguous grid order)
    int ablate;            // profiling only (RSK_ABLATE_TILE): 1 skip image load, 2 skip scoring, 4 stores only,
                           // 8 code gathers from one line
    unsigned n_assign, n_out, n_pods, n_recs, n_key;  // element counts (debug bounds build)
};

// Side rows of the compact path (rsk_side16.hip): every row above the tiles,
// in launches by degree class; a work item is (row, chunk of 64 scenarios).
struct SideArgs {
    const int *items;         // [n_rows][4]: out row, offset into col, degree, 0 (degree descending)
    int n_rows, nchunk;       // work items = n_rows * nchunk, chunk-major
    const int *col;           // neighbour lists
    const int *assign;
    const unsigned short *code;
    const int *cap, *use;
    const int *zc_cnt;
    const unsigned long long *zc_key;
    int *out_target, *out_score;
    int S, N;
    int H, hshift, K;         // per-team LDS geometry (side16_geometry), word offsets below
    int off_dl, off_ndl, off_dummy, off_fx, off_h2, h2cap;
    unsigned lds_team;
    int xcd_per;              // workgroups per XCD run (set by launch_side16)
    int ablate;               // profiling only (results wrong): 1 no exact recounts, 2 pass 1 only, 4 no (1), 8 no (2)
    unsigned *gscratch;       // teams whose table exceeds the LDS: lds_team bytes per block in global memory
    // on-the-fly node state (kOTF launches, code == null): codes from cap / use /
    // haz with B from the workgroup's own max(cap), the zero case scanned per
    // scenario when needed, so the launch depends on no prep kernel and runs
    // beside car_prep
    const uint8_t *haz;
};
struct SideGeom {
    int dmax, Dc, H, hshift, K, T, W, kB;
    int off_dl, off_ndl, off_dummy, off_fx, off_h2, h2cap;
    size_t lds_team;
};
SideGeom side16_geometry(int dmax, int N, int T = 0);  // T: waves per item (0: 1 up to 256 neighbours, else 8)
void side16_apply_geometry(SideArgs &a, const SideGeom &g);  // the geometry's LDS layout into the launch arguments
// Rows above the side classes, scored in the fused grid one (row, scenario)
// cell per workgroup (targets only): the cell's neighbour nodes counted in an
// LDS hash of packed words ((node + 1) << 16 | count), H words + 4 reduction
// words within the tile's LDS, exact cap - use of the nodes at the max count.
struct DirectArgs {
    const int *rp, *ci;       // the plan's deduplicated rows without self edges
    const int *rows;          // plan row -> pod (null: the identity)
    const int *items;         // item k's plan row at items[k * istride]
    int istride, Q;           // Q rows: cells = Q * S
    const int *assign, *use, *cap;
    const uint8_t *haz;
    int S, N, H;
    int *out_target;
};
// H for a packed table of rows up to dmax neighbours within lds bytes (0: none fits)
int direct16_table(int dmax, int N, size_t lds);
struct FuseMap {
    int direct_blocks; // the first direct_blocks blocks: one (row, scenario) cell each (da), a multiple of 8
    int big_blocks;    // then big_blocks blocks: 4-wave side teams (ba), a multiple of 8
    int R, k1;         // then k1 periods of R rows of 8 blocks: R - 1 tile rows, one single-wave side row (sa)
    int side_rows, tile_rows;  // then the tile rows left, then the side rows left
};
// lean tiles + single-wave side items of one class (4 per workgroup, kB 16) +
// optionally 4-wave side teams (kB 16) in one grid; ba.n_rows == 0: no teams
int launch_fused16(hipStream_t stream, const Tile16Args &a, const SideArgs &sa, int side_blocks, const SideArgs &ba,
                   const DirectArgs &da, bool score, bool off32, unsigned tile_blocks, size_t lds);
// scratch: device memory for rows whose table exceeds the LDS (grown on demand)
int launch_side16(hipStream_t stream, const SideArgs &a, const SideGeom &g, bool off32, DevBuf *scratch);
// the same rows with node state computed on the fly (a.code null, a.haz / a.capmax set)
int launch_side16_otf(hipStream_t stream, const SideArgs &a, const SideGeom &g, bool off32, DevBuf *scratch);

int launch_prep(hipStream_t stream, const Prep16Args &a);
int launch_tile16(hipStream_t stream, const Tile16Args &a, bool score, bool off32, unsigned blocks, size_t lds);
size_t tile16_lds_bytes(int rmax, int lsl, int rec_cap);
unsigned tile16_debug_take();
int tile16_rows_built();       // image rows per tile the compact kernels are compiled for (RSK_TILE16_ROWS)

}  // namespace rsk
