// rsk_metrics.hip — spread / binpack / random placement and the per-node
// reductions ("kernel 3") of the placement path, on gfx950.
//
// All per-scenario arrays are scenario-minor (x[n*S + s]).  Most kernels map
// thread t -> (scenario s = t % S, node or pod chunk t / S), so one wave reads 64
// consecutive scenarios of the same node / pod: a coalesced row.  Per-scenario
// winners are combined with 64-bit integer atomicMax / atomicMin on packed
// keys (order-independent, hence deterministic); floating-point sums use
// fixed-order partials, never atomics.
#include <climits>
#include <cmath>
#include <cstring>
#include <vector>

#include "rsk_car.h"  // rsk_common.h + const_ptr (scalar loads)

namespace rsk {

// chunk size so the grid has ~512K threads
static int chunk_for(int64_t items, int S) {
    const int64_t target = 256 * 2048;
    return (int)std::max<int64_t>(1, ceil_div(items * S, target));
}

__device__ __forceinline__ unsigned long long pack_hi_lo(int hi, unsigned lo) {
    return ((unsigned long long)((unsigned)hi ^ 0x80000000u) << 32) | (unsigned long long)lo;
}

// ---------------------------------------------------------------------------
// One CAR placement in one workgroup (rsk_car_row; rescheduling.py:183-214):
// the node histogram of the related pods in LDS, then two block maxima — the
// best score M over non-hazard nodes, then (cap - use, -node) over the nodes
// at M and how many they are.  M = 0 (no related pod on a candidate) is the
// same rule: every non-hazard node ties at 0.
constexpr int kRowThreads = 1024;
constexpr int kRowMaxN = 32768;
__device__ __forceinline__ void row_block_max_u64(unsigned long long &v, unsigned long long *red) {
    // wave maxima by DPP, then across the 16 waves through LDS
    unsigned long long w;
    w = (unsigned long long)__shfl_xor((long long)v, 32); v = w > v ? w : v;
    w = (unsigned long long)__shfl_xor((long long)v, 16); v = w > v ? w : v;
    w = (unsigned long long)__shfl_xor((long long)v, 8); v = w > v ? w : v;
    w = (unsigned long long)__shfl_xor((long long)v, 4); v = w > v ? w : v;
    w = (unsigned long long)__shfl_xor((long long)v, 2); v = w > v ? w : v;
    w = (unsigned long long)__shfl_xor((long long)v, 1); v = w > v ? w : v;
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    v = 0ull;
    for (int i = 0; i < kRowThreads / 64; ++i) v = red[i] > v ? red[i] : v;
    __syncthreads();
}

__global__ __launch_bounds__(kRowThreads) void car_row_kernel(const int *__restrict__ node_of, int k,
                                                              const int *__restrict__ cap, const int *__restrict__ use,
                                                              const uint8_t *__restrict__ haz, int N,
                                                              int *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned rl[];
    unsigned *cnt = rl;  // [N]
    unsigned long long *red = reinterpret_cast<unsigned long long *>(rl + ((N + 3) & ~3));
    __shared__ int nm;
    for (int n = threadIdx.x; n < N; n += kRowThreads) cnt[n] = 0u;
    if (threadIdx.x == 0) nm = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < k; i += kRowThreads) {
        const int n = node_of[i];
        if ((unsigned)n < (unsigned)N && !haz[n]) atomicAdd(&cnt[n], 1u);
    }
    __syncthreads();
    // M: the best score over candidates, +1 so that "no candidate" is 0
    unsigned long long m = 0ull;
    for (int n = threadIdx.x; n < N; n += kRowThreads)
        if (!haz[n]) m = max(m, (unsigned long long)cnt[n] + 1ull);
    row_block_max_u64(m, red);
    if (m == 0ull) {  // every node is hazard: max() of an empty sequence
        if (threadIdx.x == 0) { out[0] = RSK_TARGET_NO_CANDIDATE; out[1] = -1; }
        return;
    }
    const unsigned M = (unsigned)(m - 1ull);
    unsigned long long b = 0ull;
    int c = 0;
    for (int n = threadIdx.x; n < N; n += kRowThreads)
        if (!haz[n] && cnt[n] == M) {
            ++c;
            const unsigned long long key = pack_hi_lo(cap[n] - use[n], ~(unsigned)n);
            b = key > b ? key : b;
        }
    if (c) atomicAdd(&nm, c);
    row_block_max_u64(b, red);
    if (threadIdx.x == 0) {
        const int rem = (int)((unsigned)(b >> 32) ^ 0x80000000u);
        const int node = (int)(~(unsigned)(b & 0xffffffffull));
        out[0] = nm == 1 ? node : (rem >= 0 ? node : RSK_TARGET_NONE);
        out[1] = (int)M;
    }
}

// ---------------------------------------------------------------------------
// spread (rescheduling.py:89-101): min (pod_count, name_rank) over non-hazard.
// binpack (rescheduling.py:121-133): max (cpu_pct, name_rank).
// key = (primary ^ sign) << 32 | rank; the winning rank maps back to its node.
// ---------------------------------------------------------------------------
template <bool kMin>
__global__ __launch_bounds__(256) void pick_node_kernel(const int *__restrict__ val, const int *__restrict__ rank,
                                                        const uint8_t *__restrict__ haz, int N, int S, int npb,
                                                        unsigned total, unsigned long long *__restrict__ best) {
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (t >= total) return;
    const int s = (int)(t % (unsigned)S);
    const int n0 = (int)(t / (unsigned)S) * npb, n1 = min(N, n0 + npb);
    unsigned long long b = kMin ? ~0ull : 0ull;
    bool any = false;
    for (int n = n0; n < n1; ++n) {
        const size_t idx = (size_t)n * S + s;
        if (haz[idx]) continue;
        const unsigned long long k = pack_hi_lo(val[idx], (unsigned)rank[n]);
        b = kMin ? (k < b ? k : b) : (k > b ? k : b);
        any = true;
    }
    if (any) {
        if (kMin) atomicMin(&best[s], b);
        else atomicMax(&best[s], b + 1ull);  // +1: 0 stays "no candidate"
    }
}

__global__ void rank_inverse_kernel(const int *__restrict__ rank, int N, int *__restrict__ inv) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n < N) {
        const int r = rank[n];
        if ((unsigned)r < (unsigned)N) inv[r] = n;
    }
}

template <bool kMin>
__global__ void pick_node_finish(const unsigned long long *__restrict__ best, const int *__restrict__ inv, int N,
                                 int S, int *__restrict__ out) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= S) return;
    unsigned long long b = best[s];
    if (kMin ? b == ~0ull : b == 0ull) { out[s] = RSK_TARGET_NO_CANDIDATE; return; }
    if (!kMin) b -= 1ull;
    const unsigned r = (unsigned)(b & 0xffffffffull);
    out[s] = r < (unsigned)N ? inv[r] : RSK_TARGET_NO_CANDIDATE;
}

// S = 1 from host arrays (the drop-in's single call): one workgroup, one
// staging copy, one launch.  Key (val, rank) per non-hazard node, min for
// spread (as the max of its complement), max for binpack; then the node whose
// name rank won writes itself.
template <bool kMin>
__global__ __launch_bounds__(kRowThreads) void pick_node_row_kernel(const int *__restrict__ val,
                                                                    const int *__restrict__ rank,
                                                                    const uint8_t *__restrict__ haz, int N,
                                                                    int *__restrict__ out) {
    __shared__ unsigned long long red[kRowThreads / 64];
    unsigned long long b = 0ull;
    for (int n = threadIdx.x; n < N; n += kRowThreads)
        if (!haz[n]) {
            // rank < N < 2^31 leaves bit 31 free: set in every candidate's key (the
            // complement sets it for spread), so 0 means "no candidate" even for
            // binpack's (INT32_MIN, rank 0)
            const unsigned long long k = pack_hi_lo(val[n], (unsigned)rank[n]);
            const unsigned long long kk = kMin ? ~k : (k | 0x80000000ull);
            b = kk > b ? kk : b;
        }
    row_block_max_u64(b, red);
    if (b == 0ull) {
        if (threadIdx.x == 0) out[0] = RSK_TARGET_NO_CANDIDATE;
        return;
    }
    const unsigned r = (unsigned)((kMin ? ~b : b) & 0x7fffffffull);
    for (int n = threadIdx.x; n < N; n += kRowThreads)
        if (!haz[n] && (unsigned)rank[n] == r) out[0] = n;
}

// Host inputs of a single-call (S = 1) kernel: packed at 16-B offsets into the
// context's mapped pinned buffer, followed by the result words.  Up to
// kZeroCopyMax bytes the kernel reads the inputs there over PCIe (no copy);
// above, one DMA copy to device staging.  The kernel writes its result words
// straight into the pinned buffer, host-visible once the stream has synced.
constexpr size_t kZeroCopyMax = 64 * 1024;
struct RowIO {
    const char *in;       // device view of the packed inputs
    char *out_dev;        // device view of the result words
    const char *out_host;
    size_t off[4];        // input offsets
};
static int row_io(rsk_ctx *ctx, const void *const *src, const size_t *len, int n, size_t out_bytes, RowIO *io) {
    size_t tot = 0;
    for (int i = 0; i < n; ++i) {
        io->off[i] = tot;
        tot += (len[i] + 15) & ~(size_t)15;
    }
    RSK_TRY(ctx->pin.reserve(tot + out_bytes));
    char *h = static_cast<char *>(ctx->pin.host);
    for (int i = 0; i < n; ++i)
        if (len[i]) std::memcpy(h + io->off[i], src[i], len[i]);
    if (tot <= kZeroCopyMax) {
        io->in = static_cast<const char *>(ctx->pin.dev);
    } else {
        RSK_TRY(ctx->host_stage[7].reserve(tot));
        RSK_HIP(hipMemcpyAsync(ctx->host_stage[7].ptr, h, tot, hipMemcpyHostToDevice, ctx->stream));
        io->in = static_cast<const char *>(ctx->host_stage[7].ptr);
    }
    io->out_dev = static_cast<char *>(ctx->pin.dev) + tot;
    io->out_host = h + tot;
    return RSK_OK;
}

// The candidate list of one scenario (rescheduling.py:149-150): non-hazard
// node indices in order, compacted by one workgroup chunk by chunk.
__global__ __launch_bounds__(kRowThreads) void candidates_row_kernel(const uint8_t *__restrict__ haz, int N,
                                                                     int *__restrict__ out_nodes,
                                                                     int *__restrict__ out_count) {
    __shared__ int wsum[kRowThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int base = 0;
    for (int n0 = 0; n0 < N; n0 += kRowThreads) {
        const int n = n0 + tid;
        const bool c = n < N && !haz[n];
        const unsigned long long m = __builtin_amdgcn_ballot_w64(c);
        if (lane == 0) wsum[w] = __builtin_popcountll(m);
        __syncthreads();
        int before = 0, total = 0;
#pragma unroll
        for (int i = 0; i < kRowThreads / 64; ++i) {
            before += i < w ? wsum[i] : 0;
            total += wsum[i];
        }
        if (c) out_nodes[base + before + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] = n;
        base += total;
        __syncthreads();
    }
    if (tid == 0) *out_count = base;
}

template <bool kMin>
static int pick_node_row(rsk_ctx *ctx, const int32_t *val, const int32_t *name_rank, const uint8_t *hazard, int32_t N,
                         int32_t *out_node, const char *tag) {
    const void *src[3] = {val, name_rank, hazard};
    const size_t len[3] = {(size_t)N * 4, (size_t)N * 4, (size_t)N};
    RowIO io;
    RSK_TRY(row_io(ctx, src, len, 3, 16, &io));
    {
        ScopedTimer tm(ctx, tag);
        pick_node_row_kernel<kMin><<<1, kRowThreads, 0, ctx->stream>>>(
            reinterpret_cast<const int *>(io.in + io.off[0]), reinterpret_cast<const int *>(io.in + io.off[1]),
            reinterpret_cast<const uint8_t *>(io.in + io.off[2]), N, reinterpret_cast<int *>(io.out_dev));
        RSK_HIP(hipGetLastError());
    }
    RSK_HIP(hipStreamSynchronize(ctx->stream));
    const int r = *reinterpret_cast<const volatile int *>(io.out_host);
    *out_node = r;
    return r == RSK_TARGET_NO_CANDIDATE ? RSK_NO_CANDIDATE : RSK_OK;
}

template <bool kMin>
static int pick_node(rsk_ctx *ctx, const int32_t *val, const int32_t *name_rank, const uint8_t *hazard, int32_t N,
                     int32_t S, int32_t *out_node, uint32_t flags, const char *tag) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(N > 0 && S > 0 && (int64_t)N * S < INT32_MAX, "bad sizes N=%d S=%d", N, S);
    RSK_CHECK(out_node, "null out_node");
    const bool dev = flags & RSK_F_DEVICE;
    if (S == 1 && !dev && val && name_rank && hazard)
        return pick_node_row<kMin>(ctx, val, name_rank, hazard, N, out_node, tag);
    const size_t NS = (size_t)N * S;
    const int *d_val, *d_rank;
    const uint8_t *d_haz;
    int *d_out;
    RSK_TRY(stage_in(ctx, 0, val, NS * 4, dev, reinterpret_cast<const void **>(&d_val)));
    RSK_TRY(stage_in(ctx, 1, name_rank, (size_t)N * 4, dev, reinterpret_cast<const void **>(&d_rank)));
    RSK_TRY(stage_in(ctx, 2, hazard, NS, dev, reinterpret_cast<const void **>(&d_haz)));
    RSK_TRY(stage_out(ctx, 3, out_node, (size_t)S * 4, dev, reinterpret_cast<void **>(&d_out)));
    RSK_TRY(ctx->work[0].reserve((size_t)S * 8));
    RSK_TRY(ctx->work[1].reserve((size_t)N * 4));
    auto *best = ctx->work[0].as<unsigned long long>();
    int *inv = ctx->work[1].as<int>();
    RSK_HIP(hipMemsetAsync(best, kMin ? 0xff : 0x00, (size_t)S * 8, ctx->stream));
    RSK_HIP(hipMemsetAsync(inv, 0xff, (size_t)N * 4, ctx->stream));
    const int npb = chunk_for(N, S);
    const unsigned total = (unsigned)(ceil_div(N, npb) * S);
    {
        ScopedTimer tm(ctx, tag);
        pick_node_kernel<kMin><<<(unsigned)ceil_div(total, 256), 256, 0, ctx->stream>>>(d_val, d_rank, d_haz, N, S,
                                                                                         npb, total, best);
        rank_inverse_kernel<<<(unsigned)ceil_div(N, 256), 256, 0, ctx->stream>>>(d_rank, N, inv);
        pick_node_finish<kMin><<<(unsigned)ceil_div(S, 256), 256, 0, ctx->stream>>>(best, inv, N, S, d_out);
        RSK_HIP(hipGetLastError());
    }
    if (!dev) {
        RSK_TRY(copy_back(ctx, out_node, d_out, (size_t)S * 4, false));
        RSK_HIP(hipStreamSynchronize(ctx->stream));
        for (int s = 0; s < S; ++s)
            if (out_node[s] == RSK_TARGET_NO_CANDIDATE) return RSK_NO_CANDIDATE;
    }
    return RSK_OK;
}

// ---------------------------------------------------------------------------
// random (rescheduling.py:149-153): count candidates, then the r-th one.
// count: per (node chunk, s) partial counts -> part[chunk][s] (+ atomic total).
// select: per scenario, walk the chunk partials to the chunk holding r, then
// the nodes of that chunk.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void count_free_kernel(const uint8_t *__restrict__ haz, int N, int S, int npb,
                                                         unsigned total, int *__restrict__ part,
                                                         int *__restrict__ count) {
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (t >= total) return;
    const int s = (int)(t % (unsigned)S), ch = (int)(t / (unsigned)S);
    const int n0 = ch * npb, n1 = min(N, n0 + npb);
    int c = 0;
    for (int n = n0; n < n1; ++n) c += !haz[(size_t)n * S + s];
    part[(size_t)ch * S + s] = c;
    if (c) atomicAdd(&count[s], c);
}

__global__ __launch_bounds__(256) void select_free_kernel(const uint8_t *__restrict__ haz, int N, int S, int npb,
                                                          int nchunks, const int *__restrict__ part,
                                                          const int *__restrict__ r, int *__restrict__ out) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= S) return;
    int want = r[s];
    if (want < 0) { out[s] = RSK_TARGET_NO_CANDIDATE; return; }
    int ch = 0;
    for (; ch < nchunks; ++ch) {
        const int c = part[(size_t)ch * S + s];
        if (want < c) break;
        want -= c;
    }
    if (ch == nchunks) { out[s] = RSK_TARGET_NO_CANDIDATE; return; }
    const int n0 = ch * npb, n1 = min(N, n0 + npb);
    int t = RSK_TARGET_NO_CANDIDATE;
    for (int n = n0; n < n1; ++n)
        if (!haz[(size_t)n * S + s]) {
            if (want == 0) { t = n; break; }
            --want;
        }
    out[s] = t;
}

// CPython random.Random: MT19937 with init_by_array seeding (see rsk_py_randbelow).
struct MT {
    uint32_t mt[624];
    int idx;
    void init_genrand(uint32_t s) {
        mt[0] = s;
        for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        idx = 624;
    }
    void init_by_array(const uint32_t *key, int len) {
        init_genrand(19650218u);
        int i = 1, j = 0;
        for (int k = (624 > len ? 624 : len); k; --k) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
            ++i;
            ++j;
            if (i >= 624) { mt[0] = mt[623]; i = 1; }
            if (j >= len) j = 0;
        }
        for (int k = 623; k; --k) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
            ++i;
            if (i >= 624) { mt[0] = mt[623]; i = 1; }
        }
        mt[0] = 0x80000000u;
        idx = 624;
    }
    uint32_t next() {
        if (idx >= 624) {
            for (int k = 0; k < 624; ++k) {
                const uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
                mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            idx = 0;
        }
        uint32_t y = mt[idx++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
};

// ---------------------------------------------------------------------------
// Kernel 3: node reductions and metrics.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void node_reduce_kernel(const int *__restrict__ assign, int P, int S,
                                                          const int *__restrict__ pod_cpu,
                                                          const long long *__restrict__ pod_mem, int N,
                                                          int *__restrict__ cnt, unsigned long long *__restrict__ cpu,
                                                          unsigned long long *__restrict__ mem) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (size_t)P * S) return;
    const int a = assign[t];
    if ((unsigned)a >= (unsigned)N) return;
    const int p = (int)(t / (size_t)S), s = (int)(t - (size_t)p * S);
    const size_t o = (size_t)a * S + s;
    atomicAdd(&cnt[o], 1);
    atomicAdd(&cpu[o], (unsigned long long)(long long)pod_cpu[p]);
    if (mem) atomicAdd(&mem[o], (unsigned long long)pod_mem[p]);
}

// The deviation form (S >= 32).  What-if scenarios perturb a common base, so a
// pod sits on one node in most scenarios: its key node k(p), the majority of
// its nodes in scenarios 0, 21 and 42 (scenario 0's when S < 43), or N when
// that is not a node.  The integer sums split exactly into
//   out[n, s] = base[n] + dev[n, s]
//   base[n]   = the sum over the pods with k(p) = n of (1, cpu, mem), every s
//   dev[n, s] = the sum over the cells a(p, s) = n != k(p) of (1, cpu, mem)
//             - the sum over the cells k(p) = n != a(p, s) of (1, cpu, mem)
// so only the deviation cells (~2 % of the bench batches' cells) carry a
// per-scenario term.  Five launches, no zeroing pass and (unless a block's
// deviations overflow) no global atomics:
//  1 nr_scan: every assign row read once, coalesced (lane = scenario, the next
//    16 rows in flight while a batch is examined): the keys (pkey), and per
//    block of kNrPods pods the count of its keys per 32-node bucket and of its
//    deviation records per (64-scenario chunk, bucket) bin (a + at the cell's
//    node, a - at the key node), one entry per deviation cell (int2: node or
//    kNrNoNode | (p - p0) << 20, s) into its wave's share of the block's
//    region of ecap = cells / 8 entries;
//  2 nr_colscan: per counter (bucket or bin) the exclusive scan of its
//    per-block counts, laid out [counter][block], and its total;
//  3 nr_place: the counters' bases (a scan of the totals in the workgroup);
//    the block's pods to their key bucket's slice as (node & 31, cpu, mem)
//    records, each entry's + and - to their bins' slices as (node & 31 |
//    minus << 5 | (s & 63) << 6, cpu, mem) records (key / cpu / mem from LDS);
//  4 nr_sum: a workgroup per bin sums the bucket's pod records (base, 32
//    nodes) and the bin's entries (dev, 32 nodes x 64 scenarios) in LDS and
//    stores out = base + dev, 64 scenarios per coalesced store;
//  5 nr_spill: a block whose entries overflowed its region listed none; its
//    deviation cells are added here, after the stores, by global atomics.
// podmonitor.py:104-121 (pods grouped by node), nodemonitor.py:24-46 (per-node
// sums).  Integer sums: the result does not depend on any order.
#ifndef RSK_NR_PODS
#define RSK_NR_PODS 4096
#endif
#ifndef RSK_NR_THREADS
#define RSK_NR_THREADS 1024
#endif
#ifndef RSK_NR_ABL
#define RSK_NR_ABL 0  // profiling variants only (results wrong): 1 no row examination (keys and pkey kept;
#endif                // the rows folded into one word)
constexpr int kNrPods = RSK_NR_PODS;       // pods per block of the scan / place / spill launches
constexpr int kNrThreads = RSK_NR_THREADS;  // their threads: 16 waves of 256 pods (r06j: 4096 / 1024
                                            // 3.5% under 2048 / 512 at 1M x 64: half the colscan blocks)
constexpr int kNrBatch = 16;      // assign rows per batch (two batches in flight per wave)
constexpr int kNrBucketBits = 5, kNrBucketNodes = 1 << kNrBucketBits;  // nodes per bucket
constexpr int kNrMaxCounters = 16384;  // buckets + bins: a block's counters in LDS (N < 2^19)
constexpr int kNrEntDiv = 8;           // a block's entry region: its cells / 8 entries
constexpr int kNrMaxS = 65536;         // (a block's entry count stays below 2^32)
constexpr int kNrNoNode = 0x7ffff;     // an entry's node field when the cell is not on a node

__device__ __forceinline__ int nr_rank(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// byte offset of assign[i * S + s] (32-bit arithmetic when P * S * 4 < 2^32:
// the saddr form of the load)
template <bool kOff32>
__device__ __forceinline__ size_t nr_off(unsigned i, unsigned S, unsigned s) {
    if (kOff32) return (size_t)((i * S + s) << 2);
    return ((size_t)i * S + s) << 2;
}

// The scan / place / spill launches map workgroup i to block (i & 7) * per +
// (i >> 3), per = ceil(nblk / 8): an XCD runs a run of consecutive blocks, so
// the neighbouring slices they write (counters, records) meet in its L2.
__device__ __forceinline__ int nr_block(int nblk) {
    const int per = (nblk + 7) >> 3;
    return (int)(blockIdx.x & 7u) * per + (int)(blockIdx.x >> 3);
}

// launch 1: a wave walks its pods' (batch of 16, chunk) units, the next unit's
// 16 rows (wave-uniform row pointers) loaded while one is examined; the 16
// pods' keys are readlanes of their chunk-0 rows (scenarios 0 / 21 / 42, the
// majority in scalar registers).  (Round 5 gathered those words with a second
// load per unit: 14 us of the launch's 72, r06q.)  A row's test is one compare
// into a wave mask (SGPRs); only rows with a deviating lane (~half of the
// bench's) write entries, into the wave's own share of the block's region.
// (Round 5's per-lane bit mask folded by a wave OR, then a ballot per flagged
// row, issued ~28 VALU instructions per row: the scan was issue-bound.)
// Counters -> bh[j * nblk + b] (the entry bins zeroed when a wave
// overflowed), the waves' entry counts (-1: the block overflowed) ->
// ecount[b * waves + w].
template <bool kOff32, bool kMaj, int kB = kNrBatch>
__global__ __launch_bounds__(kNrThreads) void nr_scan_kernel(const int *__restrict__ assign, int P, int S, int N,
                                                             int nbk, int nchunk, int nblk, size_t ecap,
                                                             int *__restrict__ pkey, int *__restrict__ bh,
                                                             int2 *__restrict__ ent, int *__restrict__ ecount) {
    extern __shared__ int lh[];  // [nbk] key buckets, then [nchunk][nbk] entry bins
    __shared__ int over;
    const int b = nr_block(nblk);
    if (b >= nblk) return;
    const int t = (int)threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);  // (uniform)
    const int nh = nbk * (1 + nchunk);
    for (int j = t; j < nh; j += kNrThreads) lh[j] = 0;
    if (t == 0) over = 0;
    __syncthreads();
    int abl_acc = 0;
    constexpr int kPW = kNrPods / (kNrThreads / 64), kW = kNrThreads / 64;
    const int p0 = b * kNrPods, q0 = p0 + wv * kPW, q1 = min(P, q0 + kPW);
    const int nv = q1 > q0 ? (q1 - q0 + kB - 1) / kB * nchunk : 0;  // the wave's units
    const char *__restrict__ asg = reinterpret_cast<const char *>(assign);
    const unsigned wcap = (unsigned)(ecap / kW);  // (< 2^24: kNrPods * kNrMaxS / kNrEntDiv / 8)
    int2 *__restrict__ E = ent + (size_t)b * ecap + (size_t)wv * wcap;
    unsigned wpos = 0u;
    bool wover = false;
    auto split = [&](int v, int &bt, int &c) {  // unit v -> (batch, chunk); nchunk = 1 when S <= 64
        if (nchunk == 1) {
            bt = v;
            c = 0;
        } else {
            bt = v / nchunk;
            c = v - bt * nchunk;
        }
    };
    auto load = [&](int v, int (&r)[kB]) {  // clamped: always valid addresses
        v = min(v, nv - 1);
        int bt, c;
        split(v, bt, c);
        const int pb = q0 + bt * kB, last = min(q1, pb + kB) - 1;
        const unsigned sc = (unsigned)min(c * 64 + lane, S - 1);
        if (kOff32 && last == pb + kB - 1) {  // a full batch: the lane's 32-bit offset plus a row stride
            const unsigned o0 = ((unsigned)pb * (unsigned)S + sc) << 2, st = (unsigned)S << 2;
#pragma unroll
            for (int u = 0; u < kB; ++u)
                r[u] = __builtin_nontemporal_load(reinterpret_cast<const int *>(asg + (o0 + (unsigned)u * st)));
        } else {
#pragma unroll
            for (int u = 0; u < kB; ++u)  // a wave-uniform row base: the load's address is the lane's 32-bit offset
                r[u] = __builtin_nontemporal_load(assign + (size_t)min(pb + u, last) * S + sc);
        }
    };
    int kvb = N;  // the current batch's keys (lane u: pod pb + u's), taken from its chunk-0 unit
    auto examine = [&](int v, const int (&r)[kB]) {
        int bt, c;
        split(v, bt, c);
        const int pb = q0 + bt * kB, nb = min(kB, q1 - pb);
        if (c == 0) {  // the keys: readlanes of the rows' scenarios 0 / 21 / 42 (the majority; S < 43: 0)
            int kn = N;
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                int k0 = __builtin_amdgcn_readlane(r[u], 0);
                if (kMaj) {
                    const int k1 = __builtin_amdgcn_readlane(r[u], 21), k2 = __builtin_amdgcn_readlane(r[u], 42);
                    k0 = (k0 == k1 || k0 == k2) ? k0 : (k1 == k2 ? k1 : k0);
                }
                k0 = (unsigned)k0 < (unsigned)N ? k0 : N;
                kn = lane == u ? k0 : kn;
            }
            kvb = kn;
            if (lane < nb) {
                pkey[pb + lane] = kn;
                if (kn < N) atomicAdd(&lh[kn >> kNrBucketBits], 1);
            }
        }
        const int kv = kvb;  // lane u < 16: pod pb + u's key
        if (RSK_NR_ABL & 1) {
#pragma unroll
            for (int u = 0; u < kB; ++u) abl_acc ^= r[u] * (u + 1);
            return;
        }
        const int s = c * 64 + lane;
        const bool live = s < S;
        const int cb = nbk + c * nbk;  // the chunk's entry bins ([chunk][bucket]: no multiply per cell)
        // row u: one compare into a wave mask (v_cmp to SGPRs; rows with no
        // deviating lane skip on it); the deviating lanes write their entries,
        // lane u of kc collects the row's count for one key-bin add per unit
        int kc = 0;
        const unsigned long long liveM = __builtin_amdgcn_ballot_w64(live);
        auto emit = [&](int u, unsigned long long dm) {
            const bool inN = (unsigned)r[u] < (unsigned)N;
            E[wpos + nr_rank(dm)] = make_int2((inN ? r[u] : kNrNoNode) | ((pb + u - p0) << 20), s);
            if (inN) atomicAdd(&lh[cb + (r[u] >> kNrBucketBits)], 1);
        };
        // (llvm.amdgcn.icmp: the compare's own SGPR mask; a ballot of the bool
        // is materialised through a VGPR, two more VALU per row)
        if (nb == kB && wpos + (unsigned)(kB * 64) <= wcap) {  // a full batch with room for every cell
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int k = __builtin_amdgcn_readlane(kv, u);
                const unsigned long long dm = __builtin_amdgcn_uicmp((unsigned)r[u], (unsigned)k, 33 /* NE */) & liveM;
                if (!dm) continue;
                if (live && r[u] != k) emit(u, dm);
                const unsigned nd = (unsigned)__popcll(dm);
                kc = lane == u ? (int)nd : kc;
                wpos += nd;
            }
        } else {
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                const int k = __builtin_amdgcn_readlane(kv, u);
                const unsigned long long dm =
                    u < nb ? __builtin_amdgcn_uicmp((unsigned)r[u], (unsigned)k, 33 /* NE */) & liveM : 0ull;
                if (!dm) continue;
                const unsigned nd = (unsigned)__popcll(dm);
                if (wpos + nd > wcap) {
                    wover = true;  // (the block lists none: nr_spill adds its cells)
                    continue;
                }
                if (live && r[u] != k) emit(u, dm);
                kc = lane == u ? (int)nd : kc;
                wpos += nd;
            }
        }
        if (kc && kv < N) atomicAdd(&lh[cb + (kv >> kNrBucketBits)], kc);  // lanes < kB: the key nodes' counts
    };
    if (nv > 0) {
        int ra[kB], rb[kB];
        load(0, ra);
        // (the empty asm after each prefetch: the compiler may not hoist the
        // examined unit's first uses of its rows above the next unit's loads)
        for (int v = 0; v < nv; v += 2) {
            load(v + 1, rb);
            asm volatile("" : "+v"(ra[0])::"memory");
            examine(v, ra);
            load(v + 2, ra);
            asm volatile("" : "+v"(rb[0])::"memory");
            if (v + 1 < nv) examine(v + 1, rb);
        }
    }
    if (wover && lane == 0) over = 1;
    __syncthreads();
    const bool bo = over != 0;
    for (int j = t; j < nh; j += kNrThreads) bh[(size_t)j * nblk + b] = (bo && j >= nbk) ? 0 : lh[j];
    if (RSK_NR_ABL) asm volatile("" ::"v"(abl_acc));  // (keeps the ablated rows' loads)
    if (lane == 0) ecount[b * kW + wv] = bo ? -1 : (int)wpos;
}

// inclusive scan over a wave (DPP row shifts and broadcasts: no LDS round trips)
__device__ __forceinline__ int nr_wave_scan(int v, int lane) {
    (void)lane;
    return dpp_scan_incl(v);
}

// launch 2: one wave per counter j: bh[j][0..nblk) -> its exclusive prefix,
// tot[j] = the sum (kPer > 0: each lane's kPer blocks in registers, one
// memory trip; 0: nblk > 64 * 8, loops)
template <int kPer>
__global__ __launch_bounds__(256) void nr_colscan_kernel(int *__restrict__ bh, int nh, int nblk,
                                                         int *__restrict__ tot) {
    const int lane = (int)threadIdx.x & 63, j = (int)blockIdx.x * 4 + ((int)threadIdx.x >> 6);
    if (j >= nh) return;
    int *__restrict__ row = bh + (size_t)j * nblk;
    const int per = kPer ? kPer : (nblk + 63) >> 6, b0 = lane * per, b1 = min(nblk, b0 + per);
    int sum = 0;
    if (kPer) {
        int x[kPer > 0 ? kPer : 1];
#pragma unroll
        for (int i = 0; i < kPer; ++i) x[i] = row[min(b0 + i, nblk - 1)];
#pragma unroll
        for (int i = 0; i < kPer; ++i) sum += b0 + i < b1 ? x[i] : 0;
        const int incl = nr_wave_scan(sum, lane);
        int run = incl - sum;
#pragma unroll
        for (int i = 0; i < kPer; ++i)
            if (b0 + i < b1) {
                row[b0 + i] = run;
                run += x[i];
            }
        if (lane == 63) tot[j] = incl;
        return;
    }
    for (int i = b0; i < b1; ++i) sum += row[i];
    const int incl = nr_wave_scan(sum, lane);
    int run = incl - sum;
    for (int i = b0; i < b1; ++i) {
        const int x = row[i];
        row[i] = run;
        run += x;
    }
    if (lane == 63) tot[j] = incl;
}

// launch 3: LDS = the block's cursors [nh], the pods' cpu [kNrPods], keys
// [kNrPods] and (kMem) mem [kNrPods]; the counters' bases (exclusive scan of tot) are computed by
// every block, and written out by block 0 (base[nh] = the total)
template <bool kMem>
__global__ __launch_bounds__(kNrThreads) void nr_place_kernel(const int *__restrict__ pkey, int P, int N, int nbk,
                                                              int nchunk, int nblk, const int *__restrict__ bh,
                                                              const int *__restrict__ tot, int *__restrict__ base,
                                                              const int *__restrict__ pod_cpu,
                                                              const long long *__restrict__ pod_mem,
                                                              const int2 *__restrict__ ent, size_t ecap,
                                                              const int *__restrict__ ecount, int4 *__restrict__ rec,
                                                              int nrec, unsigned *__restrict__ err) {
    extern __shared__ __align__(16) int cur[];
    __shared__ int wsum[kNrThreads / 64];
    const int b = nr_block(nblk);
    if (b >= nblk) return;
    const int t = (int)threadIdx.x, lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);  // (uniform)
    const int nh = nbk * (1 + nchunk);
    int *lc = cur + nh, *lk = lc + kNrPods;
    long long *lm = reinterpret_cast<long long *>(lk + kNrPods + (nh & 1));  // 8-B aligned
    const int p0 = b * kNrPods, p1 = min(P, p0 + kNrPods);
    constexpr int kU = kNrPods / kNrThreads;
    int k[kU], c[kU];
    long long m[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {  // the pods' fields in flight while the bases are scanned
        const int p = min(p0 + u * kNrThreads + t, P - 1);
        k[u] = pkey[p];
        c[u] = pod_cpu[p];
        m[u] = kMem ? pod_mem[p] : 0;
    }
    // bases: thread t scans tot[t * per, ...) after the block's exclusive scan
    // of the threads' sums; its totals and column prefixes are loaded at once
    // into registers (predicated; a loop of loads waited on each in turn)
    constexpr int kPer = (kNrMaxCounters + kNrThreads - 1) / kNrThreads;
    const int per = (nh + kNrThreads - 1) / kNrThreads, j0 = min(nh, t * per), j1 = min(nh, j0 + per);
    int tv[kPer], hv[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const bool in = j0 + i < j1;
        tv[i] = in ? tot[j0 + i] : 0;
        hv[i] = in ? bh[(size_t)(j0 + i) * nblk + b] : 0;
    }
    int s = 0;
#pragma unroll
    for (int i = 0; i < kPer; ++i) s += tv[i];
    const int incl = nr_wave_scan(s, lane);
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int run = incl - s;
    for (int w = 0; w < wv; ++w) run += wsum[w];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        if (j0 + i < j1) {
            cur[j0 + i] = run + hv[i];
            if (b == 0) base[j0 + i] = run;
        }
        run += tv[i];
    }
    if (b == 0 && t == kNrThreads - 1) base[nh] = run;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        lc[u * kNrThreads + t] = c[u];
        lk[u * kNrThreads + t] = k[u];
        if (kMem) lm[u * kNrThreads + t] = m[u];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const int p = p0 + u * kNrThreads + t;
        if (p < p1 && k[u] < N) {
            const int pos = atomicAdd(&cur[k[u] >> kNrBucketBits], 1);
            if ((unsigned)pos < (unsigned)nrec)  // the offsets come from nr_scan's counts: guarded (dev_err)
                rec[pos] = make_int4(k[u] & (kNrBucketNodes - 1), c[u], (int)(unsigned)(unsigned long long)m[u],
                                     (int)(m[u] >> 32));
            else
                *err = kErrNrPlace;
        }
    }
    // the entries of the block's 8 wave regions, concatenated (-1: overflowed,
    // nr_spill adds the block's deviations)
    constexpr int kW = kNrThreads / 64;
    int wc[kW], ne = 0;
#pragma unroll
    for (int w = 0; w < kW; ++w) {
        wc[w] = max(0, ecount[b * kW + w]);
        ne += wc[w];
    }
    const size_t wcap = ecap / kW;
    const int2 *__restrict__ E = ent + (size_t)b * ecap;
    constexpr int kV = 4;
    for (int i0 = 0; i0 < ne; i0 += kNrThreads * kV) {
        int2 e[kV];
#pragma unroll
        for (int v = 0; v < kV; ++v) {
            int i = min(i0 + v * kNrThreads + t, ne - 1), w = 0;
#pragma unroll
            for (int x = 0; x < kW - 1; ++x)
                if (w == x && i >= wc[x]) {
                    i -= wc[x];
                    w = x + 1;
                }
            e[v] = E[(size_t)w * wcap + i];
        }
#pragma unroll
        for (int v = 0; v < kV; ++v) {
            if (i0 + v * kNrThreads + t < ne) {
                const int node = e[v].x & kNrNoNode, lp = (int)((unsigned)e[v].x >> 20), sc = e[v].y;
                const int key = lk[lp], lane = (sc & 63) << 6;
                const long long mm = kMem ? lm[lp] : 0;
                const int mlo = (int)(unsigned)(unsigned long long)mm, mhi = (int)(mm >> 32);
                if (node < N) {  // + the pod at its node
                    const int pos = atomicAdd(&cur[nbk + __umul24(sc >> 6, nbk) + (node >> kNrBucketBits)], 1);
                    if ((unsigned)pos < (unsigned)nrec) rec[pos] = make_int4((node & (kNrBucketNodes - 1)) | lane, lc[lp], mlo, mhi);
                    else *err = kErrNrPlace;
                }
                if (key < N) {  // - the pod at its key node
                    const int pos = atomicAdd(&cur[nbk + __umul24(sc >> 6, nbk) + (key >> kNrBucketBits)], 1);
                    if ((unsigned)pos < (unsigned)nrec) rec[pos] = make_int4((key & (kNrBucketNodes - 1)) | 32 | lane, lc[lp], mlo, mhi);
                    else *err = kErrNrPlace;
                }
            }
        }
    }
}

// launch 4: a workgroup per bin (chunk c, bucket b)
constexpr int kNrSumThreads = 256;
template <bool kMem>
__global__ __launch_bounds__(kNrSumThreads) void nr_sum_kernel(const int *__restrict__ base, int nbk, int nchunk,
                                                               const int4 *__restrict__ rec, int N, int S,
                                                               int *__restrict__ cnt,
                                                               unsigned long long *__restrict__ cpu,
                                                               unsigned long long *__restrict__ mem) {
    constexpr int kE = kNrBucketNodes * 64;
    __shared__ int bc[kNrBucketNodes];
    __shared__ unsigned long long bcpu[kNrBucketNodes], bmem[kNrBucketNodes];
    __shared__ int dc[kE];
    __shared__ unsigned long long dcpu[kE], dmem[kMem ? kE : 1];
    const int t = (int)threadIdx.x, g = (int)blockIdx.x, c = g / nbk, b = g - c * nbk;
    const int lo = base[b], hi = base[b + 1];
    const int j = nbk + g, elo = base[j], ehi = base[j + 1];  // bins [chunk][bucket]
    if (t < kNrBucketNodes) {
        bc[t] = 0;
        bcpu[t] = 0ull;
        bmem[t] = 0ull;
    }
    for (int e = t; e < kE; e += kNrSumThreads) {
        dc[e] = 0;
        dcpu[e] = 0ull;
        if (kMem) dmem[e] = 0ull;
    }
    __syncthreads();
    constexpr int kV = 4;
    for (int i0 = lo; i0 < hi; i0 += kNrSumThreads * kV) {  // the bucket's pods: base
        int4 r[kV];
#pragma unroll
        for (int v = 0; v < kV; ++v) r[v] = rec[min(i0 + v * kNrSumThreads + t, hi - 1)];
#pragma unroll
        for (int v = 0; v < kV; ++v) {
            if (i0 + v * kNrSumThreads + t < hi) {
                const int n = r[v].x;
                atomicAdd(&bc[n], 1);
                atomicAdd(&bcpu[n], (unsigned long long)(long long)r[v].y);
                if (kMem) atomicAdd(&bmem[n], ((unsigned long long)(unsigned)r[v].w << 32) | (unsigned)r[v].z);
            }
        }
    }
    for (int i0 = elo; i0 < ehi; i0 += kNrSumThreads * kV) {  // the bin's deviation entries
        int4 r[kV];
#pragma unroll
        for (int v = 0; v < kV; ++v) r[v] = rec[min(i0 + v * kNrSumThreads + t, ehi - 1)];
#pragma unroll
        for (int v = 0; v < kV; ++v) {
            if (i0 + v * kNrSumThreads + t < ehi) {
                const int x = r[v].x, e = (x & (kNrBucketNodes - 1)) * 64 + ((x >> 6) & 63);
                const bool neg = (x >> 5) & 1;
                const long long cv = r[v].y;
                atomicAdd(&dc[e], neg ? -1 : 1);
                atomicAdd(&dcpu[e], (unsigned long long)(neg ? -cv : cv));
                if (kMem) {
                    const unsigned long long mv = ((unsigned long long)(unsigned)r[v].w << 32) | (unsigned)r[v].z;
                    atomicAdd(&dmem[e], neg ? 0ull - mv : mv);
                }
            }
        }
    }
    __syncthreads();
    for (int e = t; e < kE; e += kNrSumThreads) {
        const int l = e >> 6, n = b * kNrBucketNodes + l, s = c * 64 + (e & 63);
        if (n >= N || s >= S) continue;
        const size_t o = (size_t)n * S + s;
        cnt[o] = bc[l] + dc[e];
        cpu[o] = bcpu[l] + dcpu[e];
        if (kMem) mem[o] = bmem[l] + dmem[e];
    }
}

// launch 5: the deviation cells of the blocks that overflowed, by atomics on
// the stored sums (none on the bench batches: every block exits at once)
template <bool kMem>
__global__ __launch_bounds__(kNrThreads) void nr_spill_kernel(const int *__restrict__ assign, int P, int S, int N,
                                                              int nblk, const int *__restrict__ pkey,
                                                              const int *__restrict__ ecount,
                                                              const int *__restrict__ pod_cpu,
                                                              const long long *__restrict__ pod_mem,
                                                              int *__restrict__ cnt,
                                                              unsigned long long *__restrict__ cpu,
                                                              unsigned long long *__restrict__ mem) {
    // (a workgroup per block: 32 workgroups striding over the blocks measured
    // 4.8 against 4.4 us on the bench batches, where no block has work)
    const int b = nr_block(nblk);
    if (b >= nblk || ecount[b * (kNrThreads / 64)] >= 0) return;
    const int p0 = b * kNrPods, p1 = min(P, p0 + kNrPods);
    const size_t n = (size_t)(p1 - p0) * S;
    for (size_t i = threadIdx.x; i < n; i += kNrThreads) {
        const int p = p0 + (int)(i / (size_t)S), s = (int)(i % (size_t)S);
        const int a = assign[(size_t)p * S + s], k = pkey[p];
        if (a == k) continue;
        const long long c = pod_cpu[p], m = kMem ? pod_mem[p] : 0;
        if ((unsigned)a < (unsigned)N) {
            const size_t o = (size_t)a * S + s;
            atomicAdd(&cnt[o], 1);
            atomicAdd(&cpu[o], (unsigned long long)c);
            if (kMem) atomicAdd(&mem[o], (unsigned long long)m);
        }
        if (k < N) {
            const size_t o = (size_t)k * S + s;
            atomicAdd(&cnt[o], -1);
            atomicAdd(&cpu[o], (unsigned long long)-c);
            if (kMem) atomicAdd(&mem[o], (unsigned long long)-m);
        }
    }
}

// get_resource_usage.py:37: int(round(u / c * 100)) — IEEE fp64 divide, then an
// fp64 multiply (no FMA can form), then round-half-even (rint).
__global__ __launch_bounds__(256) void cpu_pct_kernel(const int *__restrict__ use, const int *__restrict__ cap, int N,
                                                      int S, int *__restrict__ pct) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (size_t)N * S) return;
    const int n = (int)(t / (size_t)S);
    const int c = cap[n];
    if (c == 0) { pct[t] = -1; return; }
    const double q = (double)use[t] / (double)c;
    pct[t] = (int)rint(q * 100.0);
}

// harzard_detect.py:3-27: hazard flag and the first node with the max pct.
__global__ __launch_bounds__(256) void detect_kernel(const int *__restrict__ pct, int N, int S, int thr, int npb,
                                                     unsigned total, uint8_t *__restrict__ haz,
                                                     unsigned long long *__restrict__ most) {
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (t >= total) return;
    const int s = (int)(t % (unsigned)S);
    const int n0 = (int)(t / (unsigned)S) * npb, n1 = min(N, n0 + npb);
    unsigned long long b = 0;
    for (int n = n0; n < n1; ++n) {
        const size_t idx = (size_t)n * S + s;
        const int v = pct[idx];
        const bool h = v >= thr;
        haz[idx] = h;
        if (h) {
            const unsigned long long k = pack_hi_lo(v, ~(unsigned)n);
            b = k > b ? k : b;
        }
    }
    if (b) atomicMax(&most[s], b);
}

__global__ void decode_first_max(const unsigned long long *__restrict__ key, int S, int *__restrict__ out) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= S) return;
    const unsigned long long k = key[s];
    out[s] = k ? (int)(~(unsigned)(k & 0xffffffffull)) : -1;
}

// nodemonitor.py:24-46.  Per (node chunk, s): count, chunk mean and M2 in one
// pass over pct = use / cap * 100 in fp64 — the reference's own operation
// order (nodemonitor.py:39), so every node's pct is bit-identical to it; nodes
// with cap <= 0 are skipped (:38-43).  Shifted sums (d = pct - the chunk's
// first pct: the sum and sum of squares of d, M2 = sq - sum^2 / c — exact 0
// for equal values, ~1e-15 relative otherwise); then per s a fixed-order Chan
// merge.  The summation order differs from numpy's pairwise mean and two-pass
// variance, so the std agrees within tolerance (the tests: 1e-9 relative; the
// north star: 1e-5), not bit for bit.  When S divides 256 a workgroup holds
// F = 256 / S whole chunks for every scenario and folds them (in order, in
// LDS) into one partial per scenario before writing: F times fewer partials
// for the merge to read (50k nodes x 64 scenarios: 500 instead of 2,000).
__device__ __forceinline__ void chan_merge(long long &n, double &mean, double &m2, long long nb, double mb, double m2b);

__global__ __launch_bounds__(256) void std_partial_kernel(const int *__restrict__ use, const int *__restrict__ cap,
                                                          int N, int S, int npb, unsigned total, int fold,
                                                          double *__restrict__ pmean, double *__restrict__ pm2,
                                                          int *__restrict__ pcnt) {
#pragma clang fp contract(off)
    __shared__ double fm[256], fq[256];
    __shared__ int fc[256];
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (!fold && t >= total) return;
    const int s = (int)(t % (unsigned)S), ch = (int)(t / (unsigned)S);
    const int n0 = ch * npb, n1 = t < total ? min(N, n0 + npb) : n0;  // past the end: an empty chunk
    constexpr int kU = 8;  // loads in flight per thread
    double sum = 0.0, sq = 0.0, K = 0.0;
    int c = 0;
    for (int n = n0; n < n1; n += kU) {
        int u[kU], cp[kU];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const int m = min(n + k, n1 - 1);  // clamped: always a valid address
            u[k] = use[(size_t)m * S + s];
            cp[k] = cap[m];
        }
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            if (n + k < n1 && cp[k] > 0) {
                const double x = (double)u[k] / (double)cp[k] * 100.0;
                if (c == 0) K = x;
                const double d = x - K;
                sum += d;
                sq += d * d;
                ++c;
            }
        }
    }
    const double mean = c ? K + sum / c : 0.0;
    const double m2 = c ? fmax(0.0, sq - sum * (sum / c)) : 0.0;
    if (!fold) {
        const size_t o = (size_t)ch * S + s;
        pmean[o] = mean;
        pm2[o] = m2;
        pcnt[o] = c;
        return;
    }
    const int tl = (int)threadIdx.x;
    fm[tl] = mean;
    fq[tl] = m2;
    fc[tl] = c;
    __syncthreads();
    if (tl >= S) return;
    long long n = 0;
    double fmean = 0.0, fm2 = 0.0;
    for (int f = tl; f < 256; f += S) chan_merge(n, fmean, fm2, fc[f], fm[f], fq[f]);
    const size_t o = (size_t)blockIdx.x * S + tl;
    pmean[o] = fmean;
    pm2[o] = fm2;
    pcnt[o] = (int)n;
}

// Chan et al.'s pairwise update: (n, mean, m2) of a union from its two parts.
__device__ __forceinline__ void chan_merge(long long &n, double &mean, double &m2, long long nb, double mb, double m2b) {
#pragma clang fp contract(off)
    if (!nb) return;
    if (!n) { n = nb; mean = mb; m2 = m2b; return; }
    const double delta = mb - mean;
    const long long nt = n + nb;
    mean += delta * ((double)nb / (double)nt);
    m2 += m2b + delta * delta * ((double)n * (double)nb / (double)nt);
    n = nt;
}

// One workgroup per scenario: thread t merges chunks t, t + 256, ... in order
// (a batch of loads in flight before it is merged), then each wave's 64
// states pairwise (xor butterfly, 6 levels), then thread 0 the four waves in
// order; the result is the same for every run (fixed order).  (One thread per
// scenario walking every chunk in a chain of fp64 divides took 1.6 ms at 50k
// nodes x 64 scenarios; one wave per scenario 15 us.)  Partials are
// [chunk][scenario], so one 64-B line holds 8 neighbouring scenarios' values:
// workgroup b takes scenario (b % 8) * S/8 + b / 8, so the workgroups that
// share an XCD (and its L2) share those lines instead of every XCD fetching
// every line.
__global__ __launch_bounds__(256) void std_merge_kernel(const double *__restrict__ pmean, const double *__restrict__ pm2,
                                                        const int *__restrict__ pcnt, int nchunks, int S,
                                                        double *__restrict__ out) {
    __shared__ double wm[4], wq[4];
    __shared__ long long wn[4];
    const int b = (int)blockIdx.x;
    const int s = (S & 7) ? b : (b & 7) * (S >> 3) + (b >> 3);
    const int t = (int)threadIdx.x, lane = t & 63, w = t >> 6;
    double mean = 0.0, m2 = 0.0;
    long long n = 0;
    constexpr int kU = 4;
    for (int ch0 = t; ch0 < nchunks; ch0 += 256 * kU) {
        int c[kU];
        double mb[kU], qb[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int ch = ch0 + 256 * u;
            const size_t o = (size_t)min(ch, nchunks - 1) * S + s;  // clamped; counted 0 past the end
            c[u] = ch < nchunks ? pcnt[o] : 0;
            mb[u] = pmean[o];
            qb[u] = pm2[o];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) chan_merge(n, mean, m2, c[u], mb[u], qb[u]);
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const long long nb = __shfl_xor(n, off, 64);
        const double mb = __shfl_xor(mean, off, 64), m2b = __shfl_xor(m2, off, 64);
        // both lanes of a pair combine (lower lane first) so they hold the same state
        if (lane & off) {
            long long n2 = nb;
            double mean2 = mb, m22 = m2b;
            chan_merge(n2, mean2, m22, n, mean, m2);
            n = n2, mean = mean2, m2 = m22;
        } else {
            chan_merge(n, mean, m2, nb, mb, m2b);
        }
    }
    if (lane == 0) {
        wn[w] = n;
        wm[w] = mean;
        wq[w] = m2;
    }
    __syncthreads();
    if (t == 0) {
        n = wn[0], mean = wm[0], m2 = wq[0];
        for (int k = 1; k < 4; ++k) chan_merge(n, mean, m2, wn[k], wm[k], wq[k]);
        out[s] = n ? sqrt(m2 / (double)n) : 0.0;
    }
}

constexpr int kCutBins = 64;

// communicationcost.py:37-45: directed count of related pairs on different nodes.
// rows [r0, r1) of the CSR; neighbours read from the full assign
__global__ __launch_bounds__(256) void cut_cost_kernel(const int *__restrict__ row_ptr, const int *__restrict__ col,
                                                       int r0, int r1, const int *__restrict__ assign, int S,
                                                       const int *__restrict__ missing, int ppt, unsigned total,
                                                       unsigned long long *__restrict__ out) {
    // thread i of the block holds scenario (b0 + i) % S: threads with equal i mod
    // min(S, 256) share a scenario, so their counts meet in one LDS slot and the
    // block issues at most 256 global atomics (not one per thread)
    __shared__ unsigned long long red[256];
    red[threadIdx.x] = 0ull;
    __syncthreads();
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    const unsigned nslot = S < 256 ? (unsigned)S : 256u;
    if (t < total) {
        const int s = (int)(t % (unsigned)S);
        const int p0 = r0 + (int)(t / (unsigned)S) * ppt, p1 = min(r1, p0 + ppt);
        unsigned long long c = 0;
        for (int p = p0; p < p1; ++p) {
            const int a = assign[(size_t)p * S + s];
            for (int k = row_ptr[p]; k < row_ptr[p + 1]; ++k) c += a != assign[(size_t)col[k] * S + s];
            if (missing && a != -1) c += (unsigned long long)missing[p];
        }
        if (c) atomicAdd(&red[threadIdx.x % nslot], c);
    }
    __syncthreads();
    // then one of kCutBins rows of per-scenario bins (blocks spread over the
    // rows so no address sees more than blocks / kCutBins atomics)
    const unsigned long long v = threadIdx.x < nslot ? red[threadIdx.x] : 0ull;
    if (v) atomicAdd(&out[(size_t)(blockIdx.x % kCutBins) * S + (blockIdx.x * 256u + threadIdx.x) % (unsigned)S], v);
}

// The same count with lane = scenario (S >= 32), edge-balanced: the waves of
// a 64-scenario chunk take fixed ranges of kCutEdges edges (grid-stride), so a
// hub row's edges spread over many waves instead of one thread walking them
// all (the thread-per-(rows, scenario) kernel above: 1.6 ms at 1M rows x 64
// scenarios, its hub threads the tail).  A range finds its first row by a
// scalar binary search over row_ptr; then per step up to 16 edges: the next 16
// row ends and the 16 neighbour ids by scalar loads, each edge's row from the
// ends by scalar compares, 32 coalesced assignment loads in flight (the row's
// own value and the neighbour's).  The rows' missing terms go in 64-row
// blocks, grid-stride as well.
constexpr int kCutEdges = 512;
__global__ __launch_bounds__(256) void cut_cost_wave_kernel(const int *__restrict__ row_ptr, const int *__restrict__ col,
                                                            int r0, int r1, const int *__restrict__ assign, int S,
                                                            const int *__restrict__ missing, int nw,
                                                            unsigned long long *__restrict__ bins) {
    const int lane = threadIdx.x & 63;
    const int wv = (int)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int chunk = wv / nw, w = wv - chunk * nw;
    if (chunk * 64 >= S) return;
    const bool live = chunk * 64 + lane < S;
    const size_t s = (size_t)min(chunk * 64 + lane, S - 1);
    const cint_ptr rp = const_ptr(row_ptr), cl = const_ptr(col), ms = const_ptr(missing);
    unsigned long long c = 0;
    if (missing) {
        // 64-bit strides: b0 + nw * 64 may pass INT32_MAX near the end
        for (long long b0 = r0 + (long long)w * 64; b0 < r1; b0 += (long long)nw * 64)
            for (int b = (int)b0; b < (int)min(b0 + 64, (long long)r1); b += 16) {
                int ap[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) ap[i] = assign[(size_t)min(b + i, r1 - 1) * S + s];
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (b + i < r1 && ap[i] != -1) c += (unsigned long long)(unsigned)ms[b + i];
            }
    }
    const int ea = rp[r0], eb = rp[r1];
    for (long long ka64 = ea + (long long)w * kCutEdges; ka64 < eb; ka64 += (long long)nw * kCutEdges) {
        const int ka = (int)ka64;
        const int kb = (int)min(ka64 + kCutEdges, (long long)eb);
        // the row of edge ka (the last p with row_ptr[p] <= ka): a 16-way
        // search, 16 independent scalar loads per round
        int lo = r0, hi = r1 - 1;
        while (hi - lo > 16) {
            const int step = (hi - lo + 15) / 16;
            int nlo = lo, nhi = hi;
#pragma unroll
            for (int i = 1; i < 16; ++i) {
                const int m = min(lo + i * step, hi);
                const bool le = rp[m] <= ka;
                nlo = le ? max(nlo, m) : nlo;
                nhi = le ? nhi : min(nhi, m - 1);
            }
            lo = nlo;
            hi = nhi;
        }
        while (lo < hi && rp[lo + 1] <= ka) ++lo;
        int p = lo, k0 = ka;
        constexpr int kW = 32;  // edges per step, row ends per window
        while (k0 < kb) {
            int o[kW];  // ends of rows p .. p + kW - 1
#pragma unroll
            for (int i = 0; i < kW; ++i) o[i] = rp[min(p + 1 + i, r1)];
            const int kend = min(min(kb, k0 + kW), o[kW - 1]);
            if (kend <= k0) { p += kW; continue; }  // kW rows without edges here
            // the row of edge k0 + j is p + #{i : o[i] <= k0 + j}: lane j counts it
            // for its edge (31 VALU for the window, not 31 per edge), and every
            // edge's count is read back as a scalar
            const int kl = min(k0 + (lane & (kW - 1)), kend - 1);
            int rl = 0;
#pragma unroll
            for (int i = 0; i < kW - 1; ++i) rl += o[i] <= kl ? 1 : 0;
            const int last = __builtin_amdgcn_readlane(rl, kend - 1 - k0);
            int aq[kW], am[kW];
#pragma unroll
            for (int j = 0; j < kW; ++j) {
                const int k = min(k0 + j, kend - 1);
                const int r = __builtin_amdgcn_readlane(rl, j);
                aq[j] = assign[(size_t)cl[k] * S + s];
                am[j] = assign[(size_t)(p + r) * S + s];
            }
#pragma unroll
            for (int j = 0; j < kW; ++j) c += (k0 + j < kend && am[j] != aq[j]) ? 1ull : 0ull;
            p += last;
            k0 = kend;
        }
    }
    if (live && c) atomicAdd(&bins[(size_t)(wv % kCutBins) * S + s], c);
}

__global__ __launch_bounds__(256) void cut_bins_sum(const unsigned long long *__restrict__ bins, int S,
                                                    unsigned long long *__restrict__ out) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= S) return;
    unsigned long long c = 0;
    for (int b = 0; b < kCutBins; ++b) c += bins[(size_t)b * S + s];
    out[s] = c;
}

// delete_replaced_pod.py:41-61: first pod (list order) with the largest cpu > -1.
__global__ __launch_bounds__(256) void pick_pod_kernel(const int *__restrict__ assign, const int *__restrict__ pod_cpu,
                                                       int P, int S, const int *__restrict__ most, int ppt,
                                                       unsigned total, unsigned long long *__restrict__ best) {
    const unsigned t = blockIdx.x * 256u + threadIdx.x;
    if (t >= total) return;
    const int s = (int)(t % (unsigned)S);
    const int m = most[s];
    if (m < 0) return;
    const int p0 = (int)(t / (unsigned)S) * ppt, p1 = min(P, p0 + ppt);
    unsigned long long b = 0;
    for (int p = p0; p < p1; ++p) {
        if (assign[(size_t)p * S + s] != m || pod_cpu[p] < 0) continue;
        const unsigned long long k = pack_hi_lo(pod_cpu[p], ~(unsigned)p);
        b = k > b ? k : b;
    }
    if (b) atomicMax(&best[s], b);
}

int launch_cpu_pct(hipStream_t stream, const int *use, const int *cap, int N, int S, int *pct) {
    const size_t NS = (size_t)N * S;
    cpu_pct_kernel<<<(unsigned)ceil_div(NS, 256), 256, 0, stream>>>(use, cap, N, S, pct);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int launch_detect(hipStream_t stream, const int *pct, int N, int S, int threshold, uint8_t *hazard,
                  unsigned long long *key_ws, int *most) {
    RSK_HIP(hipMemsetAsync(key_ws, 0, (size_t)S * 8, stream));
    const int npb = chunk_for(N, S);
    const unsigned total = (unsigned)(ceil_div(N, npb) * S);
    detect_kernel<<<(unsigned)ceil_div(total, 256), 256, 0, stream>>>(pct, N, S, threshold, npb, total, hazard,
                                                                       key_ws);
    decode_first_max<<<(unsigned)ceil_div(S, 256), 256, 0, stream>>>(key_ws, S, most);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int launch_decode_first_max(hipStream_t stream, const unsigned long long *key, int S, int *out_pod) {
    decode_first_max<<<(unsigned)ceil_div(S, 256), 256, 0, stream>>>(key, S, out_pod);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int launch_pick_max_pod(hipStream_t stream, const int *assign, const int *pod_cpu, int P, int S, const int *most,
                        unsigned long long *key_ws, int *out_pod) {
    RSK_HIP(hipMemsetAsync(key_ws, 0, (size_t)S * 8, stream));
    if (P > 0) {
        const int ppt = chunk_for(P, S);
        const int64_t tot = ceil_div(P, ppt) * S;
        RSK_CHECK(tot < INT32_MAX, "grid too large");
        pick_pod_kernel<<<(unsigned)ceil_div(tot, 256), 256, 0, stream>>>(assign, pod_cpu, P, S, most, ppt,
                                                                          (unsigned)tot, key_ws);
    }
    decode_first_max<<<(unsigned)ceil_div(S, 256), 256, 0, stream>>>(key_ws, S, out_pod);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

}  // namespace rsk

using namespace rsk;

extern "C" {

int rsk_spread_place(rsk_ctx *ctx, const int32_t *pod_count, const int32_t *name_rank, const uint8_t *hazard,
                     int32_t N, int32_t S, int32_t *out_node, uint32_t flags) {
    return pick_node<true>(ctx, pod_count, name_rank, hazard, N, S, out_node, flags, "spread");
}

int rsk_binpack_place(rsk_ctx *ctx, const int32_t *cpu_pct, const int32_t *name_rank, const uint8_t *hazard,
                      int32_t N, int32_t S, int32_t *out_node, uint32_t flags) {
    return pick_node<false>(ctx, cpu_pct, name_rank, hazard, N, S, out_node, flags, "binpack");
}

static int random_count_impl(rsk_ctx *ctx, const uint8_t *d_haz, int N, int S, int **d_count, int *npb_out,
                             int *nchunks_out) {
    const int npb = chunk_for(N, S);
    const int nchunks = (int)ceil_div(N, npb);
    RSK_TRY(ctx->work[2].reserve((size_t)nchunks * S * 4));
    RSK_TRY(ctx->work[3].reserve((size_t)S * 4));
    RSK_HIP(hipMemsetAsync(ctx->work[3].ptr, 0, (size_t)S * 4, ctx->stream));
    const unsigned total = (unsigned)((int64_t)nchunks * S);
    ScopedTimer tm(ctx, "random_count");
    count_free_kernel<<<(unsigned)ceil_div(total, 256), 256, 0, ctx->stream>>>(d_haz, N, S, npb, total,
                                                                               ctx->work[2].as<int>(),
                                                                               ctx->work[3].as<int>());
    RSK_HIP(hipGetLastError());
    *d_count = ctx->work[3].as<int>();
    *npb_out = npb;
    *nchunks_out = nchunks;
    return RSK_OK;
}

int rsk_random_count(rsk_ctx *ctx, const uint8_t *hazard, int32_t N, int32_t S, int32_t *out_count,
                     uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(N > 0 && S > 0 && (int64_t)N * S < INT32_MAX && out_count, "bad arguments");
    const bool dev = flags & RSK_F_DEVICE;
    const uint8_t *d_haz;
    RSK_TRY(stage_in(ctx, 0, hazard, (size_t)N * S, dev, reinterpret_cast<const void **>(&d_haz)));
    int *d_cnt, npb, nch;
    RSK_TRY(random_count_impl(ctx, d_haz, N, S, &d_cnt, &npb, &nch));
    if (dev) {
        RSK_HIP(hipMemcpyAsync(out_count, d_cnt, (size_t)S * 4, hipMemcpyDeviceToDevice, ctx->stream));
    } else {
        RSK_TRY(copy_back(ctx, out_count, d_cnt, (size_t)S * 4, false));
        RSK_HIP(hipStreamSynchronize(ctx->stream));
    }
    return RSK_OK;
}

static int random_select_impl(rsk_ctx *ctx, const uint8_t *d_haz, int N, int S, const int *d_r, int *d_out) {
    int *d_cnt, npb, nch;
    RSK_TRY(random_count_impl(ctx, d_haz, N, S, &d_cnt, &npb, &nch));
    ScopedTimer tm(ctx, "random_select");
    select_free_kernel<<<(unsigned)ceil_div(S, 256), 256, 0, ctx->stream>>>(d_haz, N, S, npb, nch,
                                                                            ctx->work[2].as<int>(), d_r, d_out);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int rsk_random_select(rsk_ctx *ctx, const uint8_t *hazard, int32_t N, int32_t S, const int32_t *r, int32_t *out_node,
                      uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(N > 0 && S > 0 && (int64_t)N * S < INT32_MAX && r && out_node, "bad arguments");
    const bool dev = flags & RSK_F_DEVICE;
    const uint8_t *d_haz;
    const int *d_r;
    int *d_out;
    RSK_TRY(stage_in(ctx, 0, hazard, (size_t)N * S, dev, reinterpret_cast<const void **>(&d_haz)));
    RSK_TRY(stage_in(ctx, 1, r, (size_t)S * 4, dev, reinterpret_cast<const void **>(&d_r)));
    RSK_TRY(stage_out(ctx, 2, out_node, (size_t)S * 4, dev, reinterpret_cast<void **>(&d_out)));
    RSK_TRY(random_select_impl(ctx, d_haz, N, S, d_r, d_out));
    if (!dev) {
        RSK_TRY(copy_back(ctx, out_node, d_out, (size_t)S * 4, false));
        RSK_HIP(hipStreamSynchronize(ctx->stream));
        for (int s = 0; s < S; ++s)
            if (out_node[s] == RSK_TARGET_NO_CANDIDATE) return RSK_NO_CANDIDATE;
    }
    return RSK_OK;
}

int32_t rsk_py_randbelow(uint64_t seed, int32_t n) {
    if (n <= 0) return -1;
    MT st;
    uint32_t key[2];
    int len = 0;
    if (seed == 0) key[len++] = 0;
    else {
        key[len++] = (uint32_t)seed;
        if (seed >> 32) key[len++] = (uint32_t)(seed >> 32);
    }
    st.init_by_array(key, len);
    int k = 0;
    while (k < 32 && ((uint32_t)n >> k)) ++k;
    uint32_t r;
    do r = st.next() >> (32 - k);
    while (r >= (uint32_t)n);
    return (int32_t)r;
}

int rsk_car_row(rsk_ctx *ctx, const int32_t *node_of, int32_t k, const int32_t *cap_cpu, const int32_t *use_cpu,
                const uint8_t *hazard, int32_t N, int32_t *out_target, int32_t *out_score, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(N > 0 && N <= kRowMaxN && k >= 0 && cap_cpu && use_cpu && hazard && out_target && (k == 0 || node_of),
              "rsk_car_row: bad arguments (N=%d, 1..%d, k=%d)", N, kRowMaxN, k);
    const bool dev = flags & RSK_F_DEVICE;
    const int *d_nodes = nullptr, *d_cap, *d_use;
    const uint8_t *d_haz;
    int *d_out;
    // host pointers: the inputs packed into the mapped pinned buffer, the result written back there
    RowIO io;
    if (dev) {
        d_nodes = node_of;
        d_cap = cap_cpu;
        d_use = use_cpu;
        d_haz = hazard;
        RSK_TRY(ctx->work[5].reserve(16));
        d_out = ctx->work[5].as<int>();
    } else {
        const void *src[4] = {node_of, cap_cpu, use_cpu, hazard};
        const size_t len[4] = {(size_t)k * 4, (size_t)N * 4, (size_t)N * 4, (size_t)N};
        RSK_TRY(row_io(ctx, src, len, 4, 16, &io));
        d_nodes = reinterpret_cast<const int *>(io.in + io.off[0]);
        d_cap = reinterpret_cast<const int *>(io.in + io.off[1]);
        d_use = reinterpret_cast<const int *>(io.in + io.off[2]);
        d_haz = reinterpret_cast<const uint8_t *>(io.in + io.off[3]);
        d_out = reinterpret_cast<int *>(io.out_dev);
    }
    const size_t lds = ((size_t)((N + 3) & ~3) + 2 * (kRowThreads / 64)) * 4;
    if (lds > 64 * 1024)
        RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&car_row_kernel),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    {
        ScopedTimer tm(ctx, "car_row");
        car_row_kernel<<<1, kRowThreads, lds, ctx->stream>>>(d_nodes, k, d_cap, d_use, d_haz, N, d_out);
        RSK_HIP(hipGetLastError());
    }
    if (dev) {
        RSK_HIP(hipMemcpyAsync(out_target, d_out, 4, hipMemcpyDeviceToDevice, ctx->stream));
        if (out_score) RSK_HIP(hipMemcpyAsync(out_score, d_out + 1, 4, hipMemcpyDeviceToDevice, ctx->stream));
        return RSK_OK;
    }
    RSK_HIP(hipStreamSynchronize(ctx->stream));
    const volatile int *r = reinterpret_cast<const volatile int *>(io.out_host);
    *out_target = r[0];
    if (out_score) *out_score = r[1];
    return r[0] == RSK_TARGET_NO_CANDIDATE ? RSK_NO_CANDIDATE : RSK_OK;
}

int rsk_random_candidates(rsk_ctx *ctx, const uint8_t *hazard, int32_t N, int32_t *out_nodes, int32_t *out_count) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(N > 0 && hazard && out_nodes && out_count, "rsk_random_candidates: bad arguments (N=%d)", N);
    const void *src[1] = {hazard};
    const size_t len[1] = {(size_t)N};
    RowIO io;
    RSK_TRY(row_io(ctx, src, len, 1, (size_t)N * 4 + 16, &io));
    {
        ScopedTimer tm(ctx, "random_candidates");
        candidates_row_kernel<<<1, kRowThreads, 0, ctx->stream>>>(reinterpret_cast<const uint8_t *>(io.in + io.off[0]),
                                                                  N, reinterpret_cast<int *>(io.out_dev) + 4,
                                                                  reinterpret_cast<int *>(io.out_dev));
        RSK_HIP(hipGetLastError());
    }
    RSK_HIP(hipStreamSynchronize(ctx->stream));
    const volatile int *r = reinterpret_cast<const volatile int *>(io.out_host);
    const int cnt = r[0];
    RSK_CHECK(cnt >= 0 && cnt <= N, "rsk_random_candidates: bad count %d", cnt);
    std::memcpy(out_nodes, const_cast<const int *>(r) + 4, (size_t)cnt * 4);
    *out_count = cnt;
    return RSK_OK;
}

int rsk_random_place(rsk_ctx *ctx, const uint8_t *hazard, int32_t N, int32_t S, const uint64_t *seeds,
                     int32_t *out_node, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(N > 0 && S > 0 && (int64_t)N * S < INT32_MAX && seeds && out_node, "bad arguments");
    const bool dev = flags & RSK_F_DEVICE;
    const uint8_t *d_haz;
    int *d_out;
    RSK_TRY(stage_in(ctx, 0, hazard, (size_t)N * S, dev, reinterpret_cast<const void **>(&d_haz)));
    RSK_TRY(stage_out(ctx, 2, out_node, (size_t)S * 4, dev, reinterpret_cast<void **>(&d_out)));
    int *d_cnt, npb, nch;
    RSK_TRY(random_count_impl(ctx, d_haz, N, S, &d_cnt, &npb, &nch));
    std::vector<int> cnt(S), r(S);
    std::vector<uint64_t> h_seeds(S);
    RSK_HIP(hipMemcpyAsync(cnt.data(), d_cnt, (size_t)S * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (dev) RSK_HIP(hipMemcpyAsync(h_seeds.data(), seeds, (size_t)S * 8, hipMemcpyDeviceToHost, ctx->stream));
    else std::memcpy(h_seeds.data(), seeds, (size_t)S * 8);
    RSK_HIP(hipStreamSynchronize(ctx->stream));
    for (int s = 0; s < S; ++s) r[s] = cnt[s] > 0 ? rsk_py_randbelow(h_seeds[s], cnt[s]) : -1;
    RSK_TRY(ctx->work[4].reserve((size_t)S * 4));
    RSK_HIP(hipMemcpyAsync(ctx->work[4].ptr, r.data(), (size_t)S * 4, hipMemcpyHostToDevice, ctx->stream));
    {
        ScopedTimer tm(ctx, "random_select");
        select_free_kernel<<<(unsigned)ceil_div(S, 256), 256, 0, ctx->stream>>>(d_haz, N, S, npb, nch,
                                                                                ctx->work[2].as<int>(),
                                                                                ctx->work[4].as<int>(), d_out);
        RSK_HIP(hipGetLastError());
    }
    if (!dev) {
        RSK_TRY(copy_back(ctx, out_node, d_out, (size_t)S * 4, false));
    }
    RSK_HIP(hipStreamSynchronize(ctx->stream));  // r[] lives on this host stack frame
    if (!dev)
        for (int s = 0; s < S; ++s)
            if (out_node[s] == RSK_TARGET_NO_CANDIDATE) return RSK_NO_CANDIDATE;
    return RSK_OK;
}

// rec_limit >= 0 (rsk_selftest_write_guard only): nr_place's record capacity
// lowered to it, so its write guard must fire
static int node_reduce_impl(rsk_ctx *ctx, const int32_t *assign, int32_t P, int32_t S, const int32_t *pod_cpu,
                            const int64_t *pod_mem, int32_t N, int32_t *pod_count, int64_t *cpu_sum, int64_t *mem_sum,
                            uint32_t flags, int64_t rec_limit) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(P >= 0 && S > 0 && N > 0 && (int64_t)N * S < INT32_MAX, "bad sizes");
    RSK_CHECK(pod_count && cpu_sum && pod_cpu && (!mem_sum || pod_mem), "null argument");
    const bool dev = flags & RSK_F_DEVICE;
    const size_t PS = (size_t)P * S, NS = (size_t)N * S;
    const int *d_assign, *d_cpu;
    const int64_t *d_mem = nullptr;
    int *d_cnt;
    int64_t *d_cs, *d_ms = nullptr;
    RSK_TRY(stage_in(ctx, 0, assign, PS * 4, dev, reinterpret_cast<const void **>(&d_assign)));
    RSK_TRY(stage_in(ctx, 1, pod_cpu, (size_t)P * 4, dev, reinterpret_cast<const void **>(&d_cpu)));
    if (mem_sum) RSK_TRY(stage_in(ctx, 2, pod_mem, (size_t)P * 8, dev, reinterpret_cast<const void **>(&d_mem)));
    RSK_TRY(stage_out(ctx, 3, pod_count, NS * 4, dev, reinterpret_cast<void **>(&d_cnt)));
    RSK_TRY(stage_out(ctx, 4, cpu_sum, NS * 8, dev, reinterpret_cast<void **>(&d_cs)));
    if (mem_sum) RSK_TRY(stage_out(ctx, 5, mem_sum, NS * 8, dev, reinterpret_cast<void **>(&d_ms)));
    RSK_TRY(ws_check_ptr(d_cs, "cpu_sum"));  // (u64 stores and atomics)
    if (d_ms) RSK_TRY(ws_check_ptr(d_ms, "mem_sum"));
    if (d_mem) RSK_TRY(ws_check_ptr(d_mem, "pod_mem"));
    const int nbk = (int)ceil_div(N, kNrBucketNodes), nchunk = (int)ceil_div(S, 64);
    const int64_t nh = (int64_t)nbk * (1 + nchunk);  // a block's counters: key buckets + entry bins
    // the deviation form while its counters and records have 32-bit offsets
    // (larger batches take the atomic form below, which handles any size)
    const int nblk = (int)ceil_div(P, kNrPods);
    const int64_t ncnt = nh * nblk;
    const size_t ecap = ((size_t)kNrPods * S / kNrEntDiv + 64) & ~(size_t)63;  // a block's entry region (8 waves')
    const int64_t nrec = (int64_t)P + 2 * (int64_t)nblk * (int64_t)ecap;  // pod records + 2 per entry
    unsigned *derr = dev_err(ctx);
    if (PS && S >= 32 && S <= kNrMaxS && nh <= kNrMaxCounters && ncnt < INT32_MAX / 2 && nrec < INT32_MAX && derr) {
        const size_t kb = ((size_t)P * 4 + 15) & ~(size_t)15;
        RSK_TRY(ctx->work[0].reserve(kb + (size_t)nrec * 16));  // keys, then the records
        RSK_TRY(ctx->work[1].reserve(((size_t)ncnt + 2 * (size_t)nh + 1 + (size_t)nblk * (kNrThreads / 64)) * 4));
        RSK_TRY(ctx->work[2].reserve((size_t)nblk * ecap * 8));
        int *pkey = ctx->work[0].as<int>();
        int4 *rec = reinterpret_cast<int4 *>(ctx->work[0].as<char>() + kb);
        int *bh = ctx->work[1].as<int>(), *tot = bh + ncnt, *base = tot + nh, *ecount = base + nh + 1;
        int2 *ent = ctx->work[2].as<int2>();
        auto *ucs = reinterpret_cast<unsigned long long *>(d_cs), *ums = reinterpret_cast<unsigned long long *>(d_ms);
        const auto *lmem = reinterpret_cast<const long long *>(d_mem);
        ScopedTimer tm(ctx, "node_reduce");
        const bool o32 = PS * 4 < ((size_t)1 << 32), maj = S >= 43;
        auto *sc = o32 ? (maj ? &nr_scan_kernel<true, true> : &nr_scan_kernel<true, false>)
                       : (maj ? &nr_scan_kernel<false, true> : &nr_scan_kernel<false, false>);
        const unsigned g8 = (unsigned)(8 * ceil_div(nblk, 8));  // (nr_block: XCD runs of consecutive blocks)
        // dynamic LDS above 64 KiB needs the attribute (nh = 16384 counters: 64 KiB + the static word)
        const size_t scan_lds = (size_t)nh * 4, pl = (size_t)nh * 4 + 8 + (size_t)kNrPods * (d_ms ? 16 : 8);
        RSK_CHECK(scan_lds + 64 <= 160 * 1024 && pl + 64 <= 160 * 1024, "node_reduce: %zu / %zu B of LDS", scan_lds, pl);
        auto *pk = d_ms ? &nr_place_kernel<true> : &nr_place_kernel<false>;
        if (scan_lds + 64 > 64 * 1024)
            RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(sc), hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)scan_lds));
        if (pl + 64 > 64 * 1024)
            RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(pk), hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)pl));
        sc<<<g8, kNrThreads, scan_lds, ctx->stream>>>(d_assign, P, S, N, nbk, nchunk, nblk, ecap, pkey, bh, ent,
                                                      ecount);
        auto *cs = nblk <= 64 * 8 ? &nr_colscan_kernel<8>
                   : nblk <= 64 * 16 ? &nr_colscan_kernel<16> : &nr_colscan_kernel<0>;
        cs<<<(unsigned)ceil_div(nh, 4), 256, 0, ctx->stream>>>(bh, (int)nh, nblk, tot);
        pk<<<g8, kNrThreads, pl, ctx->stream>>>(pkey, P, N, nbk, nchunk, nblk, bh, tot, base, d_cpu, lmem, ent, ecap,
                                                ecount, rec, (int)(rec_limit >= 0 ? std::min(nrec, rec_limit) : nrec),
                                                derr);
        auto *sk = d_ms ? &nr_sum_kernel<true> : &nr_sum_kernel<false>;
        sk<<<(unsigned)(nbk * nchunk), kNrSumThreads, 0, ctx->stream>>>(base, nbk, nchunk, rec, N, S, d_cnt, ucs, ums);
        auto *xk = d_ms ? &nr_spill_kernel<true> : &nr_spill_kernel<false>;
        xk<<<g8, kNrThreads, 0, ctx->stream>>>(d_assign, P, S, N, nblk, pkey, ecount, d_cpu, lmem, d_cnt, ucs, ums);
        RSK_HIP(hipGetLastError());
    } else {
        ScopedTimer tm(ctx, "node_reduce");
        RSK_HIP(hipMemsetAsync(d_cnt, 0, NS * 4, ctx->stream));
        RSK_HIP(hipMemsetAsync(d_cs, 0, NS * 8, ctx->stream));
        if (d_ms) RSK_HIP(hipMemsetAsync(d_ms, 0, NS * 8, ctx->stream));
        if (PS)
            node_reduce_kernel<<<(unsigned)ceil_div(PS, 256), 256, 0, ctx->stream>>>(
                d_assign, P, S, d_cpu, reinterpret_cast<const long long *>(d_mem), N, d_cnt,
                reinterpret_cast<unsigned long long *>(d_cs), reinterpret_cast<unsigned long long *>(d_ms));
        RSK_HIP(hipGetLastError());
    }
    if (!dev) {
        RSK_TRY(copy_back(ctx, pod_count, d_cnt, NS * 4, false));
        RSK_TRY(copy_back(ctx, cpu_sum, d_cs, NS * 8, false));
        if (mem_sum) RSK_TRY(copy_back(ctx, mem_sum, d_ms, NS * 8, false));
        RSK_HIP(hipStreamSynchronize(ctx->stream));
        RSK_TRY(check_dev_err(ctx));
    }
    return RSK_OK;
}

int rsk_node_reduce(rsk_ctx *ctx, const int32_t *assign, int32_t P, int32_t S, const int32_t *pod_cpu,
                    const int64_t *pod_mem, int32_t N, int32_t *pod_count, int64_t *cpu_sum, int64_t *mem_sum,
                    uint32_t flags) {
    return node_reduce_impl(ctx, assign, P, S, pod_cpu, pod_mem, N, pod_count, cpu_sum, mem_sum, flags, -1);
}

int rsk_selftest_write_guard(rsk_ctx *ctx) {
    RSK_TRY(activate(ctx));
    constexpr int P = 4096, S = 64, N = 64;
    std::vector<int32_t> a((size_t)P * S), cpu(P, 1);
    for (int p = 0; p < P; ++p)
        for (int s = 0; s < S; ++s) a[(size_t)p * S + s] = (p + (s == 7 && p % 5 == 0)) % N;
    int32_t *d = nullptr;
    const size_t ab = (size_t)P * S * 4, ob = (size_t)N * S * 4;
    RSK_HIP(hipMalloc(&d, ab + (size_t)P * 4 + ob + 2 * ob));
    int32_t *dc = d + (size_t)P * S, *dn = dc + P;
    int64_t *ds = reinterpret_cast<int64_t *>(dn + (size_t)N * S);
    int rc = hipMemcpy(d, a.data(), ab, hipMemcpyHostToDevice) == hipSuccess &&
                     hipMemcpy(dc, cpu.data(), (size_t)P * 4, hipMemcpyHostToDevice) == hipSuccess
                 ? RSK_OK
                 : RSK_EHIP;
    if (rc == RSK_OK)  // 1,000 records for 4,096 pods: nr_place must skip the rest and raise the word
        rc = node_reduce_impl(ctx, d, P, S, dc, nullptr, N, dn, ds, nullptr, RSK_F_DEVICE, 1000);
    if (rc == RSK_OK) rc = hipStreamSynchronize(ctx->stream) == hipSuccess ? check_dev_err(ctx) : RSK_EHIP;
    (void)hipFree(d);
    if (rc == RSK_OK) {
        set_error("rsk_selftest_write_guard: the nr_place guard did not fire");
        return RSK_EINVAL;
    }
    return rc;  // RSK_EHIP naming nr_place: the guard works
}

int rsk_cpu_pct(rsk_ctx *ctx, const int32_t *use_cpu, const int32_t *cap_cpu, int32_t N, int32_t S, int32_t *out_pct,
                uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(N > 0 && S > 0 && (int64_t)N * S < INT32_MAX && out_pct, "bad arguments");
    const bool dev = flags & RSK_F_DEVICE;
    const size_t NS = (size_t)N * S;
    const int *d_use, *d_cap;
    int *d_out;
    RSK_TRY(stage_in(ctx, 0, use_cpu, NS * 4, dev, reinterpret_cast<const void **>(&d_use)));
    RSK_TRY(stage_in(ctx, 1, cap_cpu, (size_t)N * 4, dev, reinterpret_cast<const void **>(&d_cap)));
    RSK_TRY(stage_out(ctx, 2, out_pct, NS * 4, dev, reinterpret_cast<void **>(&d_out)));
    {
        ScopedTimer tm(ctx, "cpu_pct");
        RSK_TRY(launch_cpu_pct(ctx->stream, d_use, d_cap, N, S, d_out));
    }
    if (!dev) {
        RSK_TRY(copy_back(ctx, out_pct, d_out, NS * 4, false));
        RSK_HIP(hipStreamSynchronize(ctx->stream));
    }
    return RSK_OK;
}

int rsk_detect(rsk_ctx *ctx, const int32_t *cpu_pct, int32_t N, int32_t S, int32_t threshold, uint8_t *out_hazard,
               int32_t *out_most, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(N > 0 && S > 0 && (int64_t)N * S < INT32_MAX && out_hazard && out_most, "bad arguments");
    const bool dev = flags & RSK_F_DEVICE;
    const size_t NS = (size_t)N * S;
    const int *d_pct;
    uint8_t *d_haz;
    int *d_most;
    RSK_TRY(stage_in(ctx, 0, cpu_pct, NS * 4, dev, reinterpret_cast<const void **>(&d_pct)));
    RSK_TRY(stage_out(ctx, 1, out_hazard, NS, dev, reinterpret_cast<void **>(&d_haz)));
    RSK_TRY(stage_out(ctx, 2, out_most, (size_t)S * 4, dev, reinterpret_cast<void **>(&d_most)));
    RSK_TRY(ctx->work[0].reserve((size_t)S * 8));
    {
        ScopedTimer tm(ctx, "detect");
        RSK_TRY(launch_detect(ctx->stream, d_pct, N, S, threshold, d_haz, ctx->work[0].as<unsigned long long>(),
                              d_most));
    }
    if (!dev) {
        RSK_TRY(copy_back(ctx, out_hazard, d_haz, NS, false));
        RSK_TRY(copy_back(ctx, out_most, d_most, (size_t)S * 4, false));
        RSK_HIP(hipStreamSynchronize(ctx->stream));
    }
    return RSK_OK;
}

int rsk_load_std(rsk_ctx *ctx, const int32_t *use_cpu, const int32_t *cap_cpu, int32_t N, int32_t S,
                 double *out_std, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(N > 0 && S > 0 && (int64_t)N * S < INT32_MAX && out_std, "bad arguments");
    const bool dev = flags & RSK_F_DEVICE;
    const size_t NS = (size_t)N * S;
    const int *d_use, *d_cap;
    double *d_out;
    RSK_TRY(stage_in(ctx, 0, use_cpu, NS * 4, dev, reinterpret_cast<const void **>(&d_use)));
    RSK_TRY(stage_in(ctx, 1, cap_cpu, (size_t)N * 4, dev, reinterpret_cast<const void **>(&d_cap)));
    RSK_TRY(stage_out(ctx, 2, out_std, (size_t)S * 8, dev, reinterpret_cast<void **>(&d_out)));
    // nodes per thread: at least RSK_STD_MIN (two batches of loads), and at
    // most 2,048 partials for the merge workgroups to walk (a folding
    // workgroup writes one partial per 256 / S chunks).  50k nodes x 64
    // scenarios: 16 nodes, 3,125 chunks, 782 partials — 14.3 us for the two
    // launches against 17.5 at 8 or 4 nodes (more partials to merge, no
    // faster partial pass) and 15.6 at 25 nodes / 500 partials (r06w, r06k)
#ifndef RSK_STD_MIN
#define RSK_STD_MIN 16
#endif
    const int fold = 256 % S == 0 && S < 256;  // a workgroup holds 256 / S whole chunks
    const int64_t max_chunks = 2048 * (fold ? 256 / S : 1);
    const int npb = std::max({chunk_for(N, S), RSK_STD_MIN, (int)ceil_div(N, max_chunks)});
    const int nch = (int)ceil_div(N, npb);
    RSK_TRY(ctx->work[0].reserve((size_t)nch * S * 8));
    RSK_TRY(ctx->work[1].reserve((size_t)nch * S * 8));
    RSK_TRY(ctx->work[2].reserve((size_t)nch * S * 4));
    const unsigned total = (unsigned)((int64_t)nch * S);
    const unsigned grid = (unsigned)ceil_div(total, 256);
    {
        ScopedTimer tm(ctx, "load_std");
        std_partial_kernel<<<grid, 256, 0, ctx->stream>>>(d_use, d_cap, N, S, npb, total, fold,
                                                          ctx->work[0].as<double>(), ctx->work[1].as<double>(),
                                                          ctx->work[2].as<int>());
        std_merge_kernel<<<(unsigned)S, 256, 0, ctx->stream>>>(ctx->work[0].as<double>(), ctx->work[1].as<double>(),
                                                               ctx->work[2].as<int>(), fold ? (int)grid : nch, S,
                                                               d_out);
        RSK_HIP(hipGetLastError());
    }
    if (!dev) {
        RSK_TRY(copy_back(ctx, out_std, d_out, (size_t)S * 8, false));
        RSK_HIP(hipStreamSynchronize(ctx->stream));
    }
    return RSK_OK;
}

int rsk_cut_cost(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, int32_t P, const int32_t *assign,
                 int32_t S, const int32_t *missing, int64_t *out_directed, uint32_t flags) {
    return rsk_cut_cost_rows(ctx, row_ptr, col_idx, P, 0, P, assign, S, missing, out_directed, flags);
}

int rsk_cut_cost_rows(rsk_ctx *ctx, const int32_t *row_ptr, const int32_t *col_idx, int32_t P, int32_t r0,
                      int32_t r1, const int32_t *assign, int32_t S, const int32_t *missing, int64_t *out_directed,
                      uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(P >= 0 && S > 0 && row_ptr && out_directed && 0 <= r0 && r0 <= r1 && r1 <= P, "bad arguments");
    const bool dev = flags & RSK_F_DEVICE;
    const int64_t nnz = dev ? 0 : row_ptr[P];  // device pointers pass through unstaged
    const int *d_rp, *d_col, *d_assign, *d_miss = nullptr;
    int64_t *d_out;
    RSK_TRY(stage_in(ctx, 0, row_ptr, (size_t)(P + 1) * 4, dev, reinterpret_cast<const void **>(&d_rp)));
    RSK_TRY(stage_in(ctx, 1, col_idx, (size_t)nnz * 4, dev, reinterpret_cast<const void **>(&d_col)));
    RSK_TRY(stage_in(ctx, 2, assign, (size_t)P * S * 4, dev, reinterpret_cast<const void **>(&d_assign)));
    if (missing) RSK_TRY(stage_in(ctx, 3, missing, (size_t)P * 4, dev, reinterpret_cast<const void **>(&d_miss)));
    RSK_TRY(stage_out(ctx, 4, out_directed, (size_t)S * 8, dev, reinterpret_cast<void **>(&d_out)));
    RSK_HIP(hipMemsetAsync(d_out, 0, (size_t)S * 8, ctx->stream));
    if (r1 > r0) {
        const int Q = r1 - r0;
        // rows per thread: each row is a dependent row_ptr -> col -> assign chain,
        // so keep ~64k workgroups of (row chunk, scenario) pairs in flight
        const int ppt = (int)std::max<int64_t>(1, ceil_div((int64_t)Q * S, (int64_t)256 * 65536));
        const int64_t tot = ceil_div(Q, ppt) * S;
        RSK_CHECK(tot < INT32_MAX, "grid too large");
        RSK_TRY(ctx->work[4].reserve((size_t)kCutBins * S * 8));
        auto *bins = ctx->work[4].as<unsigned long long>();
        RSK_HIP(hipMemsetAsync(bins, 0, (size_t)kCutBins * S * 8, ctx->stream));
        ScopedTimer tm(ctx, "cut_cost");
        if (S >= 32) {  // lane = scenario, edge-balanced (nnz may be device-resident: grid-stride)
            const int nw = 4096;  // waves per 64-scenario chunk
            const int64_t waves = ceil_div(S, 64) * nw;
            RSK_CHECK(ceil_div(waves, 4) < INT32_MAX, "grid too large");
            cut_cost_wave_kernel<<<(unsigned)ceil_div(waves, 4), 256, 0, ctx->stream>>>(d_rp, d_col, r0, r1, d_assign, S,
                                                                                      d_miss, nw, bins);
        } else {
            cut_cost_kernel<<<(unsigned)ceil_div(tot, 256), 256, 0, ctx->stream>>>(d_rp, d_col, r0, r1, d_assign, S,
                                                                                  d_miss, ppt, (unsigned)tot, bins);
        }
        RSK_HIP(hipGetLastError());
        cut_bins_sum<<<(unsigned)ceil_div(S, 256), 256, 0, ctx->stream>>>(bins, S,
                                                                           reinterpret_cast<unsigned long long *>(d_out));
        RSK_HIP(hipGetLastError());
    }
    if (!dev) {
        RSK_TRY(copy_back(ctx, out_directed, d_out, (size_t)S * 8, false));
        RSK_HIP(hipStreamSynchronize(ctx->stream));
    }
    return RSK_OK;
}

int rsk_pick_max_pod(rsk_ctx *ctx, const int32_t *assign, const int32_t *pod_cpu, int32_t P, int32_t S,
                     const int32_t *most, int32_t *out_pod, uint32_t flags) {
    RSK_TRY(activate(ctx));
    RSK_CHECK(P >= 0 && S > 0 && most && out_pod, "bad arguments");
    const bool dev = flags & RSK_F_DEVICE;
    const int *d_assign, *d_cpu, *d_most;
    int *d_out;
    RSK_TRY(stage_in(ctx, 0, assign, (size_t)P * S * 4, dev, reinterpret_cast<const void **>(&d_assign)));
    RSK_TRY(stage_in(ctx, 1, pod_cpu, (size_t)P * 4, dev, reinterpret_cast<const void **>(&d_cpu)));
    RSK_TRY(stage_in(ctx, 2, most, (size_t)S * 4, dev, reinterpret_cast<const void **>(&d_most)));
    RSK_TRY(stage_out(ctx, 3, out_pod, (size_t)S * 4, dev, reinterpret_cast<void **>(&d_out)));
    RSK_TRY(ctx->work[0].reserve((size_t)S * 8));
    {
        ScopedTimer tm(ctx, "pick_max_pod");
        RSK_TRY(launch_pick_max_pod(ctx->stream, d_assign, d_cpu, P, S, d_most, ctx->work[0].as<unsigned long long>(),
                                    d_out));
    }
    if (!dev) {
        RSK_TRY(copy_back(ctx, out_pod, d_out, (size_t)S * 4, false));
        RSK_HIP(hipStreamSynchronize(ctx->stream));
    }
    return RSK_OK;
}

}  // extern "C"
