// rsk_hub16.hip — CAR for the hub rows of the compact path (N <= 65535): rows
// above the mid classes (degree 65..kHubMax), in three launches by degree
// (65..128, 129..256, 257..kHubMax).
//
// Reference: the score loop + argmax of `communication`,
// rescheduling.py:183-214 (see rsk_car.hip for the full statement).
//
// Work item = (row, group of G = 2^lg scenarios) with d * G <= 4096, one
// workgroup of kHW waves:
//   stage   the G x d cells (code << 16 | node) in LDS, every thread up to kHB
//           (neighbour, scenario) elements with all loads in flight: neighbour
//           id (plan) -> assign word -> 16-bit code gather (an assignment
//           outside [0, N) reads the zero code row N: never a candidate);
//   count   one wave per scenario, lanes = neighbours: counters in the wave's
//           LDS table — direct and node-indexed (u8 for degree <= 255, else
//           u16) or an open-addressing hash of (node + 1) << 16 | count words,
//           whichever is smaller for the launch;
//   decide  one u64 DPP max over (count, code, -node) gives the best node; a
//           ballot tells whether another node reaches the same count (a tie:
//           the best code decides, None when it is code 1 = rem < 0) and
//           whether it shares an inexact code (rare: exact cap - use).
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "rsk_car.h"

namespace rsk {

constexpr int kHW = 4;      // waves per workgroup
constexpr int kHT = 64 * kHW;
constexpr int kHB = 16;     // staging elements in flight per thread
constexpr int kHStage = kHT * kHB;  // cells per work item (d * G <= kHStage)

enum { kTabU8 = 0, kTabU16 = 1, kTabHash = 2 };

// A wave's count table for one scenario.  Every call takes the entry's
// candidate flag and is branch-free for the lanes without one (they touch word
// 0 of a direct table with a zero increment, or the hash table's sink word H),
// so the compiler emits no exec-mask branches around the LDS traffic.
template <int kTab>
struct HubTab16 {
    unsigned *w;
    unsigned mask;  // hash: slots - 1 (the sink word H = mask + 1 follows)
    int shift;      // hash: 32 - log2(slots)
    __device__ __forceinline__ unsigned home(unsigned k) const { return (k * 2654435761u) >> shift; }
    __device__ __forceinline__ void add(int n, bool cand) const {
        if (kTab == kTabU8) {
            atomicAdd(&w[cand ? n >> 2 : 0], cand ? 1u << ((n & 3) * 8) : 0u);
        } else if (kTab == kTabU16) {
            atomicAdd(&w[cand ? n >> 1 : 0], cand ? 1u << ((n & 1) * 16) : 0u);
        } else {
            // first probe: claim the home slot, or add 1 to it when it holds
            // the key (0 otherwise); collided lanes walk the chain
            const unsigned k = (unsigned)n + 1u;
            unsigned h = cand ? home(k) : mask + 1u;
            unsigned prev = atomicCAS(&w[h], 0u, (k << 16) | 1u);
            bool hit = cand && prev != 0u && (prev >> 16) == k;
            atomicAdd(&w[h], hit ? 1u : 0u);
            bool more = cand && prev != 0u && !hit;
            if (__builtin_amdgcn_ballot_w64(more)) {
                while (more) {
                    h = (h + 1u) & mask;
                    prev = atomicCAS(&w[h], 0u, (k << 16) | 1u);
                    hit = prev != 0u && (prev >> 16) == k;
                    if (hit) atomicAdd(&w[h], 1u);
                    more = prev != 0u && !hit;
                }
            }
        }
    }
    __device__ __forceinline__ int get(int n, bool cand) const {  // 0 when !cand
        unsigned v;
        if (kTab == kTabU8) {
            v = (w[cand ? n >> 2 : 0] >> ((n & 3) * 8)) & 0xffu;
        } else if (kTab == kTabU16) {
            v = (w[cand ? n >> 1 : 0] >> ((n & 1) * 16)) & 0xffffu;
        } else {
            const unsigned k = (unsigned)n + 1u;
            unsigned h = cand ? home(k) : mask + 1u;
            unsigned x = w[h];
            bool miss = cand && (x >> 16) != k;
            if (__builtin_amdgcn_ballot_w64(miss)) {
                while (miss) {
                    h = (h + 1u) & mask;
                    x = w[h];
                    miss = (x >> 16) != k;
                }
            }
            v = x & 0xffffu;
        }
        return cand ? (int)v : 0;
    }
    // direct tables: zero the counter word of n (every other node in that
    // word is one of this scenario's entries, cleared too; word 0 gets zeroed
    // by the lanes without a candidate); hash: the caller wipes the table
    __device__ __forceinline__ void clear(int n, bool cand) const {
        if (kTab == kTabU8) w[cand ? n >> 2 : 0] = 0u;
        else if (kTab == kTabU16) w[cand ? n >> 1 : 0] = 0u;
    }
};

__device__ __forceinline__ unsigned dpp_max_u32(unsigned v) {  // identity 0
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

// Running best (count, code, -node) key over a lane's entries (count 0 = not
// a candidate).
struct HubDecide {
    unsigned long long best;
    __device__ __forceinline__ void init() { best = 0ull; }
    __device__ __forceinline__ void put(unsigned x, int cnt) {
        const unsigned long long k = cnt ? ((unsigned long long)cnt << 32) | (unsigned long long)cell_cand(x) : 0ull;
        best = k > best ? k : best;
    }
};

// Rare path: among the entries at count M with the inexact code bk, the node
// with the largest exact remaining CPU, then the lower index.  Reads counts,
// so it runs before the table is cleared.
template <int kTab>
__device__ __forceinline__ int hub16_exact(const Hub16Args &a, const HubTab16<kTab> &tb, const unsigned *cs, int d,
                                           int M, unsigned bk, int s, int lane) {
    unsigned long long kx = 0ull;
    for (int j = lane; j < d; j += 64) {
        const unsigned x = cs[j];
        if (cell_code(x) == bk && tb.get(cell_node(x), true) == M) {
            const int nd = cell_node(x);
            const int rem = a.cap[nd] - ld32(a.use, (unsigned)nd * (unsigned)a.S + (unsigned)s);
            const unsigned long long k = pack_rn(rem, nd);
            kx = k > kx ? k : kx;
        }
    }
    kx = dpp_max_u64(kx);
    return (int)(kNodeMask - (unsigned)(kx & kNodeMask));
}

// Output of one scenario from its reduced state (rescheduling.py:199-214).
__device__ __forceinline__ void hub16_emit(const Hub16Args &a, int oi, int s, int M, unsigned bw, bool any_tie,
                                           bool any_amb, int ex) {
    const unsigned bk = cell_code(bw);
    int t, sc = 0;
    if (M == 0) {
        t = zero_target(load_zc(a.zc_cnt, a.zc_key, s), sc);
    } else {
        sc = M;
        t = !any_tie ? cand_node(bw) : (bk >= 2u ? cand_node(bw) : RSK_TARGET_NONE);
        if (any_tie && any_amb && code_inexact(bk)) t = ex;
    }
    const size_t o = (size_t)oi * (unsigned)a.S + (unsigned)s;
    a.out_target[o] = t;
    if (a.out_score) a.out_score[o] = sc;
}

template <int kTab>
__device__ __forceinline__ void tab_wipe(const HubTab16<kTab> &tb, int H, int lane) {
    if (kTab == kTabHash) {  // a probe may pass any slot: wipe the whole table
        uint4 *w4 = reinterpret_cast<uint4 *>(tb.w);
        for (int k = lane; k <= (H >> 2); k += 64) w4[k] = make_uint4(0u, 0u, 0u, 0u);  // + the sink
    }
}

// NS scenarios of a row of degree d <= 64 * NJ at once (independent chains
// the scheduler interleaves): entries and their counts in registers, one
// table per scenario.  cs[k] = the staged cells of scenario k (null: none).
template <int kTab, int NJ, int NS>
__device__ __forceinline__ void hub16_multi(const Hub16Args &a, const HubTab16<kTab> (&tb)[NS],
                                            const unsigned *const (&cs)[NS], int d, int oi, int s0, int lane) {
    unsigned x[NS][NJ];
    int c[NS][NJ];
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int i = 0; i < NJ; ++i) {
            const int j = i * 64 + lane;
            x[k][i] = cs[k] ? cs[k][min(j, d - 1)] : kCellPad;
            if (j >= d) x[k][i] = kCellPad;
        }
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int i = 0; i < NJ; ++i) tb[k].add(cell_node(x[k][i]), cell_code(x[k][i]) != kCodeHaz);
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int i = 0; i < NJ; ++i) c[k][i] = tb[k].get(cell_node(x[k][i]), cell_code(x[k][i]) != kCodeHaz);
    // the maximal count, then the best (code, -node) word at it: two 32-bit DPP maxima
    int M[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        int m = 0;
#pragma unroll
        for (int i = 0; i < NJ; ++i) m = max(m, c[k][i]);
        M[k] = dpp_max(m);
    }
    unsigned bw[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        unsigned v = 0u;
#pragma unroll
        for (int i = 0; i < NJ; ++i) v = max(v, c[k][i] == M[k] && M[k] > 0 ? cell_cand(x[k][i]) : 0u);
        bw[k] = dpp_max_u32(v);
    }
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        const int bn = cand_node(bw[k]);
        const unsigned bk = cell_code(bw[k]);
        bool tie = false, amb = false;
#pragma unroll
        for (int i = 0; i < NJ; ++i) {
            const bool o = c[k][i] == M[k] && M[k] > 0 && cell_node(x[k][i]) != bn;
            tie = tie || o;
            amb = amb || (o && cell_code(x[k][i]) == bk);
        }
        const bool any_tie = __builtin_amdgcn_ballot_w64(tie) != 0ull;
        const bool any_amb = __builtin_amdgcn_ballot_w64(amb) != 0ull;
        int ex = -1;
        if (any_tie && any_amb && code_inexact(bk)) ex = hub16_exact<kTab>(a, tb[k], cs[k], d, M[k], bk, s0 + k, lane);
        if (lane == k && cs[k]) hub16_emit(a, oi, s0 + k, M[k], bw[k], any_tie, any_amb, ex);
    }
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        if (kTab != kTabHash) {
#pragma unroll
            for (int i = 0; i < NJ; ++i) tb[k].clear(cell_node(x[k][i]), cell_code(x[k][i]) != kCodeHaz);
        }
        tab_wipe<kTab>(tb[k], a.H, lane);
    }
}

// One scenario of a row of any degree: entries re-read from the staged cells.
template <int kTab>
__device__ __forceinline__ void hub16_scenario(const Hub16Args &a, const HubTab16<kTab> &tb, const unsigned *cs, int d,
                                               int oi, int s, int lane) {
    for (int j = lane; j < d; j += 64) {
        const unsigned x = cs[j];
        tb.add(cell_node(x), cell_code(x) != kCodeHaz);
    }
    HubDecide h;
    h.init();
    for (int j = lane; j < d; j += 64) {
        const unsigned x = cs[j];
        h.put(x, tb.get(cell_node(x), cell_code(x) != kCodeHaz));
    }
    const unsigned long long best = dpp_max_u64(h.best);
    const int M = (int)(best >> 32);
    const unsigned bw = (unsigned)best;
    const int bn = cand_node(bw);
    const unsigned bk = cell_code(bw);
    bool tie = false, amb = false;
    if (M > 0) {
        for (int j = lane; j < d; j += 64) {
            const unsigned x = cs[j];
            if (cell_code(x) != kCodeHaz && cell_node(x) != bn && tb.get(cell_node(x), true) == M) {
                tie = true;
                amb = amb || cell_code(x) == bk;
            }
        }
    }
    const bool any_tie = __builtin_amdgcn_ballot_w64(tie) != 0ull;
    const bool any_amb = __builtin_amdgcn_ballot_w64(amb) != 0ull;
    int ex = -1;
    if (any_tie && any_amb && code_inexact(bk)) ex = hub16_exact<kTab>(a, tb, cs, d, M, bk, s, lane);
    if (kTab != kTabHash) {
        for (int j = lane; j < d; j += 64) {
            const unsigned x = cs[j];
            tb.clear(cell_node(x), cell_code(x) != kCodeHaz);
        }
    }
    tab_wipe<kTab>(tb, a.H, lane);
    if (lane == 0) hub16_emit(a, oi, s, M, bw, any_tie, any_amb, ex);
}

// One scenario of a long row by the whole workgroup (NJ < 0, "team"): the
// entries spread over all kHT threads and ONE table, the maxima and flags
// combined across the waves through LDS (red: 16 ints + 4 u64).  A wave
// alone would walk d / 64 entries per lane four times over; config 4's
// 1,025..1,756-neighbour rows with only 64 scenarios left most waves idle.
template <int kTab>
__device__ __forceinline__ void hub16_team(const Hub16Args &a, const HubTab16<kTab> &tb, const unsigned *cs, int d,
                                           int oi, int s, int tid, int lane, int wave, int *red) {
    for (int j = tid; j < d; j += kHT) tb.add(cell_node(cs[j]), cell_code(cs[j]) != kCodeHaz);
    __syncthreads();
    int m = 0;
    for (int j = tid; j < d; j += kHT) m = max(m, tb.get(cell_node(cs[j]), cell_code(cs[j]) != kCodeHaz));
    m = dpp_max(m);
    if (lane == 0) red[wave] = m;
    __syncthreads();
    int M = red[0];
#pragma unroll
    for (int w = 1; w < kHW; ++w) M = max(M, red[w]);
    unsigned v = 0u;
    if (M > 0)
        for (int j = tid; j < d; j += kHT) {
            const unsigned x = cs[j];
            v = max(v, tb.get(cell_node(x), cell_code(x) != kCodeHaz) == M ? cell_cand(x) : 0u);
        }
    v = dpp_max_u32(v);
    if (lane == 0) red[kHW + wave] = (int)v;
    __syncthreads();
    unsigned bw = (unsigned)red[kHW];
#pragma unroll
    for (int w = 1; w < kHW; ++w) bw = max(bw, (unsigned)red[kHW + w]);
    const int bn = cand_node(bw);
    const unsigned bk = cell_code(bw);
    bool tie = false, amb = false;
    if (M > 0)
        for (int j = tid; j < d; j += kHT) {
            const unsigned x = cs[j];
            if (cell_code(x) != kCodeHaz && cell_node(x) != bn && tb.get(cell_node(x), true) == M) {
                tie = true;
                amb = amb || cell_code(x) == bk;
            }
        }
    const int fl = (__builtin_amdgcn_ballot_w64(tie) != 0ull ? 1 : 0) | (__builtin_amdgcn_ballot_w64(amb) != 0ull ? 2 : 0);
    if (lane == 0) red[2 * kHW + wave] = fl;
    __syncthreads();
    int f = 0;
#pragma unroll
    for (int w = 0; w < kHW; ++w) f |= red[2 * kHW + w];
    const bool any_tie = f & 1, any_amb = f & 2;
    int ex = -1;
    if (any_tie && any_amb && code_inexact(bk)) {  // rare (workgroup-uniform): exact remaining CPU
        unsigned long long kx = 0ull;
        for (int j = tid; j < d; j += kHT) {
            const unsigned x = cs[j];
            if (cell_code(x) == bk && tb.get(cell_node(x), true) == M) {
                const int nd = cell_node(x);
                const int rem = a.cap[nd] - ld32(a.use, (unsigned)nd * (unsigned)a.S + (unsigned)s);
                const unsigned long long k = pack_rn(rem, nd);
                kx = k > kx ? k : kx;
            }
        }
        kx = dpp_max_u64(kx);
        unsigned long long *r64 = reinterpret_cast<unsigned long long *>(red + 4 * kHW);
        if (lane == 0) r64[wave] = kx;
        __syncthreads();
#pragma unroll
        for (int w = 0; w < kHW; ++w) kx = max(kx, r64[w]);
        ex = (int)(kNodeMask - (unsigned)(kx & kNodeMask));
    }
    __syncthreads();  // every lookup of this scenario done: clear
    if (kTab != kTabHash) {
        for (int j = tid; j < d; j += kHT) tb.clear(cell_node(cs[j]), cell_code(cs[j]) != kCodeHaz);
    } else {
        uint4 *w4 = reinterpret_cast<uint4 *>(tb.w);
        for (int k = tid; k <= (a.H >> 2); k += kHT) w4[k] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (tid == 0) hub16_emit(a, oi, s, M, bw, any_tie, any_amb, ex);
    __syncthreads();  // cleared before the next scenario's adds
}

template <int kTab, int NJ, int NS>
__global__ __launch_bounds__(kHT) void car_hub16_kernel(Hub16Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned hlds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const cint_ptr it = const_ptr(a.items) + (size_t)blockIdx.x * 4;
    const int oi = it[0], rb = it[1], d = it[2], gw = it[3];
    const int s0 = gw & 0xffffff, lg = gw >> 24;
    const int G = 1 << lg;
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    unsigned *col = hlds;  // [G][d], d * G <= a.stage <= kHStage
    HubTab16<kTab> tb[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
        tb[k].w = hlds + a.stage + (wave * NS + k) * (a.H + 4);
        tb[k].mask = (unsigned)a.H - 1u;
        tb[k].shift = a.hshift;
    }

    {   // stage: element e -> (neighbour j = e >> lg, scenario si = e & (G - 1)),
        // one batch, loads unconditional (clamped)
        const int total = d << lg;
        int e[kHB], n[kHB];
        unsigned c[kHB];
#pragma unroll
        for (int u = 0; u < kHB; ++u) {
            e[u] = min(u * kHT + tid, total - 1);
            n[u] = a.hcol[rb + (e[u] >> lg)];
        }
#pragma unroll
        for (int u = 0; u < kHB; ++u) {
            const unsigned s = min((unsigned)(s0 + (e[u] & (G - 1))), S - 1u);
            n[u] = a.assign[(size_t)n[u] * S + s];
        }
#pragma unroll
        for (int u = 0; u < kHB; ++u) {
            const unsigned s = min((unsigned)(s0 + (e[u] & (G - 1))), S - 1u);
            n[u] = (int)min((unsigned)n[u], N);
            c[u] = ld16(a.code, (unsigned)n[u] * S + s);
        }
#pragma unroll
        for (int u = 0; u < kHB; ++u)
            if (u * kHT + tid < total) col[(e[u] & (G - 1)) * d + (e[u] >> lg)] = (c[u] << 16) | (unsigned)n[u];
        // zero the tables (each wave's clears keep them zero between scenarios)
        uint4 *t4 = reinterpret_cast<uint4 *>(hlds + a.stage);
        constexpr int kTabs = NJ < 0 ? 1 : kHW * NS;
        for (int k = tid; k < (kTabs * (a.H + 4)) >> 2; k += kHT) t4[k] = make_uint4(0u, 0u, 0u, 0u);
    }
    __syncthreads();
    if constexpr (NJ < 0) {
        HubTab16<kTab> t1 = tb[0];
        t1.w = hlds + a.stage;
        int *red = reinterpret_cast<int *>(hlds + a.stage + a.H + 4);
        for (int si = 0; si < G && s0 + si < a.S; ++si)
            hub16_team<kTab>(a, t1, col + si * d, d, oi, s0 + si, tid, lane, wave, red);
    } else if constexpr (NJ > 0) {
        for (int sb = wave * NS; sb < G && s0 + sb < a.S; sb += kHW * NS) {
            const unsigned *cs[NS];
#pragma unroll
            for (int k = 0; k < NS; ++k) cs[k] = (sb + k < G && s0 + sb + k < a.S) ? col + (sb + k) * d : nullptr;
            hub16_multi<kTab, NJ, NS>(a, tb, cs, d, oi, s0 + sb, lane);
        }
    } else {
        for (int si = wave; si < G && s0 + si < a.S; si += kHW)
            hub16_scenario<kTab>(a, tb[0], col + si * d, d, oi, s0 + si, lane);
    }
}

Hub16Geom hub16_geometry(int dmax, int N) {
    Hub16Geom g;
    g.dmax = dmax;
    const int direct = dmax <= 255 ? (N + 3) / 4 : (N + 1) / 2;  // u8 / u16 counter words
    int H = 64;
    while (H < 2 * dmax) H <<= 1;
    static const int force = [] { const char *e = getenv("RSK_HUB16_TABLE"); return e ? atoi(e) : -1; }();
    // rows above 256 neighbours: one scenario at a time by the whole workgroup
    // (one table); RSK_HUB16_TEAM=0: one wave per scenario
    static const bool team_on = [] { const char *e = getenv("RSK_HUB16_TEAM"); return !e || atoi(e) != 0; }();
    const bool team = dmax > 256 && team_on;
    const int tables = team ? 1 : kHW;
    // direct tables (no probe chains, the fastest per scenario) while they fit
    // 48 KiB beside the staging area; the hash beyond (large N)
    const bool use_hash = force >= 0 ? force == kTabHash : (size_t)tables * (direct + 4) * 4 > 48 * 1024;
    if (use_hash) {
        g.tab = kTabHash;
        g.H = H;
        int l = 0;
        while ((1 << l) < H) ++l;
        g.hshift = 32 - l;
    } else {
        g.tab = dmax <= 255 ? kTabU8 : kTabU16;
        g.H = (direct + 3) & ~3;
        g.hshift = 0;
    }
    g.nj = team ? -1 : (dmax <= 128 ? 2 : (dmax <= 256 ? 4 : 0));
    static const int ns_env = [] { const char *e = getenv("RSK_HUB16_NS"); return e ? atoi(e) : 0; }();
    // scenarios per wave at once: 1 with direct tables (LDS-bound), 2 with the hash (measured)
    g.ns = g.nj <= 0 ? 1 : (ns_env == 1 || ns_env == 2 || ns_env == 4 ? ns_env : (use_hash ? 2 : 1));
    // tables: H words + sink / padding each; the team's reduction scratch after its one table
    g.lds = team ? ((size_t)kHStage + (g.H + 4) + 32) * 4 : ((size_t)kHStage + (size_t)kHW * g.ns * (g.H + 4)) * 4;
    return g;
}

int hub16_lg(int d, int S) {  // log2 of the scenario group of a degree-d row
    // staging cells per work item of the rows above 255 neighbours (the team
    // class): 2048 — smaller groups, more workgroups in flight (config 4
    // 0.273 -> 0.261 ms, config 3 within noise; RSK_HUB16_STAGE overrides,
    // RSK_HUB16_STAGE_ALL=1 applies it to every class)
    static const int cap = [] {
        const char *e = getenv("RSK_HUB16_STAGE");
        const int v = e ? atoi(e) : 2048;
        return v >= 256 && v <= kHStage ? v : kHStage;
    }();
    static const bool all = [] { const char *e = getenv("RSK_HUB16_STAGE_ALL"); return e && atoi(e) != 0; }();
    const int lim = (all || d > 255) ? std::max(cap, d) : kHStage;
    int lg = 0;
    while (lg < 6 && ((int64_t)d << (lg + 1)) <= lim && (1 << lg) < S) ++lg;
    return lg;
}

int launch_hub16(hipStream_t stream, const Hub16Args &a0, const Hub16Geom &g, int n_items) {
    if (n_items == 0) return RSK_OK;
    // the staging area sized to the launch's largest item (a.stage cells, set by
    // the caller from the items' d << lg; kHStage when unset): small scenario
    // groups leave room for more workgroups per CU
    Hub16Args a = a0;
    a.stage = a.stage > 0 ? std::min((a.stage + 3) & ~3, kHStage) : kHStage;
    const size_t lds = g.lds - (size_t)(kHStage - a.stage) * 4;
    RSK_CHECK(g.dmax <= kHStage, "hub row degree %d exceeds %d", g.dmax, kHStage);
    RSK_CHECK(lds <= 160 * 1024, "hub rows need %zu B of LDS", lds);
    using K = void (*)(Hub16Args);
#define RSK_HUB16_NS(T, J)                                                                           \
    (g.ns == 4 ? &car_hub16_kernel<T, J, 4> : g.ns == 2 ? &car_hub16_kernel<T, J, 2> : &car_hub16_kernel<T, J, 1>)
#define RSK_HUB16_NJ(T)                                                                                         \
    (g.nj == 2 ? RSK_HUB16_NS(T, 2) : g.nj == 4 ? RSK_HUB16_NS(T, 4) : g.nj < 0 ? &car_hub16_kernel<T, -1, 1> \
                                                                                : &car_hub16_kernel<T, 0, 1>)
    const K kern = g.tab == kTabU8 ? RSK_HUB16_NJ(kTabU8) : g.tab == kTabU16 ? RSK_HUB16_NJ(kTabU16) : RSK_HUB16_NJ(kTabHash);
#undef RSK_HUB16_NJ
#undef RSK_HUB16_NS
    if (lds > 64 * 1024)
        RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
    kern<<<dim3((unsigned)n_items), dim3(kHT), lds, stream>>>(a);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

}  // namespace rsk
