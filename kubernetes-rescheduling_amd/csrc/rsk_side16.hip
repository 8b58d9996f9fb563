// rsk_side16.hip — CAR for the side rows of the compact path (N <= 65535):
// every row above the tile classes (degree > light_max), any degree whose
// distinct-node table fits the LDS (side16_geometry).
//
// Reference: the score loop + argmax of `communication`,
// rescheduling.py:183-214 (see rsk_car.hip for the full statement).
//
// A work item is (row, chunk of 64 scenarios), lane = scenario, handled by a
// team of T waves (T = 1 for rows up to 256 neighbours: no barriers, the
// waves of a workgroup run independent items; T = 4 / 8 above, splitting the
// neighbour loads).  What-if scenarios share most of their assignment, so per
// neighbour j the team takes a pivot node p_j — the value most of the wave's
// lanes hold — and the row's histogram splits into a part every lane shares
// and a few per-lane deviations:
//   pass 1   the neighbours' assign rows (one 256-B row each, kB in flight):
//            the pivot of each entry, the lanes that deviate from it appended
//            to their own list (p_j << 16 | own node), the pivots counted in an
//            LDS hash keyed by node (one parallel insert per batch);
//   marks    each lane flags (a 64-bit lane mask per table slot) the pivot
//            nodes whose count differs in its scenario: the old and the new
//            node of each of its deviations;
//   levels   the distinct pivot nodes ordered by count, descending (counting
//            sort on min(count, 64));
//   walk     level by level, wave-uniform: the lane's code of node u (one
//            coalesced 128-B gather), a candidate unless hazard or flagged; the
//            two largest (count, code, -node) keys; stops once every lane's best
//            count exceeds every count left;
//   touched  each flagged / new node of the lane counted exactly (Hp + new -
//            old over the lane's own list), into the same two keys;
//   decide   as the tile scorers (rsk_car16.hip): count 0 -> the zero case, a
//            tie -> the larger code, None when it is code 1.
// Lanes whose deviation list overflowed, and ties between distinct nodes with
// the same inexact code, are recounted exactly, one scenario at a time by the
// whole wave (lanes = neighbours) — rare.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "rsk_car.h"

namespace rsk {

// The team's hash table: H words (node + 1) << 16 | count, and per slot the
// lanes whose count of that node differs from the pivot count.
struct SideTab {
    unsigned *tab;
    unsigned long long *umask;
    unsigned mask;
    int shift;
    __device__ __forceinline__ unsigned home(unsigned k) const { return (k * 2654435761u) >> shift; }
    // lane-parallel: key k (node + 1) gets +1 (claims a free slot or adds to its
    // own); true when this lane claimed the key's slot
    __device__ __forceinline__ bool add(unsigned k) const {
        unsigned h = home(k);
        while (true) {
            const unsigned prev = atomicCAS(&tab[h], 0u, (k << 16) | 1u);
            if (prev == 0u) return true;
            if ((prev >> 16) == k) { atomicAdd(&tab[h], 1u); return false; }
            h = (h + 1u) & mask;
        }
    }
    // slot of key k, -1 when absent (the table is at most 2/3 full: every chain ends)
    __device__ __forceinline__ int find(unsigned k) const {
        unsigned h = home(k);
        while (true) {
            const unsigned w = tab[h];
            if ((w >> 16) == k) return (int)h;
            if (w == 0u) return -1;
            h = (h + 1u) & mask;
        }
    }
};

// The wave's pivot for one neighbour: the node of the first lane or of the
// first lane that differs from it, whichever more lanes hold (any choice is
// exact; a majority keeps the deviations few).
__device__ __forceinline__ int side_pivot(int v) {
    const int c0 = __builtin_amdgcn_readfirstlane(v);
    const unsigned long long b0 = __builtin_amdgcn_ballot_w64(v == c0);
    const int n0 = __builtin_popcountll(b0);
    if (n0 >= 33) return c0;
    const int c1 = __builtin_amdgcn_readlane(v, __builtin_ctzll(~b0));
    const int n1 = __builtin_popcountll(__builtin_amdgcn_ballot_w64(v == c1));
    return n1 > n0 ? c1 : c0;
}

template <bool kOff32>
__device__ __forceinline__ int side_ld_assign(const int *__restrict__ assign, unsigned q, unsigned S, unsigned s) {
    if (kOff32) return ld32(assign, q * S + s);
    return assign[(size_t)q * S + s];
}

// The two largest keys over distinct nodes (keys of distinct nodes differ).
__device__ __forceinline__ void top2(unsigned long long k, unsigned long long &k1, unsigned long long &k2) {
    const bool g = k > k1;
    k2 = g ? k1 : (k > k2 ? k : k2);
    k1 = g ? k : k1;
}

__device__ __forceinline__ unsigned long long side_key(unsigned cnt, unsigned code, unsigned node) {
    return ((unsigned long long)cnt << 32) | (code << 16) | (0xffffu - node);
}

__device__ __forceinline__ int wave_incl_sum(int v, int lane) {  // inclusive prefix sum over lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(v, o, 64);
        v += lane >= o ? u : 0;
    }
    return v;
}

// Scenario ss of the row, exactly, by one wave (lanes = neighbours): the
// reference's decision (rescheduling.py:188-214) with exact remaining CPU for
// ties on an inexact code.  cells: scratch of >= min(d, ncap) words; the
// table is zeroed here and left dirty.
template <bool kOff32>
__device__ int side_exact(const SideArgs &a, const SideTab &tb, unsigned *cells, int ncap, cint_ptr nb, int d, int ss,
                          int lane, int H, int &score) {
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    for (int i = lane; i < H; i += 64) tb.tab[i] = 0u;
    // neighbour cells (code << 16 | node) staged in LDS segments of ncap, all counted
    unsigned long long best = 0ull, sec = 0ull;
    for (int pass = 0; pass < 3; ++pass) {  // 0: count, 1: best key, 2: second key (another node)
        for (int g0 = 0; g0 < d; g0 += ncap) {
            const int gn = min(ncap, d - g0);
            if (pass == 0 || d > ncap) {
                for (int j = lane; j < gn; j += 256) {
                    unsigned v[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        v[u] = min((unsigned)side_ld_assign<kOff32>(a.assign, (unsigned)nb[g0 + min(j + 64 * u, gn - 1)], S,
                                                                  (unsigned)ss), N);
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const unsigned c = ld16(a.code, v[u] * S + (unsigned)ss);  // row N: code 0
                        if (j + 64 * u < gn) cells[j + 64 * u] = (c << 16) | v[u];
                    }
                }
            }
            for (int j = lane; j < gn; j += 64) {
                const unsigned x = cells[j];
                const unsigned c = x >> 16, n = x & 0xffffu;
                if (c == kCodeHaz) continue;
                if (pass == 0) {
                    tb.add(n + 1u);
                } else {
                    const unsigned long long k = side_key(tb.tab[tb.find(n + 1u)] & 0xffffu, c, n);
                    if (pass == 1) best = k > best ? k : best;
                    else if (k != best) sec = k > sec ? k : sec;
                }
            }
        }
        if (pass == 1) best = dpp_max_u64(best);
    }
    const unsigned long long k1 = best, k2 = dpp_max_u64(sec);
    const int M = (int)(k1 >> 32);
    if (M == 0) return zero_target(load_zc(a.zc_cnt, a.zc_key, ss), score);
    score = M;
    const unsigned bw = (unsigned)k1, bk = bw >> 16;
    const bool tie = (int)(k2 >> 32) == M;
    if (!tie) return cand_node(bw);
    if (bk < 2u) return RSK_TARGET_NONE;
    if (!code_inexact(bk) || ((unsigned)k2 >> 16) != bk) return cand_node(bw);
    // equal inexact codes at the top: the largest exact cap - use, then the lower node
    unsigned long long kx = 0ull;
    for (int g0 = 0; g0 < d; g0 += ncap) {
        const int gn = min(ncap, d - g0);
        if (d > ncap) {
            for (int j = lane; j < gn; j += 64) {
                const unsigned n = min((unsigned)side_ld_assign<kOff32>(a.assign, (unsigned)nb[g0 + j], S, (unsigned)ss), N);
                cells[j] = (ld16(a.code, n * S + (unsigned)ss) << 16) | n;
            }
        }
        for (int j = lane; j < gn; j += 64) {
            const unsigned x = cells[j];
            const unsigned c = x >> 16, n = x & 0xffffu;
            if (c == bk && (int)(tb.tab[tb.find(n + 1u)] & 0xffffu) == M) {
                const int rem = a.cap[n] - ld32(a.use, n * S + (unsigned)ss);
                const unsigned long long k = pack_rn(rem, (int)n);
                kx = k > kx ? k : kx;
            }
        }
    }
    kx = dpp_max_u64(kx);
    return (int)(kNodeMask - (unsigned)(kx & kNodeMask));
}

// kW waves per workgroup, teams of kT waves (kT == 1: every wave its own item;
// kT == kW: one item per workgroup, barriers), kB neighbour loads in flight.
// kFast (single-wave teams): pass 1 also gathers each lane's codes and keeps
// its two best (1, code, -node) keys; when the pivots are distinct and no
// lane's deviations land on a pivot node or on each other, every candidate
// node counts 1 in every lane and those keys are the answer (no walk).
template <int kW, int kT, int kB, bool kOff32, bool kFast>
__global__ __launch_bounds__(64 * kW, (kT > 1 ? 1 : 8)) void car_side16_kernel(SideArgs a) {
    static_assert(kT == 1 || kT == kW, "a team is one wave or the whole workgroup");
    static_assert(!kFast || kT == 1, "the fast path is per wave");
    extern __shared__ __attribute__((aligned(16))) unsigned slds[];
    const int lane = (int)threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int team = wave / kT, tw = wave % kT;
    int blk = (int)blockIdx.x;
    if (a.xcd_per) blk = (int)(blockIdx.x & 7u) * a.xcd_per + (int)(blockIdx.x >> 3);  // blocks b, b + 8 share an XCD
    const int item = blk * (kW / kT) + team;
    if (item >= a.n_rows * a.nchunk) return;  // the whole team (kT > 1: the whole workgroup)
    const int chunk = item / a.n_rows, r = item - chunk * a.n_rows;
    const cint_ptr itp = const_ptr(a.items) + 4 * r;
    const int oi = itp[0], d = itp[2];
    const cint_ptr nb = const_ptr(a.col) + itp[1];
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    const int s0 = chunk * 64;
    const int s = min(s0 + lane, a.S - 1);
    const int H = a.H, K = a.K;

    unsigned *base = slds + (size_t)team * (a.lds_team >> 2);
    SideTab tb;
    tb.tab = base;
    tb.umask = reinterpret_cast<unsigned long long *>(base + a.off_umask);
    tb.mask = (unsigned)H - 1u;
    tb.shift = a.hshift;
    uint2 *srt = reinterpret_cast<uint2 *>(base + a.off_srt);  // level-sorted {count << 16 | node, table slot}
    unsigned *lvl = base + a.off_lvl;                           // [64] level counts, [64] level cursors
    unsigned *dl = base + a.off_dl;                             // [K][64] deviations (pivot << 16 | own node)
    int *ndl = reinterpret_cast<int *>(base + a.off_ndl);       // [64] deviations per lane (teams)

    for (int i = tw * 64 + lane; i < H; i += 64 * kT) {
        tb.tab[i] = 0u;
        tb.umask[i] = 0ull;
    }
    if (kT > 1) {
        if (tw == 0) ndl[lane] = 0;
        __syncthreads();
    }

    // ---- pass 1: pivots, deviations, pivot counts ----
    int nd = 0;  // kT == 1: this lane's deviations (teams count in ndl)
    int n_piv = 0, n_new = 0;              // kFast: pivots inserted, distinct pivot keys
    unsigned long long f1 = 0ull, f2 = 0ull;  // kFast: the lane's two best (1, code, -node) keys
    // each batch's neighbour ids in one vector load (lane u: entry j0 + u),
    // broadcast by readlane (no chain of dependent scalar loads), the next
    // batch's ids loaded behind this batch's assign rows
    const int *__restrict__ nbv = a.col + itp[1];
    int qnext = nbv[min(tw * kB + lane, d - 1)];
    for (int j0 = tw * kB; j0 < d; j0 += kB * kT) {
        const int myq = qnext;
        int v[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u)
            v[u] = side_ld_assign<kOff32>(a.assign, (unsigned)__builtin_amdgcn_readlane(myq, u), S, (unsigned)s);
        qnext = nbv[min(j0 + kB * kT + lane, d - 1)];
        if (kFast) {
            unsigned c[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) c[u] = ld16(a.code, min((unsigned)v[u], N) * S + (unsigned)s);  // row N: 0
#pragma unroll
            for (int u = 0; u < kB; ++u)
                if (j0 + u < d && c[u] != kCodeHaz) top2(side_key(1u, c[u], (unsigned)v[u]), f1, f2);
        }
        unsigned mine = 0u;  // lane u: key of entry j0 + u's pivot
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            if (j0 + u < d) {  // wave-uniform
                const int x = (int)min((unsigned)v[u], N);
                const int p = side_pivot(x);
                const bool dv = x != p;
                if (__builtin_amdgcn_ballot_w64(dv)) {
                    if (dv) {
                        const int k = kT > 1 ? atomicAdd(&ndl[lane], 1) : nd++;
                        if (k < K) dl[k * 64 + lane] = ((unsigned)p << 16) | (unsigned)x;
                    }
                }
                mine = (lane == u && p < (int)N) ? (unsigned)p + 1u : mine;
            }
        }
        bool fresh = false;
        if (mine) fresh = tb.add(mine);
        if (kFast) {
            n_piv += __builtin_popcountll(__builtin_amdgcn_ballot_w64(mine != 0u));
            n_new += __builtin_popcountll(__builtin_amdgcn_ballot_w64(fresh));
        }
    }
    if (kT > 1) {
        __syncthreads();
        nd = ndl[lane];
    }
    const int ndk = min(nd, K);

    unsigned long long k1 = 0ull, k2 = 0ull;
    bool fast = false;
    if (kFast && n_new == n_piv) {  // distinct pivots: is every lane's multiset of nodes duplicate-free?
        const int ndm = __builtin_amdgcn_readfirstlane(dpp_max(ndk));
        bool clean = nd <= K;
        for (int k = 0; k < ndm; ++k) {
            const unsigned x = k < ndk ? dl[k * 64 + lane] & 0xffffu : 0xffffu;
            if (x < N) {
                clean = clean && tb.find(x + 1u) < 0;  // lands on a pivot node (maybe one whose entry left too: conservative)
                for (int i = 0; i < k; ++i) clean = clean && (dl[i * 64 + lane] & 0xffffu) != x;
            }
        }
        fast = !__builtin_amdgcn_ballot_w64(!clean);
    }
    if (fast) {
        k1 = f1;
        k2 = f2;
    } else {

    // ---- marks: the pivot nodes whose count differs in the lane's scenario ----
    {
        const unsigned long long bit = 1ull << lane;
        const int ndmax = __builtin_amdgcn_readfirstlane(dpp_max(ndk));
        for (int k = tw; k < ndmax; k += kT) {
            if (k < ndk) {
                const unsigned x = dl[k * 64 + lane];
                const unsigned po = x >> 16, pn = x & 0xffffu;
                if (po < N) atomicOr(&tb.umask[tb.find(po + 1u)], bit);
                if (pn < N) {
                    const int h = tb.find(pn + 1u);
                    if (h >= 0) atomicOr(&tb.umask[h], bit);
                }
            }
        }
    }
    if (kT > 1) __syncthreads();
    if (tw != 0) return;  // the rest is one wave's (no more barriers)
    if (a.ablate & 2) {  // profiling: pass 1 and the marks only (results are wrong)
        if (s0 + lane < a.S) a.out_target[(size_t)(unsigned)oi * S + (unsigned)(s0 + lane)] = nd;
        return;
    }
    const int ndmax = __builtin_amdgcn_readfirstlane(dpp_max(ndk));

    // ---- levels: distinct pivot nodes by count, descending ----
    lvl[lane] = 0u;
    for (int h = lane; h < H; h += 64) {
        const unsigned w = tb.tab[h];
        if (w) atomicAdd(&lvl[min(w & 0xffffu, 64u) - 1u], 1u);
    }
    const int lc = (int)lvl[lane];  // nodes at level `lane` (count lane + 1; level 63: counts >= 64)
    const int incl = wave_incl_sum(lc, lane);
    const int tot = __builtin_amdgcn_readlane(incl, 63);
    const int lstart = tot - incl;  // levels above come first
    lvl[64 + lane] = (unsigned)lstart;
    for (int h = lane; h < H; h += 64) {
        const unsigned w = tb.tab[h];
        if (w) {
            const unsigned p = atomicAdd(&lvl[64 + min(w & 0xffffu, 64u) - 1u], 1u);
            srt[p] = make_uint2(((w & 0xffffu) << 16) | ((w >> 16) - 1u), (unsigned)h);
        }
    }

    // ---- walk: unflagged pivot nodes, level by level ----
    if (!(a.ablate & 4)) {
        const unsigned lsh = (unsigned)lane & 31u;
        const bool hiw = lane >= 32;
        unsigned long long lm = __builtin_amdgcn_ballot_w64(lc > 0);
        constexpr int kU = 8;
        while (lm) {
            const int L = 63 - __builtin_clzll(lm);
            lm &= ~(1ull << L);
            const int p0 = __builtin_amdgcn_readlane(lstart, L), p1 = p0 + __builtin_amdgcn_readlane(lc, L);
            for (int i0 = p0; i0 < p1; i0 += kU) {
                unsigned key[kU], ml[kU], c[kU];
#pragma unroll
                for (int w = 0; w < kU; ++w) {
                    const uint2 e = srt[min(i0 + w, p1 - 1)];
                    key[w] = (unsigned)__builtin_amdgcn_readfirstlane((int)e.x);
                    const unsigned long long m = tb.umask[__builtin_amdgcn_readfirstlane((int)e.y)];
                    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)m);
                    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(m >> 32));
                    ml[w] = hiw ? hi : lo;
                }
#pragma unroll
                for (int w = 0; w < kU; ++w) c[w] = ld16(a.code, (key[w] & 0xffffu) * S + (unsigned)s);
#pragma unroll
                for (int w = 0; w < kU; ++w) {
                    if (i0 + w < p1) {
                        const bool ok = c[w] != kCodeHaz && ((ml[w] >> lsh) & 1u) == 0u;
                        top2(ok ? side_key(key[w] >> 16, c[w], key[w] & 0xffffu) : 0ull, k1, k2);
                    }
                }
            }
            if (!lm) break;
            const unsigned next = (unsigned)(63 - __builtin_clzll(lm)) + 1u;  // the largest count left (exact below 64)
            if (!__builtin_amdgcn_ballot_w64((unsigned)(k1 >> 32) <= next)) break;
        }
    }

    // ---- touched: exact counts of the lane's flagged / new nodes ----
    for (int k0 = 0; k0 < ((a.ablate & 8) ? 0 : ndmax); k0 += 4) {
        unsigned t[8];
        int delta[8];
        bool seen[8];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const unsigned x = k0 + m < ndk ? dl[(k0 + m) * 64 + lane] : 0xffffffffu;
            t[2 * m] = x >> 16;
            t[2 * m + 1] = x & 0xffffu;
        }
#pragma unroll
        for (int m = 0; m < 8; ++m) { delta[m] = 0; seen[m] = false; }
        for (int i = 0; i < ndmax; ++i) {
            const unsigned xi = i < ndk ? dl[i * 64 + lane] : 0xffffffffu;
            const unsigned io = xi >> 16, in = xi & 0xffffu;
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                delta[m] += (int)(in == t[m]) - (int)(io == t[m]);
                seen[m] = seen[m] || (i < k0 + m / 2 && (io == t[m] || in == t[m]));
            }
        }
        int cnt[8];
        bool any = false;
        const int mcur = max(1, (int)(k1 >> 32));  // a node below the best count so far can neither win nor tie
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const bool ok = t[m] < N && !seen[m];
            int h = -1;
            if (ok) h = tb.find(t[m] + 1u);
            cnt[m] = ok ? (h >= 0 ? (int)(tb.tab[h] & 0xffffu) : 0) + delta[m] : 0;
            cnt[m] = cnt[m] >= mcur ? cnt[m] : 0;
            any = any || cnt[m] > 0;
        }
        if (__builtin_amdgcn_ballot_w64(any)) {  // wave-uniform: the codes of the nodes that can matter
            unsigned c[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) c[m] = ld16(a.code, (cnt[m] > 0 ? t[m] : N) * S + (unsigned)s);  // row N: 0
#pragma unroll
            for (int m = 0; m < 8; ++m)
                if (cnt[m] > 0 && c[m] != kCodeHaz) top2(side_key((unsigned)cnt[m], c[m], t[m]), k1, k2);
        }
    }
    }  // !fast

    // ---- decide ----
    const int M = (int)(k1 >> 32);
    bool slow = nd > K;
    int tg, sc;
    if (M == 0) {
        tg = zero_target(load_zc(a.zc_cnt, a.zc_key, s), sc);
    } else {
        sc = M;
        const unsigned bw = (unsigned)k1, bk = bw >> 16;
        const bool tie = (int)(k2 >> 32) == M;
        tg = !tie ? cand_node(bw) : (bk >= 2u ? cand_node(bw) : RSK_TARGET_NONE);
        slow = slow || (tie && code_inexact(bk) && ((unsigned)k2 >> 16) == bk);
    }
    unsigned long long sm = __builtin_amdgcn_ballot_w64(slow);
    if (sm && !(a.ablate & 1)) {  // rare: the wave, one scenario at a time
        while (sm) {
            const int ln = __builtin_ctzll(sm);
            sm &= sm - 1ull;
            int sx;
            const int tx = side_exact<kOff32>(a, tb, reinterpret_cast<unsigned *>(srt), a.cells, nb, d,
                                              min(s0 + ln, a.S - 1), lane, H, sx);
            tg = lane == ln ? tx : tg;
            sc = lane == ln ? sx : sc;
        }
    }
    if (s0 + lane < a.S) {
        const size_t o = kOff32 ? (size_t)((unsigned)oi * S + (unsigned)(s0 + lane))
                                : (size_t)(unsigned)oi * S + (unsigned)(s0 + lane);
        a.out_target[o] = tg;
        if (a.out_score) a.out_score[o] = sc;
    }
}

// ---------------------------------------------------------------------------
// Single-wave items (rows up to 256 neighbours): the same algorithm with the
// per-entry work kept on the vector unit — majority-of-three pivots, deviation
// appends without branches (lanes that do not deviate write a dummy word), the
// running best as (count, two 32-bit candidate words) — and a fast path:
//   kFast  pass 1 also gathers each lane's codes and keeps the best two
//          count-1 words.  When the pivots are distinct and a lane's
//          deviations land neither on a pivot node nor on each other, every
//          candidate node counts 1 in that lane: those words are its answer.
//          Up to kFastSlowMax lanes that fail this are recounted exactly one by
//          one; more, or repeated pivots, take the walk.
// ---------------------------------------------------------------------------
constexpr int kFastSlowMax = 6;

// Running best over distinct nodes: the largest count M and the two largest
// candidate words (code << 16 | 0xffff - node) among the nodes at M.
struct Best {
    int M;
    unsigned w1, w2;
    __device__ __forceinline__ void init() { M = 0; w1 = w2 = 0u; }
    __device__ __forceinline__ void put(bool ok, int c, unsigned w) {
        const bool gt = ok && c > M, eq = ok && c == M;
        const bool g1 = eq && w > w1;
        w2 = gt ? 0u : (g1 ? w1 : ((eq && w > w2) ? w : w2));
        w1 = (gt || g1) ? w : w1;
        M = gt ? c : M;
    }
};

__device__ __forceinline__ int side_pivot3(int x) {  // majority of lanes 0, 21, 42 (lane 0 without one)
    const int a = __builtin_amdgcn_readlane(x, 0), b = __builtin_amdgcn_readlane(x, 21),
              c = __builtin_amdgcn_readlane(x, 42);
    return (a == b || a == c) ? a : (b == c ? b : a);
}

template <int kW, int kB, bool kOff32, bool kFast>
__global__ __launch_bounds__(64 * kW, 8) void car_side16_wave_kernel(SideArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned slds[];
    const int lane = (int)threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    int blk = (int)blockIdx.x;
    if (a.xcd_per) blk = (int)(blockIdx.x & 7u) * a.xcd_per + (int)(blockIdx.x >> 3);  // blocks b, b + 8 share an XCD
    const int item = blk * kW + wave;
    if (item >= a.n_rows * a.nchunk) return;  // whole wave (no barriers in this kernel)
    const int chunk = item / a.n_rows, r = item - chunk * a.n_rows;
    const cint_ptr itp = const_ptr(a.items) + 4 * r;
    const int oi = itp[0], d = itp[2];
    const int *__restrict__ nbv = a.col + itp[1];
    const cint_ptr nb = const_ptr(a.col) + itp[1];
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    const int s0 = chunk * 64;
    const int s = min(s0 + lane, a.S - 1);
    const int H = a.H, K = a.K;

    unsigned *base = slds + (size_t)wave * (a.lds_team >> 2);
    SideTab tb;
    tb.tab = base;
    tb.umask = reinterpret_cast<unsigned long long *>(base + a.off_umask);
    tb.mask = (unsigned)H - 1u;
    tb.shift = a.hshift;
    uint2 *srt = reinterpret_cast<uint2 *>(base + a.off_srt);
    unsigned *lvl = base + a.off_lvl;
    unsigned *dl = base + a.off_dl;
    unsigned *dummy = base + a.off_ndl;  // [64] sink of the non-deviating lanes' writes
    for (int i = lane; i < H; i += 64) tb.tab[i] = 0u;

    // ---- pass 1 ----
    int nd = 0, n_piv = 0, n_new = 0;
    Best fb;
    fb.init();
    int qnext = nbv[min(lane, d - 1)];
    for (int j0 = 0; j0 < d; j0 += kB) {
        const int myq = qnext;
        int v[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u)
            v[u] = side_ld_assign<kOff32>(a.assign, (unsigned)__builtin_amdgcn_readlane(myq, u), S, (unsigned)s);
        qnext = nbv[min(j0 + kB + lane, d - 1)];
        unsigned c[kB];
        if (kFast) {
#pragma unroll
            for (int u = 0; u < kB; ++u) c[u] = ld16(a.code, min((unsigned)v[u], N) * S + (unsigned)s);  // row N: 0
        }
        const int nu = min(kB, d - j0);
        unsigned mine = 0u;
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            if (u < nu) {  // wave-uniform
                const int x = (int)min((unsigned)v[u], N);
                const int p = side_pivot3(x);
                const bool dv = x != p;
                unsigned *dst = (dv && nd < K) ? dl + nd * 64 + lane : dummy + lane;
                *dst = ((unsigned)p << 16) | (unsigned)x;
                nd += dv ? 1 : 0;
                mine = lane == u ? (unsigned)p + 1u : mine;
                if (kFast) fb.put(c[u] != kCodeHaz, 1, (c[u] << 16) | (0xffffu - (unsigned)x));
            }
        }
        const bool ins = mine != 0u && mine <= N;  // pivot node < N (N: unassigned, never counted)
        bool fresh = false;
        if (ins) fresh = tb.add(mine);
        if (kFast) {
            n_piv += __builtin_popcountll(__builtin_amdgcn_ballot_w64(ins));
            n_new += __builtin_popcountll(__builtin_amdgcn_ballot_w64(fresh));
        }
    }
    const int ndk = min(nd, K);
    const int ndmax = __builtin_amdgcn_readfirstlane(dpp_max(ndk));

    Best b;
    bool slow = nd > K, done = false;
    if (kFast && n_new == n_piv) {  // distinct pivots: which lanes hold a node twice?
        bool clean = nd <= K;
        for (int k = 0; k < ndmax; ++k) {
            const unsigned x = k < ndk ? dl[k * 64 + lane] & 0xffffu : 0xffffu;
            if (x < N) {
                clean = clean && tb.find(x + 1u) < 0;  // on a pivot node (whose entry may have left too: conservative)
                for (int i = 0; i < k; ++i) clean = clean && (dl[i * 64 + lane] & 0xffffu) != x;
            }
        }
        if (__builtin_popcountll(__builtin_amdgcn_ballot_w64(!clean)) <= kFastSlowMax) {
            b = fb;
            slow = slow || !clean;
            done = true;
        }
    }
    if (!done) {
        b.init();
        for (int i = lane; i < H; i += 64) tb.umask[i] = 0ull;
        // ---- marks ----
        const unsigned long long bit = 1ull << lane;
        for (int k = 0; k < ndmax; ++k) {
            if (k < ndk) {
                const unsigned x = dl[k * 64 + lane];
                const unsigned po = x >> 16, pn = x & 0xffffu;
                if (po < N) atomicOr(&tb.umask[tb.find(po + 1u)], bit);
                if (pn < N) {
                    const int h = tb.find(pn + 1u);
                    if (h >= 0) atomicOr(&tb.umask[h], bit);
                }
            }
        }
        // ---- levels ----
        lvl[lane] = 0u;
        for (int h = lane; h < H; h += 64) {
            const unsigned w = tb.tab[h];
            if (w) atomicAdd(&lvl[min(w & 0xffffu, 64u) - 1u], 1u);
        }
        const int lc = (int)lvl[lane];
        const int incl = wave_incl_sum(lc, lane);
        const int lstart = __builtin_amdgcn_readlane(incl, 63) - incl;
        lvl[64 + lane] = (unsigned)lstart;
        for (int h = lane; h < H; h += 64) {
            const unsigned w = tb.tab[h];
            if (w) {
                const unsigned p = atomicAdd(&lvl[64 + min(w & 0xffffu, 64u) - 1u], 1u);
                srt[p] = make_uint2(((w & 0xffffu) << 16) | ((w >> 16) - 1u), (unsigned)h);
            }
        }
        // ---- walk: level by level, until every lane's best count beats what is left ----
        const unsigned lsh = (unsigned)lane & 31u;
        const bool hiw = lane >= 32;
        unsigned long long lm = __builtin_amdgcn_ballot_w64(lc > 0);
        constexpr int kU = 8;
        while (lm) {
            const int L = 63 - __builtin_clzll(lm);
            lm &= ~(1ull << L);
            const int p0 = __builtin_amdgcn_readlane(lstart, L), p1 = p0 + __builtin_amdgcn_readlane(lc, L);
            for (int i0 = p0; i0 < p1; i0 += kU) {
                unsigned key[kU], ml[kU], c[kU];
#pragma unroll
                for (int w = 0; w < kU; ++w) {
                    const uint2 e = srt[min(i0 + w, p1 - 1)];
                    key[w] = e.x;
                    const unsigned long long m = tb.umask[e.y];
                    ml[w] = hiw ? (unsigned)(m >> 32) : (unsigned)m;
                }
#pragma unroll
                for (int w = 0; w < kU; ++w) c[w] = ld16(a.code, (key[w] & 0xffffu) * S + (unsigned)s);
#pragma unroll
                for (int w = 0; w < kU; ++w) {
                    const bool ok = i0 + w < p1 && c[w] != kCodeHaz && ((ml[w] >> lsh) & 1u) == 0u;
                    b.put(ok, (int)(key[w] >> 16), (c[w] << 16) | (0xffffu - (key[w] & 0xffffu)));
                }
            }
            if (!lm) break;
            const int next = 64 - __builtin_clzll(lm);  // the largest count left (exact below 64)
            if (!__builtin_amdgcn_ballot_w64(b.M <= next)) break;
        }
        // ---- touched ----
        for (int k0 = 0; k0 < ndmax; k0 += 4) {
            unsigned t[8];
            int delta[8];
            bool seen[8];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const unsigned x = k0 + m < ndk ? dl[(k0 + m) * 64 + lane] : 0xffffffffu;
                t[2 * m] = x >> 16;
                t[2 * m + 1] = x & 0xffffu;
            }
#pragma unroll
            for (int m = 0; m < 8; ++m) { delta[m] = 0; seen[m] = false; }
            for (int i = 0; i < ndmax; ++i) {
                const unsigned xi = i < ndk ? dl[i * 64 + lane] : 0xffffffffu;
                const unsigned io = xi >> 16, in = xi & 0xffffu;
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    delta[m] += (int)(in == t[m]) - (int)(io == t[m]);
                    seen[m] = seen[m] || (i < k0 + m / 2 && (io == t[m] || in == t[m]));
                }
            }
            int cnt[8];
            bool any = false;
            const int mcur = max(1, b.M);
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const bool ok = t[m] < N && !seen[m];
                int h = -1;
                if (ok) h = tb.find(t[m] + 1u);
                cnt[m] = ok ? (h >= 0 ? (int)(tb.tab[h] & 0xffffu) : 0) + delta[m] : 0;
                cnt[m] = cnt[m] >= mcur ? cnt[m] : 0;
                any = any || cnt[m] > 0;
            }
            if (__builtin_amdgcn_ballot_w64(any)) {
                unsigned c[8];
#pragma unroll
                for (int m = 0; m < 8; ++m) c[m] = ld16(a.code, (cnt[m] > 0 ? t[m] : N) * S + (unsigned)s);
#pragma unroll
                for (int m = 0; m < 8; ++m)
                    b.put(cnt[m] > 0 && c[m] != kCodeHaz, cnt[m], (c[m] << 16) | (0xffffu - t[m]));
            }
        }
    }

    // ---- decide ----
    int tg, sc;
    if (b.M == 0) {
        tg = zero_target(load_zc(a.zc_cnt, a.zc_key, s), sc);
    } else {
        sc = b.M;
        const unsigned bk = b.w1 >> 16;
        const bool tie = b.w2 != 0u;
        tg = !tie ? cand_node(b.w1) : (bk >= 2u ? cand_node(b.w1) : RSK_TARGET_NONE);
        slow = slow || (tie && code_inexact(bk) && (b.w2 >> 16) == bk);
    }
    unsigned long long sm = __builtin_amdgcn_ballot_w64(slow);
    if (sm && !(a.ablate & 1)) {  // rare: the wave, one scenario at a time
        while (sm) {
            const int ln = __builtin_ctzll(sm);
            sm &= sm - 1ull;
            int sx;
            const int tx = side_exact<kOff32>(a, tb, reinterpret_cast<unsigned *>(srt), a.cells, nb, d,
                                              min(s0 + ln, a.S - 1), lane, H, sx);
            tg = lane == ln ? tx : tg;
            sc = lane == ln ? sx : sc;
        }
    }
    if (s0 + lane < a.S) {
        const size_t o = kOff32 ? (size_t)((unsigned)oi * S + (unsigned)(s0 + lane))
                                : (size_t)(unsigned)oi * S + (unsigned)(s0 + lane);
        a.out_target[o] = tg;
        if (a.out_score) a.out_score[o] = sc;
    }
}

SideGeom side16_geometry(int dmax, int N) {
    SideGeom g;
    g.dmax = dmax;
    g.Dc = std::max(1, std::min(dmax, N));  // distinct pivot nodes (node N = unassigned is never counted)
    int H = 64;
    while (H < g.Dc + g.Dc / 2 + 1) H <<= 1;  // load <= 2/3
    g.H = H;
    int l = 0;
    while ((1 << l) < H) ++l;
    g.hshift = 32 - l;
    g.K = std::min(64, 8 + dmax / 32);  // deviation slots per lane (overflow: the exact recount)
    g.T = dmax <= 256 ? 1 : 8;
    // the duplicate-free fast path where distinct pivots are the common case
    static const int fast_max = [] { const char *e = getenv("RSK_SIDE_FAST_MAX"); return e ? atoi(e) : 128; }();
    g.fast = g.T == 1 && dmax <= fast_max;
    // neighbour loads in flight per wave: 32 where registers allow (the fast
    // path's codes double the batch's registers: 16)
    g.kB = dmax <= 32 ? 8 : (dmax <= 64 || g.fast ? 16 : 32);
    // words: tab H | umask 2H | srt 2 Dc (also the recount's cells) | lvl 128 | dl 64 K | ndl 64
    g.cells = std::max(2 * g.Dc, std::min(dmax, 4096));
    g.off_umask = H;
    g.off_srt = 3 * H;
    g.off_lvl = g.off_srt + ((g.cells + 3) & ~3);
    g.off_dl = g.off_lvl + 128;
    g.off_ndl = g.off_dl + 64 * g.K;
    g.lds_team = ((size_t)(g.off_ndl + 64) * 4 + 15) & ~(size_t)15;
    // teams per workgroup: 4 single-wave teams while they fit 40 KiB, else fewer
    if (g.T > 1) g.W = g.T;
    else g.W = 4 * g.lds_team <= 40 * 1024 ? 4 : (2 * g.lds_team <= 80 * 1024 ? 2 : 1);
    return g;
}

int launch_side16(hipStream_t stream, const SideArgs &a0, const SideGeom &g, bool off32) {
    if (a0.n_rows == 0) return RSK_OK;
    const size_t lds = (size_t)(g.T > 1 ? 1 : g.W) * g.lds_team;
    RSK_CHECK(lds <= 160 * 1024,
              "a relation row of degree %d needs %zu B of LDS for its %d distinct nodes (limit 160 KiB)", g.dmax,
              g.lds_team, g.Dc);
    SideArgs a = a0;
    a.H = g.H;
    a.hshift = g.hshift;
    a.K = g.K;
    a.cells = g.cells;
    a.lds_team = (unsigned)g.lds_team;
    a.off_umask = g.off_umask;
    a.off_srt = g.off_srt;
    a.off_lvl = g.off_lvl;
    a.off_dl = g.off_dl;
    a.off_ndl = g.off_ndl;
    const int64_t items = (int64_t)a.n_rows * a.nchunk;
    RSK_CHECK(items < INT32_MAX / 8, "side grid too large");
    const int teams = g.T > 1 ? 1 : g.W;
    const int64_t blocks_needed = ceil_div(items, teams);
    a.xcd_per = (int)ceil_div(blocks_needed, 8);
    const int64_t blocks = 8 * (int64_t)a.xcd_per;
    using K = void (*)(SideArgs);
#define RSK_SIDE_O(W, T, B, F) (off32 ? &car_side16_kernel<W, T, B, true, F> : &car_side16_kernel<W, T, B, false, F>)
#define RSK_SIDE_B(W, T, F) \
    (g.kB == 8 ? RSK_SIDE_O(W, T, 8, F) : g.kB == 16 ? RSK_SIDE_O(W, T, 16, F) : RSK_SIDE_O(W, T, 32, F))
#define RSK_WAVE_O(W, B, F) (off32 ? &car_side16_wave_kernel<W, B, true, F> : &car_side16_wave_kernel<W, B, false, F>)
#define RSK_WAVE_B(W, F) \
    (g.kB == 8 ? RSK_WAVE_O(W, 8, F) : g.kB == 16 ? RSK_WAVE_O(W, 16, F) : RSK_WAVE_O(W, 32, F))
#define RSK_SIDE_F(W) (g.fast ? RSK_WAVE_B(W, true) : RSK_WAVE_B(W, false))
    const K kern = g.T == 8 ? RSK_SIDE_B(8, 8, false)
                            : (g.W == 4 ? RSK_SIDE_F(4) : g.W == 2 ? RSK_SIDE_F(2) : RSK_SIDE_F(1));
#undef RSK_SIDE_F
#undef RSK_WAVE_B
#undef RSK_WAVE_O
#undef RSK_SIDE_B
#undef RSK_SIDE_O
    if (lds > 64 * 1024)
        RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
    kern<<<dim3((unsigned)blocks), dim3(64 * g.W), lds, stream>>>(a);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

}  // namespace rsk
