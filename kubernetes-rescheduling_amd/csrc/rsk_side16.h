// rsk_side16.h — the side-row scorer of the compact path as a device
// function (one workgroup's work items), shared by car_side16_kernel
// (rsk_side16.hip) and the fused tile + side kernel (rsk_car16.hip).
// The algorithm and its reference lines: rsk_side16.hip's header.
#pragma once

#include "rsk_car.h"

namespace rsk {

// The team's hash table: H words (node + 1) << 16 | count.
struct SideTab {
    unsigned *tab;
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

template <bool kOff32>
__device__ __forceinline__ int side_ld_assign(const int *__restrict__ assign, unsigned q, unsigned S, unsigned s) {
    if (kOff32) return ld32(assign, q * S + s);
    return assign[(size_t)q * S + s];
}

__device__ __forceinline__ unsigned long long side_key(unsigned cnt, unsigned code, unsigned node) {
    return ((unsigned long long)cnt << 32) | (code << 16) | (0xffffu - node);
}

// Scenario ss of the row, exactly, by one wave (lanes = neighbours): the
// reference's decision (rescheduling.py:188-214) with exact remaining CPU for
// ties on an inexact code.  cells: scratch of >= min(d, ncap) words; the
// table is zeroed here and left dirty.
// Work areas in global memory (a.gscratch, tables beyond the LDS): plain loads
// may hit stale L1 lines after other lanes' stores or atomics (performed in L2),
// so every switch from writing to reading such an area goes through an
// agent-scope fence, which invalidates the L1.
__device__ __forceinline__ void glob_fence(bool glob) {
    if (glob) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
}

// A node's code: the prep kernel's table, or (kOTF) computed from cap / use /
// hazard as car_prep computes it (node N and beyond: no candidate).
template <bool kOTF>
__device__ __forceinline__ unsigned side_code(const SideArgs &a, unsigned n, unsigned s, int B) {
    if (!kOTF) return ld16(a.code, n * (unsigned)a.S + s);  // row N: code 0
    if (n >= (unsigned)a.N) return kCodeHaz;
    const unsigned i = n * (unsigned)a.S + s;
    return code16(a.cap[n] - ld32(a.use, i), a.haz[i] != 0, B);
}

// kOTF: the zero case of scenario ss (car_prep's per-scenario reduction:
// non-hazard count, max packed (cap - use, ~node)) by the whole wave, lanes over
// the nodes — only for lanes whose rows reach no candidate node (rare).
__device__ __noinline__ ZeroCase side_zc_scan(const SideArgs &a, int ss, int lane) {
    const unsigned S = (unsigned)a.S;
    int cnt = 0;
    unsigned long long key = 0ull;
    for (int n0 = 0; n0 < a.N; n0 += 64) {
        const int n = n0 + lane;
        const bool ok = n < a.N && a.haz[(size_t)n * S + (unsigned)ss] == 0;
        cnt += __builtin_popcountll(__builtin_amdgcn_ballot_w64(ok));
        const unsigned long long k = ok ? zc_pack(a.cap[n] - a.use[(size_t)n * S + (unsigned)ss], n) : 0ull;
        key = k > key ? k : key;
    }
    ZeroCase z;
    z.cnt = cnt;
    z.key = dpp_max_u64(key);
    return z;
}

template <bool kOff32, bool kOTF = false>
__device__ int side_exact(const SideArgs &a, const SideTab &tb, unsigned *cells, int ncap, cint_ptr nb, int d, int ss,
                          int lane, int H, int &score, int B = 0) {
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    const bool glob = a.gscratch != nullptr;
    for (int i = lane; i < H; i += 64) tb.tab[i] = 0u;
    glob_fence(glob);
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
                        const unsigned c = side_code<kOTF>(a, v[u], (unsigned)ss, B);  // node N: code 0
                        if (j + 64 * u < gn) cells[j + 64 * u] = (c << 16) | v[u];
                    }
                }
            }
            glob_fence(glob);  // the staged cells and the pass-0 counts before they are read
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
        glob_fence(glob);
    }
    const unsigned long long k1 = best, k2 = dpp_max_u64(sec);
    const int M = (int)(k1 >> 32);
    if (M == 0) return zero_target(kOTF ? side_zc_scan(a, ss, lane) : load_zc(a.zc_cnt, a.zc_key, ss), score);
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
                cells[j] = (side_code<kOTF>(a, n, (unsigned)ss, B) << 16) | n;
            }
            glob_fence(glob);
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

// The two largest distinct candidate words (0 = none); equal words are the same node.
struct Top2 {
    unsigned w1, w2;
    __device__ __forceinline__ void init() { w1 = w2 = 0u; }
    __device__ __forceinline__ void put(unsigned w) {
        const bool g1 = w > w1;
        w2 = g1 ? w1 : ((w != w1 && w > w2) ? w : w2);
        w1 = g1 ? w : w1;
    }
};

__device__ __forceinline__ unsigned cand_word(unsigned code, unsigned node) { return (code << 16) | (0xffffu - node); }

__device__ __forceinline__ int side_pivot3(int x) {  // majority of lanes 0, 21, 42 (lane 0 without one)
    const int a = __builtin_amdgcn_readlane(x, 0), b = __builtin_amdgcn_readlane(x, 21),
              c = __builtin_amdgcn_readlane(x, 42);
    return (a == b || a == c) ? a : (b == c ? b : a);
}

// kW waves per workgroup, teams of kT waves (kT == 1: every wave its own item,
// no barriers; kT == kW: one item per workgroup), kB neighbour loads in flight
// per wave.
//
// Why no walk over the count levels is needed: let X be the lane's multiset of
// neighbour nodes.  Pass 1 keeps the lane's two largest distinct candidate
// words over X (f).  If no candidate node occurs twice in X, every candidate
// scores 1 and f is the answer.  A node u occurs twice only if its pivot count
// C[u] >= 2, or the lane has a deviation whose own node is u (otherwise its
// count is at most C[u] <= 1); the lane's count of u is C[u] minus its
// deviations away from u plus its deviations onto u.  So the exact count >= 2
// candidates are: the table's entries with C >= 2 (a handful), and the lane's
// deviation nodes — both small sets.
template <int kW, int kT, int kB, bool kOff32, bool kPipe, bool kGlobal = false, bool kOTF = false>
__device__ __forceinline__ void side16_block(const SideArgs &a, int blk, int slot = -1, int Bw = 0) {
    static_assert(kT == 1 || kT == kW, "a team is one wave or the whole workgroup");
    extern __shared__ __attribute__((aligned(16))) unsigned slds[];
    const int lane = (int)threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int team = wave / kT, tw = wave % kT;
    const int item = blk * (kW / kT) + team;
    if (item >= a.n_rows * a.nchunk) return;  // the whole team (kT > 1: the whole workgroup)
    const int chunk = item / a.n_rows, r = item - chunk * a.n_rows;
    const cint_ptr itp = const_ptr(a.items) + 4 * r;
    const int oi = itp[0], d = itp[2];
    const int *__restrict__ nbv = a.col + itp[1];
    const cint_ptr nb = const_ptr(a.col) + itp[1];
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    const int s0 = chunk * 64;
    const int s = min(s0 + lane, a.S - 1);
    const int H = a.H, K = a.K;
    const int B = kOTF ? Bw : 0;  // the exact code window (rsk_car.h), from the kernel's max(cap)

    // kGlobal (one team per workgroup): the team's table, lists and merge area in
    // global scratch (a table beyond the LDS); the same code with global atomics
    unsigned *base = kGlobal ? a.gscratch + (size_t)(unsigned)(slot >= 0 ? slot : blk) * (a.lds_team >> 2)
                             : slds + (size_t)team * (a.lds_team >> 2);
    SideTab tb;
    tb.tab = base;
    tb.mask = (unsigned)H - 1u;
    tb.shift = a.hshift;
    unsigned *dl = base + a.off_dl;                        // [K][64] deviations (pivot << 16 | own node)
    int *ndl = reinterpret_cast<int *>(base + a.off_ndl);  // [64] deviations per lane (teams)
    unsigned *dummy = base + a.off_dummy;                  // [64] sink of the non-deviating lanes' writes
    unsigned *fx = base + a.off_fx;                        // teams: [kT][2][64] the waves' top-2 words
    unsigned *h2 = base + a.off_h2;                        // [1 + n2] counter, table words counted >= 2
    unsigned *bx = h2;                                     // teams, after the list: [kT][3][64] the waves' bests

    for (int i = tw * 64 + lane; i < H; i += 64 * kT) tb.tab[i] = 0u;
    if (kT > 1) {
        if (tw == 0) {
            ndl[lane] = 0;
            if (lane == 0) h2[0] = 0u;
        }
        glob_fence(kGlobal);
        __syncthreads();
    }

    // ---- pass 1: the lane's top-2 words, pivots counted, deviations listed ----
    int nd = 0;  // kT == 1: this lane's deviations (teams count in ndl)
    Top2 f;
    f.init();
    // each batch's neighbour ids in one vector load (lane u: entry j0 + u),
    // broadcast by readlane; kPipe: the next batch's assign rows are loaded
    // before this batch is scored (its code gathers wait only for its own rows)
    int qnext = nbv[min(tw * kB + lane, d - 1)];
    int v[kB];
    if (kPipe) {
        const int myq = qnext;
#pragma unroll
        for (int u = 0; u < kB; ++u)
            v[u] = side_ld_assign<kOff32>(a.assign, (unsigned)__builtin_amdgcn_readlane(myq, u), S, (unsigned)s);
        qnext = nbv[min(tw * kB + kB * kT + lane, d - 1)];
    }
    for (int j0 = tw * kB; j0 < d; j0 += kB * kT) {
        if (!kPipe) {
            const int myq = qnext;
#pragma unroll
            for (int u = 0; u < kB; ++u)
                v[u] = side_ld_assign<kOff32>(a.assign, (unsigned)__builtin_amdgcn_readlane(myq, u), S, (unsigned)s);
            qnext = nbv[min(j0 + kB * kT + lane, d - 1)];
        }
        unsigned c[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) c[u] = side_code<kOTF>(a, min((unsigned)v[u], N), (unsigned)s, B);  // row N: 0
        int vn[kB];
        if (kPipe) {  // ids clamped to the row: always valid addresses
            const int myq = qnext;
#pragma unroll
            for (int u = 0; u < kB; ++u)
                vn[u] = side_ld_assign<kOff32>(a.assign, (unsigned)__builtin_amdgcn_readlane(myq, u), S, (unsigned)s);
            qnext = nbv[min(j0 + 2 * kB * kT + lane, d - 1)];
        }
        const int nu = min(kB, d - j0);
        unsigned mine = 0u;  // lane u: key of entry j0 + u's pivot
#pragma unroll
        for (int u = 0; u < kB; ++u) {
            if (u < nu) {  // wave-uniform
                const int x = (int)min((unsigned)v[u], N);
                const int p = side_pivot3(x);
                const bool dv = x != p;
                const unsigned rec = ((unsigned)p << 16) | (unsigned)x;
                if (kT == 1) {  // branch-free append
                    unsigned *dst = (dv && nd < K) ? dl + nd * 64 + lane : dummy + lane;
                    *dst = rec;
                    nd += dv ? 1 : 0;
                } else if (__builtin_amdgcn_ballot_w64(dv)) {
                    if (dv) {
                        const int k = atomicAdd(&ndl[lane], 1);
                        if (k < K) dl[k * 64 + lane] = rec;
                    }
                }
                mine = lane == u ? (unsigned)p + 1u : mine;
                f.put(c[u] != kCodeHaz ? cand_word(c[u], (unsigned)x) : 0u);
            }
        }
        if (mine != 0u && mine <= N) tb.add(mine);  // pivot node < N (N: unassigned, never counted)
        if (kPipe) {
#pragma unroll
            for (int u = 0; u < kB; ++u) v[u] = vn[u];
        }
    }
    if (kT > 1) {
        fx[(2 * tw) * 64 + lane] = f.w1;
        fx[(2 * tw + 1) * 64 + lane] = f.w2;
        glob_fence(kGlobal);
        __syncthreads();
        glob_fence(kGlobal);
        nd = ndl[lane];
    }
    const int ndk = min(nd, K);
    const int ndmax = __builtin_amdgcn_readfirstlane(dpp_max(ndk));
    if (RSK_ABL(a) & 2) {  // profiling: pass 1 only (results are wrong)
        if (tw == 0 && s0 + lane < a.S) a.out_target[(size_t)(unsigned)oi * S + (unsigned)(s0 + lane)] = (int)f.w1 + nd;
        return;
    }

    // ---- the nodes the lane may count twice or more, exactly ----
    // the table entries counted >= 2, listed (few)
    int n2 = 0;
    for (int h0 = tw * 64; h0 < H; h0 += 64 * kT) {
        const unsigned w = tb.tab[h0 + lane];
        const bool big = (w & 0xffffu) >= 2u;
        const unsigned long long m = __builtin_amdgcn_ballot_w64(big);
        if (!m) continue;
        int pos;
        if (kT == 1) {
            pos = n2 + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
            n2 += __builtin_popcountll(m);
        } else {
            pos = big ? (int)atomicAdd(&h2[0], 1u) : 0;
        }
        if (big && pos < a.h2cap) h2[1 + pos] = w;
    }
    if (kT > 1) {
        glob_fence(kGlobal);
        __syncthreads();
        glob_fence(kGlobal);
        n2 = (int)h2[0];
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the list's LDS writes before its reads
    }
    const bool h2over = n2 > a.h2cap;  // more nodes counted twice than the list holds: every lane recounts
    n2 = min(n2, a.h2cap);
    Best b;
    b.init();
    // (1) the listed nodes, eight at a time (their codes gathered together); the
    // team's waves take turns
    for (int i0 = tw * 8; i0 < ((RSK_ABL(a) & 4) ? 0 : n2); i0 += 8 * kT) {
        unsigned key[8], c[8];
        int delta[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            key[i] = i0 + i < n2 ? h2[1 + i0 + i] : 0u;  // wave-uniform
            delta[i] = 0;
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] = side_code<kOTF>(a, key[i] ? (key[i] >> 16) - 1u : N, (unsigned)s, B);
        for (int k = 0; k < ndmax; ++k) {
            const unsigned x = k < ndk ? dl[k * 64 + lane] : 0xffffffffu;
            const unsigned io = (x >> 16) + 1u, in = (x & 0xffffu) + 1u;  // table keys (node + 1)
#pragma unroll
            for (int i = 0; i < 8; ++i) delta[i] += (int)(in == key[i] >> 16) - (int)(io == key[i] >> 16);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int cnt = (int)(key[i] & 0xffffu) + delta[i];
            b.put(key[i] != 0u && c[i] != kCodeHaz && cnt >= 2, cnt, cand_word(c[i], (key[i] >> 16) - 1u));
        }
    }
    // (2) the lane's deviation nodes (first occurrence each) not counted >= 2 as a
    // pivot; the team's waves take turns
    for (int k = tw; k < ((RSK_ABL(a) & 8) ? 0 : ndmax); k += kT) {
        const unsigned t = k < ndk ? dl[k * 64 + lane] & 0xffffu : 0xffffu;
        bool ok = t < N;
        int cnt = 0;
        if (__builtin_amdgcn_ballot_w64(ok)) {
            const int h = ok ? tb.find(t + 1u) : -1;
            const int C = h >= 0 ? (int)(tb.tab[h] & 0xffffu) : 0;
            ok = ok && C < 2;
            int delta = 0;
            bool seen = false;
            for (int i = 0; i < ndmax; ++i) {
                const unsigned xi = i < ndk ? dl[i * 64 + lane] : 0xffffffffu;
                const bool to = (xi & 0xffffu) == t;
                delta += (int)to - (int)((xi >> 16) == t);
                seen = seen || (i < k && to);
            }
            cnt = ok && !seen ? C + delta : 0;
        }
        if (__builtin_amdgcn_ballot_w64(cnt >= 2)) {
            const unsigned c = side_code<kOTF>(a, cnt >= 2 ? t : N, (unsigned)s, B);
            b.put(cnt >= 2 && c != kCodeHaz, cnt, cand_word(c, t));
        }
    }
    if (kT > 1) {  // the waves' bests (disjoint node sets) and top-2 words to wave 0
        __syncthreads();  // every wave is done with the list bx overwrites
        bx[(3 * tw) * 64 + lane] = (unsigned)b.M;
        bx[(3 * tw + 1) * 64 + lane] = b.w1;
        bx[(3 * tw + 2) * 64 + lane] = b.w2;
        glob_fence(kGlobal);
        __syncthreads();
        glob_fence(kGlobal);
        if (tw != 0) return;  // the rest is one wave's (no more barriers)
#pragma unroll 1
        for (int w = 1; w < kT; ++w) {
            const int Mw = (int)bx[(3 * w) * 64 + lane];
            const unsigned w2w = bx[(3 * w + 2) * 64 + lane];
            b.put(Mw > 0, Mw, bx[(3 * w + 1) * 64 + lane]);
            b.put(Mw > 0 && w2w != 0u, Mw, w2w);
            f.put(fx[(2 * w) * 64 + lane]);
            f.put(fx[(2 * w + 1) * 64 + lane]);
        }
    }

    // ---- decide (rescheduling.py:199-214) ----
    const bool two = b.M >= 2;
    const int M = two ? b.M : (f.w1 ? 1 : 0);
    const unsigned w1 = two ? b.w1 : f.w1, w2 = two ? b.w2 : f.w2;
    bool slow = nd > K || h2over;
    int tg, sc;
    if (M == 0) {
        if (kOTF) tg = RSK_TARGET_NO_CANDIDATE, sc = -1;  // set below from the scanned zero case
        else tg = zero_target(load_zc(a.zc_cnt, a.zc_key, s), sc);
    } else {
        sc = M;
        const unsigned bk = w1 >> 16;
        const bool tie = w2 != 0u;
        tg = !tie ? cand_node(w1) : (bk >= 2u ? cand_node(w1) : RSK_TARGET_NONE);
        slow = slow || (tie && code_inexact(bk) && (w2 >> 16) == bk);
    }
    if (kOTF) {  // lanes that reach no candidate node: their scenario's zero case, scanned
        unsigned long long zm = __builtin_amdgcn_ballot_w64(M == 0);
        while (zm) {
            const int ln = __builtin_ctzll(zm);
            zm &= zm - 1ull;
            int sx;
            const int tx = zero_target(side_zc_scan(a, min(s0 + ln, a.S - 1), lane), sx);
            tg = lane == ln ? tx : tg;
            sc = lane == ln ? sx : sc;
        }
    }
    // rare: deviation lists that overflowed, equal inexact codes at the top —
    // the wave recounts those scenarios exactly, one at a time (the table and
    // the deviation lists are scratch from here on)
    unsigned long long sm = __builtin_amdgcn_ballot_w64(slow);
    if (sm && !(RSK_ABL(a) & 1)) {
        while (sm) {
            const int ln = __builtin_ctzll(sm);
            sm &= sm - 1ull;
            int sx;
            const int tx = side_exact<kOff32, kOTF>(a, tb, dl, 64 * K, nb, d, min(s0 + ln, a.S - 1), lane, H, sx, B);
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

}  // namespace rsk
