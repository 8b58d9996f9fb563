// rsk_slot.hip — CAR for the compact side rows of degree 33..128 (pivot
// class 0: the mid rows and the smallest hubs), S >= 64.
//
// Reference: the score loop + argmax of `communication`,
// rescheduling.py:183-214 (see rsk_car.hip for the full statement).
//
// One wave per (row, chunk of 64 scenarios), lane = scenario, four
// independent waves per workgroup.  Each wave owns an LDS slot table: H keys
// (node + 1, open addressing, shared by its 64 lanes — what-if scenarios
// mostly hold the same nodes, so the table stays near the row's degree) and
// H x 64 one-byte counters, slot-major so a lane's counter is byte
// (slot * 64 + lane).  Per neighbour entry a lane finds (or inserts) its
// node's slot, bumps its own counter and folds the new count into a running
// (count, code, -node) maximum: counts only grow, so the entries that raise a
// node to the final maximum M are exactly one per maximal node, and the
// running state ends as the tile scorers' walk does (M, nodes at M, best word,
// how many of them share its code).  Work per entry is a few VALU and three
// LDS accesses, against the per-lane bitonic sort (log^2 d compare-exchanges
// per entry) or the hub kernel's per-scenario wave reductions.
//
// Inserts are write-then-verify: the table is private to the wave, whose LDS
// accesses execute in order, so of the lanes writing one empty slot in one
// instruction exactly one key survives and the others probe on.  A table
// that fills (adversarial inputs: thousands of distinct nodes per row and
// chunk) flags the lanes that could not insert; they recount exactly from
// global memory.  Ties between distinct nodes with equal inexact codes read
// the exact remaining CPU of the nodes at M (their counts from the table).
#include <algorithm>
#include <climits>

#include "rsk_car.h"

namespace rsk {

constexpr int kSW = 4;   // waves (independent tasks) per workgroup
constexpr int kSB = 16;  // neighbour entries in flight per lane
#ifndef RSK_SLOT_LG
#define RSK_SLOT_LG 7
#endif

__device__ __forceinline__ unsigned slot_home(unsigned node, int lgH) {
    return ((node & 0xffffu) * 0x9E3779u) >> (24 - lgH) & ((1u << lgH) - 1u);  // node < 2^16: a 24-bit multiply
}

// Exact recount for a lane whose table overflowed: per entry the count of its
// node over the row (first occurrence only), the same running state.
__device__ __forceinline__ void slot_recount(const PivotArgs &a, const HeavyItem &it, unsigned sl, int &M, unsigned &bw,
                                          int &Rn, int &namb) {
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    M = 0; bw = 0u; Rn = 0; namb = 0;
    for (int e = 0; e < it.d; ++e) {
        const unsigned ne = min((unsigned)ld32(a.assign, (unsigned)a.hcol[it.rb + e] * S + sl), N);
        const unsigned c = ld16(a.code, ne * S + sl);
        if (c == kCodeHaz) continue;
        int cnt = 0;
        bool first = true;
        for (int i = 0; i < it.d; ++i) {
            const unsigned ni = min((unsigned)ld32(a.assign, (unsigned)a.hcol[it.rb + i] * S + sl), N);
            cnt += ni == ne;
            first = first && !(i < e && ni == ne);
        }
        if (!first) continue;
        const unsigned wv = (c << 16) | (ne ^ 0xffffu);
        const bool gt = cnt > M, eq = cnt == M;
        const unsigned kb = cell_code(bw);
        namb = gt ? 1 : (eq ? (c > kb ? 1 : (c == kb ? namb + 1 : namb)) : namb);
        bw = gt ? wv : (eq ? max(bw, wv) : bw);
        Rn = gt ? 1 : (eq ? Rn + 1 : Rn);
        M = gt ? cnt : M;
    }
}

template <int lgH>
__global__ __launch_bounds__(64 * kSW) void car_slot16_kernel(PivotArgs a, int nchunk) {
    constexpr int H = 1 << lgH;
    __shared__ unsigned keys_all[kSW][H];
    __shared__ __attribute__((aligned(16))) unsigned char cnt_all[kSW][H * 64];
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int task = (int)blockIdx.x * kSW + wave;
    if (task >= a.n_items * nchunk) return;  // whole wave; no workgroup barrier below
    const int item = task / nchunk, chunk = task - item * nchunk;
    const HeavyItem it = a.items[item];
    const unsigned S = (unsigned)a.S, N = (unsigned)a.N;
    const int s0 = chunk * 64;
    const unsigned sl = (unsigned)min(s0 + lane, a.S - 1);
    const char *__restrict__ asg = reinterpret_cast<const char *>(a.assign);
    const char *__restrict__ codeb = reinterpret_cast<const char *>(a.code);
    const unsigned S2 = 2u * S, sl2 = 2u * sl;
    unsigned *K = keys_all[wave];
    unsigned char *C = cnt_all[wave];
    for (int i = lane; i < H; i += 64) K[i] = 0u;
    for (int i = lane; i < H * 4; i += 64) reinterpret_cast<uint4 *>(C)[i] = make_uint4(0u, 0u, 0u, 0u);

    int M = 0, Rn = 0, namb = 0;
    unsigned bw = 0u;
    bool ovf = false;
    const cint_ptr nb = const_ptr(a.hcol) + it.rb;
    for (int e0 = 0; e0 < it.d; e0 += kSB) {
        unsigned v[kSB], cd[kSB];
#pragma unroll
        for (int u = 0; u < kSB; ++u) {
            const unsigned q = (unsigned)nb[min(e0 + u, it.d - 1)];
            v[u] = *reinterpret_cast<const unsigned *>(asg + ((q * S + sl) << 2));
        }
#pragma unroll
        for (int u = 0; u < kSB; ++u) {
            v[u] = min(v[u], N);  // outside [0, N): node N, code row N = 0 (no candidate)
            cd[u] = *reinterpret_cast<const unsigned short *>(codeb + __umul24(v[u], S2) + sl2);
        }
#pragma unroll
        for (int u = 0; u < kSB; ++u) {
            const unsigned n = v[u], c = cd[u], key = n + 1u;
            unsigned h = slot_home(n, lgH);
            bool pending = c != kCodeHaz && e0 + u < it.d, hit = false;  // past d: wave-uniform skip
            int probes = 0;
            while (__builtin_amdgcn_ballot_w64(pending)) {
                if (pending) {
                    asm volatile("" ::: "memory");  // other lanes write the table: no value forwarding
                    const unsigned k = K[h];
                    unsigned k2 = k;
                    if (k == 0u) {
                        K[h] = key;  // claim; the re-read sees the surviving writer
                        asm volatile("" ::: "memory");
                        k2 = K[h];
                    }
                    if (k2 == key) {
                        hit = true;
                        pending = false;
                    } else {
                        h = (h + 1u) & (H - 1u);
                        if (++probes == H) { ovf = true; pending = false; }
                    }
                }
            }
            if (hit) {
                const int cc = C[h * 64u + lane] + 1;
                C[h * 64u + lane] = (unsigned char)cc;
                const unsigned wv = (c << 16) | (n ^ 0xffffu);
                const bool gt = cc > M, eq = cc == M;
                const unsigned kb = cell_code(bw);
                namb = gt ? 1 : (eq ? (c > kb ? 1 : (c == kb ? namb + 1 : namb)) : namb);
                bw = gt ? wv : (eq ? max(bw, wv) : bw);
                Rn = gt ? 1 : (eq ? Rn + 1 : Rn);
                M = gt ? cc : M;
            }
        }
    }
    if (__builtin_amdgcn_ballot_w64(ovf)) {  // rare: exact recount of the overflowed lanes
        if (ovf) slot_recount(a, it, sl, M, bw, Rn, namb);
    }
    const unsigned bk = cell_code(bw);
    int t = Rn == 1 ? cand_node(bw) : (bk >= 2u ? cand_node(bw) : RSK_TARGET_NONE);
    const bool need = M > 0 && Rn > 1 && code_inexact(bk) && namb > 1;
    if (__builtin_amdgcn_ballot_w64(need)) {  // rare: equal inexact codes at the maximum
        if (need) {
            int br = INT_MIN, bn = INT_MAX;
            for (int e = 0; e < it.d; ++e) {
                const unsigned ne = min((unsigned)ld32(a.assign, (unsigned)nb[e] * S + sl), N);
                if (ne >= N || ld16(a.code, ne * S + sl) != bk) continue;
                int cnt = 0;  // exact count of ne (the table may have overflowed for this lane)
                for (int i = 0; i < it.d; ++i)
                    cnt += min((unsigned)ld32(a.assign, (unsigned)nb[i] * S + sl), N) == ne;
                if (cnt != M) continue;
                const int ex = a.cap[ne] - ld32(a.use, ne * S + sl);
                if (ex > br || (ex == br && (int)ne < bn)) { br = ex; bn = (int)ne; }
            }
            t = bn;
        }
    }
    int sc = M;
    if (M == 0) t = zero_target(load_zc(a.zc_cnt, a.zc_key, (int)sl), sc);
    if (s0 + lane < a.S) {
        const size_t o = (size_t)it.oi * S + (unsigned)(s0 + lane);
        a.out_target[o] = t;
        if (a.out_score) a.out_score[o] = sc;
    }
}

int launch_slot(hipStream_t stream, const PivotArgs &a, int dmax) {
    if (a.n_items == 0) return RSK_OK;
    RSK_CHECK(a.S >= 64, "slot kernel needs S >= 64 (S=%d)", a.S);
    const int nchunk = (int)ceil_div(a.S, 64);
    const int64_t tasks = (int64_t)nchunk * a.n_items;
    RSK_CHECK(tasks < INT32_MAX, "slot grid too large");
    const unsigned blocks = (unsigned)ceil_div(tasks, kSW);
    if (dmax <= 64) car_slot16_kernel<RSK_SLOT_LG><<<dim3(blocks), dim3(64 * kSW), 0, stream>>>(a, nchunk);
    else car_slot16_kernel<RSK_SLOT_LG + 1><<<dim3(blocks), dim3(64 * kSW), 0, stream>>>(a, nchunk);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

}  // namespace rsk
