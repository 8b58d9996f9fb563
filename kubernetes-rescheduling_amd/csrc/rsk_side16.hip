// rsk_side16.hip — CAR for the side rows of the compact path (N <= 65535):
// every row above the tile classes (degree > light_max), any degree whose
// distinct-node table fits the LDS (side16_geometry).
//
// Reference: the score loop + argmax of `communication`,
// rescheduling.py:183-214 (see rsk_car.hip for the full statement).
//
// A work item is (row, chunk of 64 scenarios), lane = scenario, handled by a
// team of T waves (T = 1 for rows up to 256 neighbours: no barriers, the
// waves of a workgroup run independent items; T = 8 above, splitting the
// neighbour loads).  What-if scenarios share most of their assignment, so per
// neighbour j the team takes a pivot node p_j — the value most of the wave's
// lanes hold — and the row's histogram splits into a part every lane shares
// and a few per-lane deviations:
//   pass 1   the neighbours' assign rows (one 256-B row each, kB in flight) and
//            the lane's codes of those nodes: the lane's two largest distinct
//            candidate words (its answer whenever no candidate node occurs
//            twice), the pivot of each entry counted in an LDS hash keyed by
//            node (one parallel insert per batch), the lanes that deviate from
//            it appended to their own list (p_j << 16 | own node);
//   twice    the nodes that can occur twice in a lane — table entries counted
//            >= 2, and the lane's own deviation nodes — counted exactly (pivot
//            count - deviations away + deviations onto the node), their codes
//            gathered, into the best (count, two words) of count >= 2;
//   decide   as the tile scorers (rsk_car16.hip): count 0 -> the zero case, a
//            tie -> the larger code, None when it is code 1.
// Lanes whose deviation list overflowed, and ties between distinct nodes with
// the same inexact code, are recounted exactly, one scenario at a time by the
// whole wave (lanes = neighbours) — rare.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include "rsk_side16.h"

namespace rsk {

// kW waves per workgroup, teams of kT waves; blocks b and b + 8 share an XCD
// (a.xcd_per: workgroups per XCD run).
template <int kW, int kT, int kB, bool kOff32, bool kPipe, bool kGlobal = false, bool kOTF = false>
__global__ __launch_bounds__(64 * kW, (kT > 1 ? 1 : (kOTF ? 4 : 8))) void car_side16_kernel(SideArgs a) {
    int B = 0;
    if (kOTF) {  // the exact code window from max(cap), by this workgroup (no prep kernel before it)
        __shared__ int red[kW];
        B = max(0, block_capmax<64 * kW>(a.cap, a.N, red) - 32766);
    }
    if (kGlobal) {  // a capped grid strides over the items; work area = the resident block's slot
        static_assert(!kGlobal || kT == kW, "global work areas are per workgroup team");
        const int items = a.n_rows * a.nchunk;
        for (int blk = (int)blockIdx.x; blk < items; blk += (int)gridDim.x) {
            side16_block<kW, kT, kB, kOff32, kPipe, kGlobal, kOTF>(a, blk, (int)blockIdx.x, B);
            glob_fence(true);
            __syncthreads();  // every wave is done with the area before the next item clears it
        }
        return;
    }
    int blk = (int)blockIdx.x;
    if (a.xcd_per) blk = (int)(blockIdx.x & 7u) * a.xcd_per + (int)(blockIdx.x >> 3);
    side16_block<kW, kT, kB, kOff32, kPipe, kGlobal, kOTF>(a, blk, -1, B);
}

constexpr int kSideH2Cap = 2048;  // listed nodes counted >= 2 (e.g. degree 5000 over 6000 nodes: ~1200)

SideGeom side16_geometry(int dmax, int N, int T) {
    if (T <= 0) {  // one wave up to 256 neighbours, 8-wave teams up to 1024, 16 above while the table fits
        if (dmax <= 256) return side16_geometry(dmax, N, 1);
        if (dmax <= 1024) return side16_geometry(dmax, N, 8);
        const SideGeom g = side16_geometry(dmax, N, 16);
        return g.lds_team <= 160 * 1024 ? g : side16_geometry(dmax, N, 8);
    }
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
    g.T = T;
    // neighbour loads in flight per wave (with their code gathers: 2 kB VGPRs;
    // 4-wave teams live in the fused tile launch: <= 64 VGPRs; 16-wave teams:
    // <= 128)
    g.kB = dmax <= 32 ? 8 : (g.T == 8 ? 32 : 16);
    // words: tab H | dl 64 K (also the recount's cells) | ndl 64 | dummy 64 |
    // h2 1 + h2cap (the entries counted >= 2: at most min(Dc, dmax / 2); a
    // longer list sends the item to the exact recount; teams: bx 192 T after
    // the list is done) | fx 128 T (teams)
    g.off_dl = H;
    g.off_ndl = g.off_dl + 64 * g.K;
    g.off_dummy = g.off_ndl + 64;
    g.off_h2 = g.off_dummy + 64;
    g.h2cap = std::min(kSideH2Cap, std::min(g.Dc, std::max(1, dmax / 2)));
    const int h2words = std::max(1 + g.h2cap, g.T > 1 ? 192 * g.T : 0);
    g.off_fx = g.off_h2 + ((h2words + 3) & ~3);
    g.lds_team = ((size_t)(g.off_fx + (g.T > 1 ? 128 * g.T : 0)) * 4 + 15) & ~(size_t)15;
    // teams per workgroup: 4 single-wave teams while they fit 40 KiB, else fewer
    if (g.T > 1) g.W = g.T;
    else g.W = 4 * g.lds_team <= 40 * 1024 ? 4 : (2 * g.lds_team <= 80 * 1024 ? 2 : 1);
    return g;
}

void side16_apply_geometry(SideArgs &a, const SideGeom &g) {
    a.H = g.H;
    a.hshift = g.hshift;
    a.K = g.K;
    a.lds_team = (unsigned)g.lds_team;
    a.off_dl = g.off_dl;
    a.off_ndl = g.off_ndl;
    a.off_dummy = g.off_dummy;
    a.off_fx = g.off_fx;
    a.off_h2 = g.off_h2;
    a.h2cap = g.h2cap;
}

template <bool kOTF>
static int launch_side16_t(hipStream_t stream, const SideArgs &a0, const SideGeom &g0, bool off32, DevBuf *scratch) {
    if (a0.n_rows == 0) return RSK_OK;
    // a table beyond the LDS: 8-wave teams with their work area in global memory
    const bool global = (size_t)(g0.T > 1 ? 1 : g0.W) * g0.lds_team > 160 * 1024;
    const SideGeom g = global ? side16_geometry(g0.dmax, g0.Dc, 8) : g0;
    const size_t lds = global ? 0 : (size_t)(g.T > 1 ? 1 : g.W) * g.lds_team;
    SideArgs a = a0;
    side16_apply_geometry(a, g);
    const int64_t items = (int64_t)a.n_rows * a.nchunk;
    RSK_CHECK(items < INT32_MAX / 8, "side grid too large");
    const int teams = g.T > 1 ? 1 : g.W;
    const int64_t blocks_needed = ceil_div(items, teams);
    a.xcd_per = (int)ceil_div(blocks_needed, 8);
    const int64_t blocks = 8 * (int64_t)a.xcd_per;
    a.gscratch = nullptr;
    if (global) {
        RSK_CHECK(scratch, "a relation row of degree %d needs a %zu-B table: no scratch", g.dmax, g.lds_team);
        // one work area per resident workgroup, not per item: at most 1024
        // workgroups (4 per CU) and 256 MiB of areas; they stride over the items
        const int64_t gblocks = std::max<int64_t>(1, std::min<int64_t>({items, 1024, (int64_t)((256u << 20) / g.lds_team)}));
        RSK_TRY(scratch->reserve((size_t)gblocks * g.lds_team));
        a.gscratch = scratch->as<unsigned>();
        using KG = void (*)(SideArgs);
        const KG kg = off32 ? &car_side16_kernel<8, 8, 32, true, false, true, kOTF>
                            : &car_side16_kernel<8, 8, 32, false, false, true, kOTF>;
        kg<<<dim3((unsigned)gblocks), dim3(64 * 8), 0, stream>>>(a);
        RSK_HIP(hipGetLastError());
        return RSK_OK;
    }
    using K = void (*)(SideArgs);
#define RSK_SIDE_P(W, T, B, O) (&car_side16_kernel<W, T, B, O, true, false, kOTF>)
#define RSK_SIDE_O(W, T, B) (off32 ? RSK_SIDE_P(W, T, B, true) : RSK_SIDE_P(W, T, B, false))
#define RSK_SIDE_W(W) (g.kB == 8 ? RSK_SIDE_O(W, 1, 8) : RSK_SIDE_O(W, 1, 16))
    RSK_CHECK(g.T == 1 || g.T == 8 || g.T == 16, "side teams of %d waves are not built", g.T);
    const K kern = g.T == 16 ? RSK_SIDE_O(16, 16, 16)
                 : g.T == 8  ? RSK_SIDE_O(8, 8, 32)
                             : (g.W == 4 ? RSK_SIDE_W(4) : g.W == 2 ? RSK_SIDE_W(2) : RSK_SIDE_W(1));
#undef RSK_SIDE_W
#undef RSK_SIDE_O
#undef RSK_SIDE_P
    if (lds > 64 * 1024)
        RSK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds));
    kern<<<dim3((unsigned)blocks), dim3(64 * g.W), lds, stream>>>(a);
    RSK_HIP(hipGetLastError());
    return RSK_OK;
}

int launch_side16(hipStream_t stream, const SideArgs &a, const SideGeom &g, bool off32, DevBuf *scratch) {
    return launch_side16_t<false>(stream, a, g, off32, scratch);
}

int launch_side16_otf(hipStream_t stream, const SideArgs &a, const SideGeom &g, bool off32, DevBuf *scratch) {
    RSK_CHECK(a.haz && a.cap && a.use, "on-the-fly side rows need cap, use and hazard");
    return launch_side16_t<true>(stream, a, g, off32, scratch);
}

}  // namespace rsk
