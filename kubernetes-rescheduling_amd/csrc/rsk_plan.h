// rsk_plan.h — the CAR plan's host side (no HIP): routing constants, and the
// builder that turns a relation CSR into tiles, side rows and wide-path rows
// (rsk_plan.cpp).  rsk_car.hip uploads the result (rsk_car_plan_create); the
// `make asan` test driver runs the same builder under AddressSanitizer.
#pragma once

#include <cstdint>
#include <vector>

#include "rsk_host.h"

namespace rsk {

constexpr int kMaxDegree = 65535;                  // 16-bit counts in the side kernel's tables (rsk_side16.hip)
constexpr int kLightMax = 32;                      // LDS-tile rows: deg <= 32
constexpr int kPairMax = 16;                       // pairwise-count classes: deg <= 16
constexpr int kPackMaxN = (1 << 24) - 1;           // wide sorted classes pack node << 8 | image row: N < kPackMaxN
constexpr int kMidMax = 64;                        // mid rows: 33..64 (17..64 when N >= kPackMaxN)
constexpr int kNumMid = 2;                         // buckets D = 32, 64
constexpr int kMidW[kNumMid] = {36, 68};           // record ints: oi, d, nb[D], pad to x4
constexpr int kNumHeavy = 6;                       // hub classes: (64,128] (128,256] ... (2048,4096]
constexpr int kHeavyMax[kNumHeavy] = {128, 255, 512, 1024, 2048, 4096};  // <= 255: u8 counters
constexpr int kHeavyNJ[kNumHeavy] = {2, 4, 8, 16, 0, 0};  // register entries per lane (0: LDS re-reads)
constexpr int kHubMax = 4096;                      // wide hub kernel: rows up to this degree

// Light-row tiles.
constexpr int kTileOwners = 128;                   // max rows scored per tile
constexpr int kTileRows = 144;                     // max image rows (distinct neighbours) per tile (< 256)
constexpr int kTileRecInts = 1020;                 // max record ints per tile (+4: unit counter)
constexpr int kTileThreads = 256;
constexpr int kNumCls = 6;                         // degree classes d = 1, 2, {0,3,4}, 5-8, 9-16, 17-32
constexpr int kClsW[kNumCls] = {2, 2, 4, 8, 12, 20};  // record ints
constexpr int kMetaW = 16;                         // tile meta ints: img_off, nrows, rec_off, rec_ints, n[6], off[6]
static_assert(kTileRecInts <= kTileThreads * 4, "records are copied to LDS as one int4 per thread");

// Side rows of the compact path (rsk_side16.hip): every row above the tiles,
// in launches by degree class; a work item is (row, chunk of 64 scenarios).
constexpr int kNumSide = 6;
constexpr int kSideMax[kNumSide] = {32, 128, 512, 2048, 8192, kMaxDegree};  // class upper degrees

struct HeavyItem {
    int oi, rb, d, pad;
};

// Everything rsk_car_plan_create uploads, built on the host.
struct PlanHost {
    std::vector<int> rp, ci;      // the CSR deduplicated, self edges dropped
    int ddmax = 0;                // its largest degree (every pod)
    int max_deg = 0;              // the largest degree of the plan's rows
    // tiles: image pods, per-tile meta [T][kMetaW], record blobs (+ 64 zero ints when T > 0)
    std::vector<int> img_pods, meta, recs;
    int T = 0, rmax = 0, recmax = 0, n_tile_rows = 0, n_sorted_rows = 0;
    int64_t img_rows_total = 0, img_pods_distinct = 0, n_recs = 4;
    // mid rows of the wide path's kPairMax plans
    int n_mid[kNumMid] = {};
    std::vector<int> mid[kNumMid];
    // hub rows of the wide path (64 < deg <= kHubMax), by class
    int n_heavy[kNumHeavy] = {}, heavy_dmax[kNumHeavy] = {};
    std::vector<HeavyItem> heavy_items[kNumHeavy];
    std::vector<int> hcol;
    // every side row (deg > light_max), degree descending, as {oi, rb, d, 0};
    // class c at [side_beg[c], side_end[c]); rows above kHubMax a prefix (n_big)
    std::vector<int> side_items, pcol;
    int side_beg[kNumSide] = {}, side_end[kNumSide] = {}, side_dmax[kNumSide] = {};
    int n_big = 0, big_dmax = 0;
    // distinct neighbour pods of the tile rows, then + side classes 0, 1, ...
    int64_t nb_distinct[kNumSide + 1] = {};
};

// Rows `rows[0..Q)` (or every pod when rows is null) of the CSR (validated by
// the caller: monotone row_ptr, col_idx in [0, P)).
int plan_build_host(const int32_t *row_ptr, const int32_t *col_idx, int32_t P, const int32_t *rows, int32_t Q,
                    int light_max, int owners_cap, int rows_cap, PlanHost *out);

}  // namespace rsk
