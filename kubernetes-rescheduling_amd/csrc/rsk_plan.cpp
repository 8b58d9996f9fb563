// rsk_plan.cpp — the CAR plan's host builder (no device code).
//
// From the relation CSR (rescheduling.py:183-195 walks every pod's relation
// list) this builds, once per graph:
//   1. the CSR deduplicated, self edges dropped (the evicted pod is off the
//      cluster, main.py:73; relation lists never double count);
//   2. a locality order of the pods (DFS, smallest subtree first);
//   3. the routing of every plan row by degree: LDS tiles (deg <= light_max),
//      the compact path's side rows (deg > light_max, by class), the wide
//      path's mid / hub / big rows.
// rsk_car.hip uploads the result; tests/test_asan.py runs this file under
// AddressSanitizer + UBSan through the `make asan` driver.
#include <algorithm>
#include <unordered_map>
#include <vector>

#include "rsk_plan.h"

namespace rsk {
namespace {

int heavy_class(int d) {
    for (int c = 0; c < kNumHeavy; ++c)
        if (d <= kHeavyMax[c]) return c;
    return -1;
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


int light_class(int d) {  // d = 0 rows go to the D = 4 class: all entries masked -> zero case
    if (d == 1) return 0;
    if (d == 2) return 1;
    if (d <= 4) return 2;
    if (d <= 8) return 3;
    if (d <= 16) return 4;
    return 5;
}

// Tiles: rows in DFS order are packed greedily into tiles of at most
// owners_cap rows whose distinct neighbours (the image rows) number at most
// rows_cap and whose records fit kTileRecInts.  On a relation tree in DFS order
// a tile's image is essentially its own pods plus a few external neighbours.
struct TileBuilder {
    std::vector<int> img_pods, meta, recs;
    std::vector<int> cur_pods;
    std::unordered_map<int, int> cur_slot;
    std::vector<int> cur_rec[kNumCls];
    int cur_rows = 0, cur_rec_ints = 0, T = 0, rmax = 0, recmax = 0, n_sorted = 0, n_rows = 0;
    int owners_cap = kTileOwners, rows_cap = kTileRows;
    int64_t img_total = 0;

    bool fits(const int *nb, int d) const {
        if (cur_rows >= owners_cap) return false;
        if (cur_rec_ints + kClsW[light_class(d)] + 2 > kTileRecInts) return false;  // + worst-case padding
        int fresh = 0;
        for (int j = 0; j < d; ++j) fresh += !cur_slot.count(nb[j]);  // nb is deduplicated
        return (int)cur_pods.size() + fresh <= rows_cap;
    }
    void add(int oi, const int *nb, int d) {
        int lr[kLightMax];
        for (int j = 0; j < d; ++j) {
            auto it = cur_slot.find(nb[j]);
            if (it == cur_slot.end()) {
                it = cur_slot.emplace(nb[j], (int)cur_pods.size()).first;
                cur_pods.push_back(nb[j]);
            }
            lr[j] = it->second;
        }
        const int c = light_class(d);
        auto &e = cur_rec[c];
        const size_t o = e.size();
        e.resize(o + kClsW[c], 0);
        e[o] = oi;
        if (c == 0) {
            e[o + 1] = lr[0];
        } else if (c == 1) {
            e[o + 1] = lr[0] | (lr[1] << 16);
        } else {
            // [oi, d, rows...]; the sorted classes (c >= 5) start their rows at
            // int 4 so the scorer reads them as aligned int4 words
            const int r0 = c >= 5 ? 4 : 2;
            e[o + 1] = d;
            for (int j = 0; j < d; ++j) e[o + r0 + j / 2] |= lr[j] << ((j & 1) * 16);
        }
        n_sorted += c >= 5;
        ++n_rows;
        cur_rec_ints += kClsW[c];
        ++cur_rows;
    }
    void close() {
        if (!cur_rows) return;
        // every tile stages >= 1 image row (a tile of deg-0 rows stages pod 0,
        // which no record reads)
        if (cur_pods.empty()) cur_pods.push_back(0);
        const int rec_off = (int)recs.size();
        int m[kMetaW] = {};
        for (int c = 0; c < kNumCls; ++c) {
            // every class starts 16-B aligned (int4 record reads, 16-B scalar block loads)
            while ((recs.size() - rec_off) % 4) recs.push_back(0);
            m[4 + kNumCls + c] = (int)recs.size() - rec_off;
            m[4 + c] = (int)cur_rec[c].size() / kClsW[c];
            recs.insert(recs.end(), cur_rec[c].begin(), cur_rec[c].end());
            cur_rec[c].clear();
        }
        while ((recs.size() - rec_off) % 4) recs.push_back(0);
        const int rec_ints = (int)recs.size() - rec_off;
        m[0] = (int)img_pods.size();
        m[1] = (int)cur_pods.size();
        m[2] = rec_off;
        m[3] = rec_ints;
        meta.insert(meta.end(), m, m + kMetaW);
        img_pods.insert(img_pods.end(), cur_pods.begin(), cur_pods.end());
        img_total += (int64_t)cur_pods.size();
        rmax = std::max(rmax, (int)cur_pods.size());
        recmax = std::max(recmax, rec_ints);
        ++T;
        cur_pods.clear();
        cur_slot.clear();
        cur_rows = 0;
        cur_rec_ints = 0;
    }
};

}  // namespace

int plan_build_host(const int32_t *row_ptr, const int32_t *col_idx, int32_t P, const int32_t *rows, int32_t Q,
                    int light_max, int owners_cap, int rows_cap, PlanHost *out) {
    RSK_CHECK(out && row_ptr && P >= 0 && Q >= 0 && light_max >= 1 && light_max <= kLightMax && owners_cap >= 1 &&
                  rows_cap >= light_max,
              "plan_build_host: bad arguments");
    PlanHost &h = *out;
    // deduplicated adjacency without self edges (the evicted pod is off the cluster)
    std::vector<int> &rp = h.rp, &ci = h.ci;
    rp.assign((size_t)P + 1, 0);
    ci.clear();
    ci.reserve(P ? row_ptr[P] : 0);
    std::vector<int> nb;
    for (int p = 0; p < P; ++p) {
        nb.assign(col_idx + row_ptr[p], col_idx + row_ptr[p + 1]);
        std::sort(nb.begin(), nb.end());
        nb.erase(std::unique(nb.begin(), nb.end()), nb.end());
        nb.erase(std::remove(nb.begin(), nb.end(), p), nb.end());
        ci.insert(ci.end(), nb.begin(), nb.end());
        rp[p + 1] = (int)ci.size();
        h.ddmax = std::max(h.ddmax, rp[p + 1] - rp[p]);
    }
    const std::vector<int> order = locality_order(P, rp, ci);
    std::vector<int> pos(P);
    for (int k = 0; k < P; ++k) pos[order[k]] = k;

    std::vector<int> light;  // row indices i with deg <= light_max, to be tiled in DFS order
    std::vector<std::vector<int>> midr(kNumMid);
    std::vector<std::vector<HeavyItem>> hitems(kNumHeavy);
    std::vector<int> hcol, pcol;
    std::vector<HeavyItem> sitems;  // compact path: every side row
    for (int i = 0; i < Q; ++i) {
        const int p = rows ? rows[i] : i;
        const int d = rp[p + 1] - rp[p];
        h.max_deg = std::max(h.max_deg, d);
        const int *nbp = ci.data() + rp[p];
        if (d <= light_max) {
            light.push_back(i);
        } else if (d <= kMidMax) {
            const int b = d <= 32 ? 0 : 1;  // bucket 0 only in the N >= kPackMaxN variant
            auto &e = midr[b];
            const size_t o = e.size();
            e.resize(o + kMidW[b], 0);
            e[o] = i;
            e[o + 1] = d;
            for (int j = 0; j < d; ++j) e[o + 2 + j] = nbp[j];
            h.n_mid[b] += 1;
        } else if (d <= kHubMax) {
            const int c = heavy_class(d);
            hitems[c].push_back({i, (int)hcol.size(), d, 0});
            hcol.insert(hcol.end(), nbp, nbp + d);
            h.n_heavy[c] += 1;
            h.heavy_dmax[c] = std::max(h.heavy_dmax[c], d);
        }
        if (d > light_max) {  // compact path: every side row through car_side16
            sitems.push_back({i, (int)pcol.size(), d, 0});
            pcol.insert(pcol.end(), nbp, nbp + d);
        }
    }
    std::stable_sort(light.begin(), light.end(), [&](int x, int y) {
        return pos[rows ? rows[x] : x] < pos[rows ? rows[y] : y];
    });
    // one tile list: every row of degree <= light_max in DFS order (the 17..32
    // rows included: the tile kernel's register-light counting walk scores them)
    TileBuilder tb;
    tb.owners_cap = owners_cap;
    tb.rows_cap = rows_cap;
    for (int i : light) {
        const int p = rows ? rows[i] : i;
        const int d = rp[p + 1] - rp[p];
        const int *nbp = ci.data() + rp[p];
        if (!tb.fits(nbp, d)) tb.close();
        tb.add(i, nbp, d);
    }
    tb.close();
    h.T = tb.T;
    h.rmax = tb.rmax;
    h.recmax = tb.recmax;
    h.n_tile_rows = (int)light.size();
    h.n_sorted_rows = tb.n_sorted;
    h.img_rows_total = tb.img_total;
    {
        std::vector<char> seen(P, 0);
        for (int q : tb.img_pods) seen[q] = 1;
        h.img_pods_distinct = std::count(seen.begin(), seen.end(), 1);
    }
    h.n_recs = std::max<int64_t>(4, (int64_t)tb.recs.size());
    // 64 zero ints past the last blob: the 64-scenario tile kernel reads record
    // blocks through the scalar cache without clamping them
    if (tb.T > 0) tb.recs.resize(tb.recs.size() + 64, 0);
    h.img_pods.swap(tb.img_pods);
    h.meta.swap(tb.meta);
    h.recs.swap(tb.recs);
    for (int b = 0; b < kNumMid; ++b) h.mid[b].swap(midr[b]);
    for (int c = 0; c < kNumHeavy; ++c) h.heavy_items[c].swap(hitems[c]);
    h.hcol.swap(hcol);
    {   // car_side16 classes: all side rows, degree descending; class c holds
        // the rows of degree (kSideMax[c - 1], kSideMax[c]] at [side_beg[c], side_end[c])
        std::vector<HeavyItem> &all = sitems;
        std::stable_sort(all.begin(), all.end(), [](const HeavyItem &x, const HeavyItem &y) { return x.d > y.d; });
        {   // the wide path's rows above kHubMax (degree descending: a prefix)
            int nb = 0;
            while (nb < (int)all.size() && all[nb].d > kHubMax) ++nb;
            h.n_big = nb;
            h.big_dmax = nb ? all[0].d : 0;
        }
        int end = (int)all.size();
        for (int c = 0; c < kNumSide; ++c) {
            int b = end;
            while (b > 0 && all[b - 1].d <= kSideMax[c]) --b;
            h.side_beg[c] = b;
            h.side_end[c] = end;
            h.side_dmax[c] = b < end ? all[b].d : 0;
            end = b;
        }
        {   // cumulative distinct neighbour pods: the images, then side classes 0, 1, ...
            std::vector<char> seen(P, 0);
            int64_t n = 0;
            for (int q : h.img_pods) n += !seen[q], seen[q] = 1;
            h.nb_distinct[0] = n;
            for (int c = 0; c < kNumSide; ++c) {
                for (int k = h.side_beg[c]; k < h.side_end[c]; ++k)
                    for (int j = 0; j < all[k].d; ++j) {
                        const int q = pcol[all[k].rb + j];
                        n += !seen[q], seen[q] = 1;
                    }
                h.nb_distinct[c + 1] = n;
            }
        }
        h.side_items.reserve(all.size() * 4);
        for (const HeavyItem &x : all) h.side_items.insert(h.side_items.end(), {x.oi, x.rb, x.d, 0});
    }
    h.pcol.swap(pcol);
    return RSK_OK;
}

}  // namespace rsk
