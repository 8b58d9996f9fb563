// Host-only sanitizer driver (tests/test_asan.py).  Built by
// `make -C kubernetes-rescheduling_amd/csrc asan` with g++ -fsanitize=address,
// undefined from librsk's host sources that take caller input: the µBench
// workmodel reader (rsk_workmodel.cpp), the quantity parser (rsk_snapshot.cpp)
// and the CAR plan builder (rsk_plan.cpp).  No device code is involved.
//
//   rsk_asan wm FILE         parse FILE from an exact-length heap copy (no NUL:
//                            any read past the end is an ASan report), then
//                            load it through the mmap path; print the sizes
//   rsk_asan qty FILE KIND   one quantity string per line, KIND cpu | mem
//   rsk_asan plan P SEED     random CSRs (duplicates, self edges, empty rows,
//                            hubs up to 5,000 neighbours, row subsets) through
//                            the plan builder at both light_max values; checks
//                            that every row is routed exactly once
// Exit 0 when every call returned (RSK_OK or a clean error status); the
// sanitizers abort the process on any finding (-fno-sanitize-recover).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "rsk.h"
#include "rsk_plan.h"

static std::string slurp(const char *path) {
    FILE *f = std::fopen(path, "rb");
    if (!f) { std::perror(path); std::exit(2); }
    std::string s;
    char buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    std::fclose(f);
    return s;
}

static int run_wm(const char *path) {
    const std::string text = slurp(path);
    char *exact = static_cast<char *>(std::malloc(text.size() ? text.size() : 1));
    std::memcpy(exact, text.data(), text.size());
    for (int pass = 0; pass < 2; ++pass) {
        rsk_workmodel *wm = nullptr;
        const int rc = pass == 0 ? rsk_workmodel_parse(exact, (int64_t)text.size(), &wm) : rsk_workmodel_load(path, &wm);
        if (rc != RSK_OK) {
            std::printf("wm pass %d: status %d (%s)\n", pass, rc, rsk_last_error());
            continue;
        }
        int32_t P = 0;
        int64_t nnz = 0, nb = 0;
        rsk_workmodel_sizes(wm, &P, &nnz, &nb);
        std::vector<int32_t> rp((size_t)P + 1), ci((size_t)(nnz ? nnz : 1));
        std::vector<char> names((size_t)(nb ? nb : 1));
        rsk_workmodel_csr(wm, rp.data(), ci.data());
        rsk_workmodel_names(wm, names.data());
        rsk_workmodel_destroy(wm);
        std::printf("wm pass %d: P=%d nnz=%lld name_bytes=%lld\n", pass, P, (long long)nnz, (long long)nb);
    }
    std::free(exact);
    return 0;
}

static int run_qty(const char *path, const char *kind) {
    const std::string text = slurp(path);
    std::vector<int64_t> offs{0};
    std::string cat;
    size_t at = 0;
    while (at <= text.size()) {
        size_t e = text.find('\n', at);
        if (e == std::string::npos) e = text.size();
        if (e > at || e < text.size()) {
            cat.append(text, at, e - at);
            offs.push_back((int64_t)cat.size());
        }
        at = e + 1;
    }
    const int64_t n = (int64_t)offs.size() - 1;
    char *exact = static_cast<char *>(std::malloc(cat.size() ? cat.size() : 1));  // no NUL terminator
    std::memcpy(exact, cat.data(), cat.size());
    std::vector<int64_t> out((size_t)(n ? n : 1));
    std::vector<uint8_t> st((size_t)(n ? n : 1));
    const int rc = rsk_parse_quantities(exact, offs.data(), n, std::strcmp(kind, "mem") == 0 ? RSK_QTY_MEM : RSK_QTY_CPU,
                                        out.data(), st.data());
    int bad = 0;
    for (int64_t i = 0; i < n; ++i) bad += st[(size_t)i] != 0;
    std::printf("qty %s: status %d, %lld strings, %d left to the Python restatement\n", kind, rc, (long long)n, bad);
    std::free(exact);
    return 0;
}

static int run_plan(int P, unsigned seed) {
    std::mt19937 rng(seed);
    for (int round = 0; round < 6; ++round) {
        std::vector<int32_t> rp{0}, ci;
        for (int p = 0; p < P; ++p) {
            int d = (int)(rng() % 6);
            if (rng() % 50 == 0) d = 20 + (int)(rng() % 40);             // 17..64
            if (rng() % 400 == 0) d = 65 + (int)(rng() % 700);            // hubs
            if (p == 3 && round >= 3) d = 5000;                           // a row above kHubMax
            for (int j = 0; j < d; ++j) ci.push_back((int32_t)(rng() % (unsigned)P));
            if (d && rng() % 7 == 0) ci.push_back(ci.back());             // a duplicate
            if (rng() % 11 == 0) ci.push_back(p);                         // a self edge
            rp.push_back((int32_t)ci.size());
        }
        std::vector<int32_t> rows;
        const bool subset = round % 2 == 1;
        if (subset)
            for (int p = 0; p < P; ++p)
                if (rng() % 3 == 0) rows.push_back(p);
        const int Q = subset ? (int)rows.size() : P;
        for (int light : {rsk::kLightMax, rsk::kPairMax}) {
            rsk::PlanHost h;
            const int rc = rsk::plan_build_host(rp.data(), ci.data(), P, subset ? rows.data() : nullptr, Q, light,
                                                rsk::kTileOwners * 80 / rsk::kTileRows, 80, &h);
            if (rc != RSK_OK) { std::printf("plan: status %d (%s)\n", rc, rsk::last_error()); return 1; }
            // every plan row routed exactly once: tile records + side rows
            std::vector<int> seen((size_t)Q, 0);
            for (int t = 0; t < h.T; ++t) {
                const int *m = h.meta.data() + (size_t)t * rsk::kMetaW;
                for (int c = 0; c < rsk::kNumCls; ++c)
                    for (int j = 0; j < m[4 + c]; ++j) ++seen[(size_t)h.recs[(size_t)(m[2] + m[4 + rsk::kNumCls + c] + rsk::kClsW[c] * j)]];
            }
            for (size_t k = 0; k < h.side_items.size(); k += 4) ++seen[(size_t)h.side_items[k]];
            for (int i = 0; i < Q; ++i)
                if (seen[(size_t)i] != 1) { std::printf("plan: row %d routed %d times\n", i, seen[(size_t)i]); return 1; }
            std::printf("plan P=%d Q=%d light=%d: T=%d side=%zu big=%d\n", P, Q, light, h.T, h.side_items.size() / 4,
                        h.n_big);
        }
    }
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 3 && !std::strcmp(argv[1], "wm")) return run_wm(argv[2]);
    if (argc >= 4 && !std::strcmp(argv[1], "qty")) return run_qty(argv[2], argv[3]);
    if (argc >= 4 && !std::strcmp(argv[1], "plan")) return run_plan(std::atoi(argv[2]), (unsigned)std::atoi(argv[3]));
    std::fprintf(stderr, "usage: rsk_asan wm FILE | qty FILE cpu|mem | plan P SEED\n");
    return 2;
}
