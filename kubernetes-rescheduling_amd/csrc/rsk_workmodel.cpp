// µBench workmodel JSON -> service relation CSR, streaming, host C++
// (the Python restatement is rsk/workmodel.py).
//
// A workmodel (workmodelC.json) is one JSON object of services; each lists
// the services it calls in external_services[*].services.  The reference
// hard-codes the symmetrised graph (main.py:31-52, communicationcost.py:69-88):
// rel(s) = {services s calls} ∪ {services that call s}.  This reader makes one
// pass over the bytes with a small recursive-descent scanner: only the
// service keys and the strings under external_services[*].services are
// materialised, every other value is skipped, so a 1M-service file costs no
// DOM.  Output: services in file order (then callees that are never defined,
// in order of first mention), and the symmetrised, deduplicated CSR without
// self edges, columns ascending.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "rsk_host.h"

struct rsk_workmodel {
    std::vector<std::string> names;
    std::vector<int32_t> row_ptr, col_idx;
};

namespace {

struct Scanner {
    const char *p, *end, *begin;
    std::string err;
    std::string scratch;

    bool fail(const char *what) {
        if (err.empty()) err = std::string(what) + " at byte offset " + std::to_string((long long)(p - begin));
        return false;
    }
    void ws() {
        while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
    }
    bool eat(char c) {
        ws();
        if (p < end && *p == c) { ++p; return true; }
        return false;
    }
    // A JSON string; `out` views the file bytes, or `scratch` when it has escapes.
    bool str(std::string_view &out) {
        ws();
        if (p >= end || *p != '"') return fail("expected a string");
        const char *s = ++p;
        bool esc = false;
        while (p < end && *p != '"') {
            if (*p == '\\') { esc = true; ++p; }
            ++p;
        }
        if (p >= end) return fail("unterminated string");
        const char *e = p++;
        if (!esc) { out = std::string_view(s, (size_t)(e - s)); return true; }
        scratch.clear();
        for (const char *q = s; q < e; ++q) {
            if (*q != '\\') { scratch.push_back(*q); continue; }
            ++q;
            switch (*q) {
                case 'n': scratch.push_back('\n'); break;
                case 't': scratch.push_back('\t'); break;
                case 'r': scratch.push_back('\r'); break;
                case 'b': scratch.push_back('\b'); break;
                case 'f': scratch.push_back('\f'); break;
                case 'u': {  // BMP code point -> UTF-8 (surrogate pairs kept as two)
                    if (e - q < 5) return fail("bad \\u escape");
                    unsigned cp = (unsigned)std::stoul(std::string(q + 1, 4), nullptr, 16);
                    q += 4;
                    if (cp < 0x80) scratch.push_back((char)cp);
                    else if (cp < 0x800) { scratch.push_back((char)(0xc0 | (cp >> 6))); scratch.push_back((char)(0x80 | (cp & 0x3f))); }
                    else {
                        scratch.push_back((char)(0xe0 | (cp >> 12)));
                        scratch.push_back((char)(0x80 | ((cp >> 6) & 0x3f)));
                        scratch.push_back((char)(0x80 | (cp & 0x3f)));
                    }
                    break;
                }
                default: scratch.push_back(*q);
            }
        }
        out = scratch;
        return true;
    }
    // Skip any value without materialising it.
    bool skip() {
        ws();
        if (p >= end) return fail("expected a value");
        if (*p == '"') { std::string_view v; return str(v); }
        if (*p == '{' || *p == '[') {
            int depth = 0;
            while (p < end) {
                const char c = *p;
                if (c == '"') { std::string_view v; if (!str(v)) return false; continue; }
                ++p;
                if (c == '{' || c == '[') ++depth;
                else if (c == '}' || c == ']') { if (--depth == 0) return true; }
            }
            return fail("unterminated container");
        }
        while (p < end && *p != ',' && *p != '}' && *p != ']' && *p != ' ' && *p != '\n' && *p != '\r' && *p != '\t') ++p;
        return true;
    }
    // Iterate an object: f(key) consumes the value; returns false on error.
    template <class F>
    bool object(F &&f) {
        if (!eat('{')) return fail("expected an object");
        if (eat('}')) return true;
        do {
            std::string_view k;
            if (!str(k)) return false;
            std::string key(k);
            if (!eat(':')) return fail("expected ':'");
            if (!f(key)) return false;
        } while (eat(','));
        if (!eat('}')) return fail("expected ',' or '}'");
        return true;
    }
    template <class F>
    bool array(F &&f) {
        if (!eat('[')) return fail("expected an array");
        if (eat(']')) return true;
        do {
            if (!f()) return false;
        } while (eat(','));
        if (!eat(']')) return fail("expected ',' or ']'");
        return true;
    }
};

int build(const char *buf, size_t len, rsk_workmodel **out) {
    Scanner sc{buf, buf + len, buf, {}, {}};
    // Every name gets a provisional id on first sight (as a service key or as
    // a callee); the final order is json.load's: defined services in order of
    // their first key, then callees that are never defined, in order of first
    // mention (relation_from_workmodel in rsk/workmodel.py).
    std::unordered_map<std::string, int32_t> id;
    std::vector<std::string> seen;               // provisional id -> name
    std::vector<int32_t> def_order;              // provisional ids of defined services, first key order
    std::vector<char> defined;
    std::vector<std::vector<int32_t>> callees;   // by provisional id (last definition wins, as in json.load)
    std::vector<std::string> pending;
    auto intern = [&](const std::string &n) {
        auto it = id.find(n);
        if (it != id.end()) return it->second;
        const int32_t v = (int32_t)seen.size();
        id.emplace(n, v);
        seen.push_back(n);
        defined.push_back(0);
        callees.emplace_back();
        return v;
    };
    auto null_or = [&](auto &&f) {
        sc.ws();
        if (sc.p < sc.end && *sc.p == 'n') return sc.skip();
        return f();
    };
    const bool ok = sc.object([&](const std::string &svc) {
        pending.clear();
        const bool r = sc.object([&](const std::string &key) {
            if (key != "external_services") return sc.skip();
            return null_or([&] {
                return sc.array([&] {
                    return sc.object([&](const std::string &k2) {
                        if (k2 != "services") return sc.skip();
                        return null_or([&] {
                            return sc.array([&] {
                                std::string_view t;
                                if (!sc.str(t)) return false;
                                pending.emplace_back(t);
                                return true;
                            });
                        });
                    });
                });
            });
        });
        if (!r) return false;
        const int32_t me = intern(svc);
        if (!defined[(size_t)me]) { defined[(size_t)me] = 1; def_order.push_back(me); }
        std::vector<int32_t> c;
        c.reserve(pending.size());
        for (const auto &t : pending) c.push_back(intern(t));
        callees[(size_t)me] = std::move(c);
        return true;
    });
    if (!ok) RSK_CHECK(false, "workmodel: %s", sc.err.c_str());
    sc.ws();
    RSK_CHECK(sc.p == sc.end, "workmodel: trailing bytes after the top-level object");
    const int32_t P = (int32_t)seen.size();
    std::vector<int32_t> fin((size_t)P);
    auto *wm = new rsk_workmodel();
    wm->names.reserve((size_t)P);
    for (int32_t v : def_order) { fin[(size_t)v] = (int32_t)wm->names.size(); wm->names.push_back(seen[(size_t)v]); }
    for (int32_t v = 0; v < P; ++v)
        if (!defined[(size_t)v]) { fin[(size_t)v] = (int32_t)wm->names.size(); wm->names.push_back(seen[(size_t)v]); }
    std::vector<std::vector<int32_t>> adj((size_t)P);
    for (int32_t v = 0; v < P; ++v)
        for (int32_t t : callees[(size_t)v]) {
            const int32_t a = fin[(size_t)v], b2 = fin[(size_t)t];
            if (a == b2) continue;  // self calls: no relation edge
            adj[(size_t)a].push_back(b2);
            adj[(size_t)b2].push_back(a);
        }
    wm->row_ptr.assign(1, 0);
    for (auto &e : adj) {
        std::sort(e.begin(), e.end());
        e.erase(std::unique(e.begin(), e.end()), e.end());
        if (wm->col_idx.size() + e.size() >= (size_t)INT32_MAX) { delete wm; RSK_CHECK(false, "workmodel: too many relations"); }
        wm->col_idx.insert(wm->col_idx.end(), e.begin(), e.end());
        wm->row_ptr.push_back((int32_t)wm->col_idx.size());
    }
    *out = wm;
    return RSK_OK;
}

}  // namespace

extern "C" {

int rsk_workmodel_parse(const char *json, int64_t len, rsk_workmodel **out) {
    RSK_CHECK(json && len >= 0 && out, "bad arguments");
    return build(json, (size_t)len, out);
}

int rsk_workmodel_load(const char *path, rsk_workmodel **out) {
    RSK_CHECK(path && out, "bad arguments");
    const int fd = open(path, O_RDONLY);
    RSK_CHECK(fd >= 0, "workmodel: cannot open %s", path);
    struct stat st;
    if (fstat(fd, &st) != 0) { close(fd); RSK_CHECK(false, "workmodel: cannot stat %s", path); }
    const size_t len = (size_t)st.st_size;
    if (len == 0) { close(fd); return build("", 0, out); }
    void *m = mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    RSK_CHECK(m != MAP_FAILED, "workmodel: cannot map %s", path);
    (void)madvise(m, len, MADV_SEQUENTIAL);
    const int rc = build(static_cast<const char *>(m), len, out);
    munmap(m, len);
    return rc;
}

int rsk_workmodel_sizes(const rsk_workmodel *wm, int32_t *P, int64_t *nnz, int64_t *name_bytes) {
    RSK_CHECK(wm && P && nnz && name_bytes, "bad arguments");
    *P = (int32_t)wm->names.size();
    *nnz = (int64_t)wm->col_idx.size();
    int64_t b = 0;
    for (const auto &n : wm->names) b += (int64_t)n.size() + 1;
    *name_bytes = b;
    return RSK_OK;
}

int rsk_workmodel_csr(const rsk_workmodel *wm, int32_t *row_ptr, int32_t *col_idx) {
    RSK_CHECK(wm && row_ptr && (col_idx || wm->col_idx.empty()), "bad arguments");
    std::memcpy(row_ptr, wm->row_ptr.data(), wm->row_ptr.size() * 4);
    if (!wm->col_idx.empty()) std::memcpy(col_idx, wm->col_idx.data(), wm->col_idx.size() * 4);
    return RSK_OK;
}

int rsk_workmodel_names(const rsk_workmodel *wm, char *buf) {
    RSK_CHECK(wm && buf, "bad arguments");
    for (const auto &n : wm->names) {
        std::memcpy(buf, n.data(), n.size());
        buf += n.size();
        *buf++ = '\0';
    }
    return RSK_OK;
}

int rsk_workmodel_destroy(rsk_workmodel *wm) {
    delete wm;
    return RSK_OK;
}

}  // extern "C"
