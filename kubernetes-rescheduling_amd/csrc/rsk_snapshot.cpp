// Kubernetes quantity strings -> integers, in bulk, host C++
// (cluster_monitoring snapshot replay; the Python
// restatement and the fallback for rare spellings is rsk/snapshot.py).
//
// The reference converts every metrics-server / node-status quantity with
// unit_convertion.py:1-32:
//   cpu  "<x>m" -> int(float(x))              (truncation toward zero)
//        "<x>n" -> round(float(x) / 1e6)      (round-half-even on the double)
//        "<x>u" -> round(float(x) / 1000)
//        "<x>"  -> round(float(x) * 1000)
//   mem  "<x>Ki|Mi|Gi|Ti|Pi|Ei" -> int(float(x) * 1024^k), else int(float(x))
// after str.strip().  Python's float() is correctly rounded, as is strtod in
// the C locale; nearbyint() under the default rounding mode is round-half-even,
// as is Python's round(); the 1024^k factors are exact doubles.  So every
// string in the plain decimal grammar below converts bit-identically here.
// Anything else (underscores, inf/nan, non-ASCII, unusual whitespace, results
// outside int64, malformed text that must raise the reference's exception) is
// flagged status 1 and converted by the Python restatement, so the whole
// function is exact by construction.
#include <locale.h>

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "rsk_host.h"

namespace {

inline bool ascii_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

// Trim ASCII whitespace; false if the text holds a byte Python's str.strip()
// might treat differently (>= 0x80: Unicode spaces; 0x1c-0x1f: separators).
inline bool trim(const char *&b, const char *&e) {
    for (const char *q = b; q < e; ++q) {
        unsigned char c = (unsigned char)*q;
        if (c >= 0x80 || (c >= 0x1c && c <= 0x1f)) return false;
    }
    while (b < e && ascii_space(*b)) ++b;
    while (e > b && ascii_space(e[-1])) --e;
    return true;
}

// [+-]? (d+ (. d*)? | . d+) ([eE] [+-]? d+)?  -> double.  False outside it.
bool parse_decimal(const char *b, const char *e, double *v) {
    if (!trim(b, e) || b == e || e - b > 120) return false;
    const char *q = b;
    if (*q == '+' || *q == '-') ++q;
    int ip = 0, fp = 0;
    while (q < e && *q >= '0' && *q <= '9') ++q, ++ip;
    if (q < e && *q == '.') {
        ++q;
        while (q < e && *q >= '0' && *q <= '9') ++q, ++fp;
    }
    if (ip + fp == 0) return false;
    if (q < e && (*q == 'e' || *q == 'E')) {
        ++q;
        if (q < e && (*q == '+' || *q == '-')) ++q;
        int xp = 0;
        while (q < e && *q >= '0' && *q <= '9') ++q, ++xp;
        if (xp == 0) return false;
    }
    if (q != e) return false;
    char tmp[128];
    std::memcpy(tmp, b, (size_t)(e - b));
    tmp[e - b] = '\0';
    // the C locale whatever the host process set (Python's float() ignores LC_NUMERIC)
    static const locale_t c_loc = newlocale(LC_NUMERIC_MASK, "C", (locale_t)0);
    char *end = nullptr;
    double d = c_loc ? strtod_l(tmp, &end, c_loc) : std::strtod(tmp, &end);
    if (end != tmp + (e - b) || !std::isfinite(d)) return false;
    *v = d;
    return true;
}

// int(x) / round(x) into int64; false when Python's int would not fit.
inline bool to_i64(double x, int64_t *out) {
    if (!std::isfinite(x) || x >= 9223372036854775808.0 || x < -9223372036854775808.0) return false;
    *out = (int64_t)x;
    return true;
}

bool cpu_one(const char *b, const char *e, int64_t *out) {
    if (!trim(b, e) || b == e) return false;
    double v;
    switch (e[-1]) {
        case 'm':
            return parse_decimal(b, e - 1, &v) && to_i64(std::trunc(v), out);
        case 'n':
            return parse_decimal(b, e - 1, &v) && to_i64(std::nearbyint(v / 1000000.0), out);
        case 'u':
            return parse_decimal(b, e - 1, &v) && to_i64(std::nearbyint(v / 1000.0), out);
        default:
            return parse_decimal(b, e, &v) && to_i64(std::nearbyint(v * 1000.0), out);
    }
}

bool mem_one(const char *b, const char *e, int64_t *out) {
    if (!trim(b, e) || b == e) return false;
    double v;
    if (e - b >= 2 && e[-1] == 'i') {
        static const char kUnits[] = "KMGTPE";
        const char *u = std::strchr(kUnits, e[-2]);
        if (u && e[-2] != '\0') {
            double mult = std::ldexp(1.0, 10 * (int)(u - kUnits + 1));
            return parse_decimal(b, e - 2, &v) && to_i64(std::trunc(v * mult), out);
        }
    }
    return parse_decimal(b, e, &v) && to_i64(std::trunc(v), out);
}

}  // namespace

extern "C" int rsk_parse_quantities(const char *buf, const int64_t *offs, int64_t n, int32_t kind,
                                    int64_t *out, uint8_t *status) {
    RSK_CHECK(n >= 0, "n=%lld < 0", (long long)n);
    if (n == 0) return RSK_OK;
    RSK_CHECK(buf && offs && out && status, "null pointer");
    RSK_CHECK(kind == RSK_QTY_CPU || kind == RSK_QTY_MEM, "kind=%d", kind);
    for (int64_t i = 0; i < n; ++i)
        RSK_CHECK(offs[i] >= 0 && offs[i] <= offs[i + 1], "offsets not ascending at %lld", (long long)i);
    for (int64_t i = 0; i < n; ++i) {
        const char *b = buf + offs[i], *e = buf + offs[i + 1];
        int64_t v = 0;
        bool ok = kind == RSK_QTY_CPU ? cpu_one(b, e, &v) : mem_one(b, e, &v);
        out[i] = ok ? v : 0;
        status[i] = ok ? 0 : 1;
    }
    return RSK_OK;
}
