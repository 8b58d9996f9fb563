// rsk_common.h — shared internals of librsk.so (HIP, gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "rsk.h"
#include "rsk_host.h"

namespace rsk {

#define RSK_HIP(expr)                                                                    \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess) {                                                          \
            ::rsk::set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(_e)); \
            return RSK_EHIP;                                                             \
        }                                                                                \
    } while (0)

// Grow-only device scratch buffer owned by a context or plan.
struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
    int reserve(size_t need);
    void release();
    template <class T> T *as() const { return static_cast<T *>(ptr); }
};

// Grow-only pinned host buffer mapped into the device's address space: the
// single-call (S = 1) host paths write their inputs here and kernels read them
// and write their results straight through `dev` (no staging copies).
struct PinBuf {
    void *host = nullptr, *dev = nullptr;
    size_t bytes = 0;
    int reserve(size_t need);
    void release();
};

struct EventPair {
    hipEvent_t start, stop;
};

}  // namespace rsk

struct rsk_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    bool profiling = false;
    std::string profile_only;            // time only this kernel name (empty: all)
    std::vector<hipEvent_t> event_pool;  // recycled timing events
    std::map<std::string, std::vector<rsk::EventPair>> pending;
    std::map<std::string, std::pair<double, int64_t>> totals;
    static constexpr int kAux = 3;  // side streams (with ctx->stream: 4 hardware queues)
    hipStream_t aux[kAux] = {};     // CAR mid/hub rows, beside the tile kernel or ahead of it
    hipEvent_t fork = nullptr, join[kAux] = {};
    rsk::DevBuf host_stage[12];  // device staging for host-pointer calls
    rsk::DevBuf work[6];         // per-call device workspace
    rsk::PinBuf pin;             // mapped pinned host memory of the single-call paths
    rsk::PinBuf errw;            // device error word (mapped pinned host memory, rsk::dev_err)
    std::vector<uint8_t> pinned;  // host scratch
};

namespace rsk {

// Event-bracketed launches: `name` accumulates kernel time when profiling is on.
struct ScopedTimer {
    rsk_ctx *ctx;
    const char *name;
    hipStream_t stream;
    hipEvent_t a = nullptr, b = nullptr;
    ScopedTimer(rsk_ctx *c, const char *n, hipStream_t s = nullptr);
    ~ScopedTimer();
};

// Fork / join of the context's first k side streams around work that may
// overlap the main stream: fork() makes aux[0..k) wait for everything queued on
// ctx->stream so far; join() makes ctx->stream wait for everything queued on them.
int aux_fork(rsk_ctx *ctx, int k);
int aux_join(rsk_ctx *ctx, int k);

int activate(rsk_ctx *ctx);

// ---- device error word (the r05v fault class) ----
// A launch whose write offsets come from an earlier launch's counts (nr_place's
// records, list_fill's base lists) checks every offset against its buffer's
// capacity; on overflow it skips the store and writes its bit into the
// context's error word, a plain vector store into mapped pinned host memory
// (nothing is written on the common path).  activate() — the first step of
// every entry point — and rsk_ctx_synchronize() read the word: a set bit is
// RSK_EHIP naming the kernel.  Host-pointer calls read it again after their own
// completion, so they report their own overflow; a device-pointer call's
// overflow is reported by the context's next call or synchronize.
enum DevErr : unsigned {
    kErrNrPlace = 1u,   // nr_place: a record offset at or past the record buffer
    kErrListFill = 2u,  // list_fill: a base-list offset at or past P
};
unsigned *dev_err(rsk_ctx *ctx);   // the word's device address (allocated on first use; null on failure)
int check_dev_err(rsk_ctx *ctx);   // RSK_EHIP (and clears the word) when a bit is set

// Host-pointer staging: copy `bytes` from host `src` into context slot `slot`
// and return the device pointer (or pass a device pointer straight through).
int stage_in(rsk_ctx *ctx, int slot, const void *src, size_t bytes, bool device, const void **out);
int stage_out(rsk_ctx *ctx, int slot, void *dst, size_t bytes, bool device, void **out);
int copy_back(rsk_ctx *ctx, void *host_dst, const void *dev_src, size_t bytes, bool device);

constexpr int kBlock = 256;

// Device-pointer launches of the per-node reductions (rsk_metrics.hip), shared
// by the public entry points and the multi-round loop (rsk_rounds.hip).
// `key_ws` is S u64 of scratch; every call queues on `stream` only.
int launch_cpu_pct(hipStream_t stream, const int *use, const int *cap, int N, int S, int *pct);
int launch_detect(hipStream_t stream, const int *pct, int N, int S, int threshold, uint8_t *hazard,
                  unsigned long long *key_ws, int *most);
int launch_pick_max_pod(hipStream_t stream, const int *assign, const int *pod_cpu, int P, int S, const int *most,
                        unsigned long long *key_ws, int *out_pod);
// key_ws[S] packed (cpu, ~pod) maxima -> pod index or -1 (the pick kernels' tail)
int launch_decode_first_max(hipStream_t stream, const unsigned long long *key, int S, int *out_pod);

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- u64 workspace slices (the r04p2 fault class) ----
// A 64-bit atomic on a word that is not 8-B aligned faults the GPU (r04p2: the
// plan's second zero-case half at S*12 + 4).  Every workspace layout that holds
// u64 words takes its slice offsets from the functions below, and the entry
// points run ws_check_u64() on the layout (and ws_check_ptr() on caller-owned
// u64 buffers) before any launch: a misaligned slice is RSK_EINVAL naming it.
constexpr int kBlkNodes = 64;  // nodes per detect block (the rounds loops' block maxima)
// the plan's zero-case words: two halves of zc_key[S] u64 + zc_cnt[S] int
inline size_t zc_half_bytes(int64_t S) { return ((size_t)S * 12 + 15) & ~(size_t)15; }
// a move workgroup's count table: 2H words of hash, then 8 words of which the
// first two hold the u64 best (car_move_one's red64); one area per workgroup
inline size_t move_tab_bytes(int64_t H) { return ((size_t)2 * H + 8) * 4; }
// block maxima [S][NB] u64 bm, [S][NB] u64 bz, [S][NB] int bc (blk / rows blk)
inline size_t blk_nb(int64_t N) { return (size_t)ceil_div(N, kBlkNodes); }
struct U64Slice {
    const char *name;
    uint64_t off;  // byte offset of the slice's first u64 within its buffer
};
constexpr int kMaxU64Slices = 12;
int ws_u64_layout(int64_t N, int64_t S, int64_t H, U64Slice *out);  // returns the count
int ws_check_u64(int64_t N, int64_t S, int64_t H);
int ws_check_ptr(const void *p, const char *name);

// One-launch CAR, a workgroup per (row, scenario) (rsk_rounds.hip): plan rows
// i = items[k * istride] for k < Q (items null: i = k) of the deduplicated CSR
// rp / ci (pod rows[i], or i), S scenarios, into out_target[i * S + s]; targets
// only, exact remaining CPU from cap / use (no node codes).
int launch_car_direct(hipStream_t st, const int *rp, const int *ci, const int *rows, int Q, const int *assign,
                      const int *use, const int *cap, const uint8_t *haz, int S, int N, int dmax, int *out_target,
                      DevBuf *scratch, const int *items = nullptr, int istride = 1);

}  // namespace rsk
