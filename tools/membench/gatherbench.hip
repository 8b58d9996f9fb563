// gatherbench — the tile kernel's memory pattern without its arithmetic:
// per work item (128 rows, chunk of SL scenarios): read src[q][chunk] (SL
// words per row, lanes = scenarios), gather key[v][s] from a node-major table
// (KB bytes per key), write dst[row][chunk] = v ^ key.  Compares the current
// layout (SL 32, 4-B keys) with a compact one (SL 64, 2-B codes).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int SL, class K, int GATHER>
__global__ __launch_bounds__(256) void k(const int *__restrict__ src, const K *__restrict__ key, int *__restrict__ dst,
                                         int P, int S, int N, int nblk, const int *__restrict__ perm) {
    const int nch = S / SL;
    const int blk = blockIdx.x % nblk, c = blockIdx.x / nblk;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int RPW = 64 / SL;
    constexpr int U = 128 / (4 * RPW);  // rows per wave, all in flight
    int v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int r = (wave + 4 * u) * RPW + lane / SL;
        const int q = perm[min(blk * 128 + r, P - 1)];
        v[u] = src[(size_t)q * S + c * SL + lane % SL];
    }
    int kk[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        kk[u] = GATHER ? (int)key[(size_t)((unsigned)v[u] % N) * S + c * SL + lane % SL] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int r = (wave + 4 * u) * RPW + lane / SL;
        const int row = min(blk * 128 + r, P - 1);
        dst[(size_t)row * S + c * SL + lane % SL] = v[u] ^ kk[u];
    }
}

int main() {
    const int P = 100000, S = 4096, N = 5000;
    const size_t n = (size_t)P * S;
    int *src, *dst, *perm, *k32;
    short *k16;
    CK(hipMalloc(&src, n * 4));
    CK(hipMalloc(&dst, n * 4));
    CK(hipMalloc(&k32, (size_t)N * S * 4));
    CK(hipMalloc(&k16, (size_t)N * S * 2));
    std::vector<int> h(n);
    srand(3);
    // like the what-if batches: a pod's node is the same in ~99% of scenarios
    for (size_t i = 0; i < n; ++i) h[i] = (int)((i / S) * 2654435761u % N);
    for (size_t i = 0; i < n / 100; ++i) h[((size_t)rand() * 65536 + rand()) % n] = rand() % N;
    CK(hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(k32, 1, (size_t)N * S * 4));
    CK(hipMemset(k16, 1, (size_t)N * S * 2));
    std::vector<int> ph(P);
    for (int i = 0; i < P; ++i) ph[i] = i;
    for (int i = P - 1; i > 0; --i) std::swap(ph[i], ph[rand() % (i + 1)]);
    CK(hipMalloc(&perm, P * 4));
    CK(hipMemcpy(perm, ph.data(), P * 4, hipMemcpyHostToDevice));
    const int nblk = (P + 127) / 128;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](auto kern, const void *key, int SL, const char *name) {
        const int grid = nblk * (S / SL);
        for (int w = 0; w < 3; ++w) kern<<<grid, 256>>>(src, (decltype(nullptr))nullptr == nullptr ? 0 : 0, dst, P, S, N, nblk, perm);
        (void)key;
    };
    (void)run;
#define RUN(SL, K, G, KEYP, NAME)                                                               \
    {                                                                                           \
        const int grid = nblk * (S / SL);                                                       \
        for (int w = 0; w < 3; ++w) k<SL, K, G><<<grid, 256>>>(src, KEYP, dst, P, S, N, nblk, perm); \
        CK(hipEventRecord(a));                                                                  \
        for (int w = 0; w < 10; ++w) k<SL, K, G><<<grid, 256>>>(src, KEYP, dst, P, S, N, nblk, perm); \
        CK(hipEventRecord(b));                                                                  \
        CK(hipEventSynchronize(b));                                                             \
        float ms;                                                                               \
        CK(hipEventElapsedTime(&ms, a, b));                                                     \
        printf("%-34s %.3f ms\n", NAME, ms / 10);                                               \
    }
    RUN(32, int, 0, k32, "copy SL32 (no gather)");
    RUN(32, int, 1, k32, "copy SL32 + 4-B key gather");
    RUN(32, short, 1, k16, "copy SL32 + 2-B code gather");
    RUN(64, int, 0, k32, "copy SL64 (no gather)");
    RUN(64, int, 1, k32, "copy SL64 + 4-B key gather");
    RUN(64, short, 1, k16, "copy SL64 + 2-B code gather");
    return 0;
}
