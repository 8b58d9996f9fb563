// phasebench — does separating reads and writes in time raise the copy rate
// of the CAR tile kernel's access pattern on gfx950?
// Copies src[P][S] -> dst[P][S] (int32, scenario-minor rows of S*4 bytes) in
// work items of 128 shuffled rows x one 64-scenario chunk (256-B segments, a
// wave holds 32 rows in registers), like the tile kernel's image loads and
// target stores.
//   free    one workgroup per item: read its rows, then write them (reads and
//           writes of different workgroups interleave freely: the tile kernel)
//   phased  a persistent grid (W workgroups per CU) whose workgroups issue
//           their reads only in even slots of the device's constant 100 MHz
//           clock (s_memrealtime) and their writes only in odd ones, L ticks
//           per slot: the memory system sees bursts of reads and of writes
// usage: phasebench   (prints ms and TB/s of read + write bytes per variant)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int kRowsPerWave = 32;  // 4 waves x 32 = 128 rows per item

__device__ __forceinline__ void item_read(const int *__restrict__ src, int S, int P, const int *__restrict__ perm,
                                          int item, int nblk, int (&v)[kRowsPerWave]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int blk = item % nblk, c = item / nblk;
#pragma unroll
    for (int u = 0; u < kRowsPerWave; ++u) {
        const int q = perm[min(blk * 128 + wave * kRowsPerWave + u, P - 1)];
        v[u] = __builtin_nontemporal_load(&src[(size_t)q * S + c * 64 + lane]);
    }
}

__device__ __forceinline__ void item_write(int *__restrict__ dst, int S, int P, const int *__restrict__ perm, int item,
                                           int nblk, const int (&v)[kRowsPerWave]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int blk = item % nblk, c = item / nblk;
#pragma unroll
    for (int u = 0; u < kRowsPerWave; ++u) {
        const int q = perm[min(blk * 128 + wave * kRowsPerWave + u, P - 1)];
        __builtin_nontemporal_store(v[u] + 1, &dst[(size_t)q * S + c * 64 + lane]);
    }
}

__global__ __launch_bounds__(256) void k_free(const int *__restrict__ src, int *__restrict__ dst, int P, int S,
                                              int nblk, const int *__restrict__ perm) {
    int v[kRowsPerWave];
    item_read(src, S, P, perm, blockIdx.x, nblk, v);
    item_write(dst, S, P, perm, blockIdx.x, nblk, v);
}

__device__ __forceinline__ void wait_slot(unsigned long long L, unsigned parity) {
    for (;;) {
        const unsigned long long t = wall_clock64();
        if (((t / L) & 1ull) == parity) return;
        __builtin_amdgcn_s_sleep(2);
    }
}

// persistent: workgroup g takes items g, g + G, ...
__global__ __launch_bounds__(256) void k_phased(const int *__restrict__ src, int *__restrict__ dst, int P, int S,
                                                int nblk, const int *__restrict__ perm, int nitems,
                                                unsigned long long L) {
    int v[kRowsPerWave];
    for (int item = blockIdx.x; item < nitems; item += gridDim.x) {
        wait_slot(L, 0);
        item_read(src, S, P, perm, item, nblk, v);
        // (the loads complete before the write slot is awaited: the values are used below)
#pragma unroll
        for (int u = 0; u < kRowsPerWave; ++u) asm volatile("" : "+v"(v[u]));
        __builtin_amdgcn_s_waitcnt(0);
        wait_slot(L, 1);
        item_write(dst, S, P, perm, item, nblk, v);
    }
}

// persistent without phases (the same loop, for the baseline of the form)
__global__ __launch_bounds__(256) void k_persist(const int *__restrict__ src, int *__restrict__ dst, int P, int S,
                                                 int nblk, const int *__restrict__ perm, int nitems) {
    int v[kRowsPerWave];
    for (int item = blockIdx.x; item < nitems; item += gridDim.x) {
        item_read(src, S, P, perm, item, nblk, v);
        item_write(dst, S, P, perm, item, nblk, v);
    }
}

int main() {
    const int P = 100000, S = 4096;
    const size_t n = (size_t)P * S;
    int *src, *dst, *perm;
    CK(hipMalloc(&src, n * 4));
    CK(hipMalloc(&dst, n * 4));
    CK(hipMemset(src, 1, n * 4));
    CK(hipMemset(dst, 0, n * 4));
    std::vector<int> ph(P);
    for (int i = 0; i < P; ++i) ph[i] = i;
    srand(1);
    for (int i = P - 1; i > 0; --i) std::swap(ph[i], ph[rand() % (i + 1)]);
    CK(hipMalloc(&perm, P * 4));
    CK(hipMemcpy(perm, ph.data(), P * 4, hipMemcpyHostToDevice));
    const int nblk = (P + 127) / 128, nitems = nblk * (S / 64);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char *name, auto launch) {
        for (int w = 0; w < 2; ++w) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        const int it = 5;
        for (int w = 0; w < it; ++w) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= it;
        printf("%-28s %.3f ms  %.2f TB/s\n", name, ms, 2.0 * n * 4 / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    timeit("free", [&] { k_free<<<nitems, 256>>>(src, dst, P, S, nblk, perm); });
    for (int W : {4, 8}) {
        char nm[64];
        snprintf(nm, sizeof nm, "persist W=%d", W);
        timeit(nm, [&] { k_persist<<<256 * W, 256>>>(src, dst, P, S, nblk, perm, nitems); });
        for (unsigned long long L : {100ull, 200ull, 400ull, 800ull, 1600ull}) {
            snprintf(nm, sizeof nm, "phased W=%d L=%.0fus", W, L / 100.0);
            timeit(nm, [&] { k_phased<<<256 * W, 256>>>(src, dst, P, S, nblk, perm, nitems, L); });
        }
    }
    return 0;
}
