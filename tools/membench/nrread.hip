// nrread — the read rate node_reduce's scan pass can get from its access
// pattern on gfx950: 1M rows x 64 int32 scenarios (256 MB), read once.
//   A  nr_scan's shape: blocks of PB pods, waves of 256 pods walking 16 rows a
//      unit (one dword per lane per row, lane = scenario), two units in flight
//   B  the same walk with 16-B loads (a wave covers 4 rows per instruction)
//   C  a flat grid-stride read, 16-B loads, 4 in flight per thread (ceiling)
// Each variant folds what it read into one word per thread (kept live).
// Round 6 (r06l): one 256-MB array read back to back ran 6.5-6.9 TB/s, the
// MALL serving part of it; the NBUF rotation below reads cold copies.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int S = 64, kB = 16;
typedef int v4i __attribute__((ext_vector_type(4)));

template <int PB, int T>
__global__ __launch_bounds__(T) void walk1(const int *__restrict__ a, int P, int *__restrict__ sink) {
    const int per = ((P + PB - 1) / PB + 7) >> 3, b = (int)(blockIdx.x & 7u) * per + (int)(blockIdx.x >> 3);
    if (b * PB >= P) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int kPW = PB / (T / 64);
    const int q0 = b * PB + wv * kPW, q1 = min(P, q0 + kPW), nv = (q1 - q0 + kB - 1) / kB;
    int acc = 0, ra[kB], rb[kB];
    auto load = [&](int v, int (&r)[kB]) {
        v = min(v, nv - 1);
        const int pb = q0 + v * kB;
#pragma unroll
        for (int u = 0; u < kB; ++u) r[u] = __builtin_nontemporal_load(a + (size_t)min(pb + u, q1 - 1) * S + lane);
    };
    load(0, ra);
    for (int v = 0; v < nv; v += 2) {
        load(v + 1, rb);
        asm volatile("" : "+v"(ra[0])::"memory");
#pragma unroll
        for (int u = 0; u < kB; ++u) acc ^= ra[u] * (u + 1);
        load(v + 2, ra);
        asm volatile("" : "+v"(rb[0])::"memory");
#pragma unroll
        for (int u = 0; u < kB; ++u) acc ^= rb[u] * (u + 3);
    }
    sink[blockIdx.x * T + threadIdx.x] = acc;
}

template <int PB, int T>
__global__ __launch_bounds__(T) void walk4(const int *__restrict__ a, int P, int *__restrict__ sink) {
    const int per = ((P + PB - 1) / PB + 7) >> 3, b = (int)(blockIdx.x & 7u) * per + (int)(blockIdx.x >> 3);
    if (b * PB >= P) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int kPW = PB / (T / 64), kI = kB / 4;  // 4 rows per instruction
    const int q0 = b * PB + wv * kPW, q1 = min(P, q0 + kPW), nv = (q1 - q0 + kB - 1) / kB;
    const v4i *__restrict__ a4 = reinterpret_cast<const v4i *>(a);
    int acc = 0;
    v4i ra[kI], rb[kI];
    auto load = [&](int v, v4i (&r)[kI]) {
        v = min(v, nv - 1);
        const int pb = q0 + v * kB;
#pragma unroll
        for (int u = 0; u < kI; ++u)
            r[u] = __builtin_nontemporal_load(a4 + (size_t)min(pb + 4 * u + (lane >> 4), q1 - 1) * (S / 4) + (lane & 15));
    };
    load(0, ra);
    for (int v = 0; v < nv; v += 2) {
        load(v + 1, rb);
        asm volatile("" : "+v"(ra[0].x)::"memory");
#pragma unroll
        for (int u = 0; u < kI; ++u) acc ^= (ra[u].x + ra[u].y * 3 + ra[u].z * 5 + ra[u].w * 7) * (u + 1);
        load(v + 2, ra);
        asm volatile("" : "+v"(rb[0].x)::"memory");
#pragma unroll
        for (int u = 0; u < kI; ++u) acc ^= (rb[u].x + rb[u].y * 3 + rb[u].z * 5 + rb[u].w * 7) * (u + 2);
    }
    sink[blockIdx.x * T + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void flat4(const v4i *__restrict__ a, size_t n4, int *__restrict__ sink) {
    const size_t stride = (size_t)gridDim.x * 256 * 4;
    int acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 * 4 + threadIdx.x; i < n4; i += stride) {
        v4i r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) r[u] = __builtin_nontemporal_load(a + min(i + (size_t)u * 256, n4 - 1));
#pragma unroll
        for (int u = 0; u < 4; ++u) acc ^= r[u].x + r[u].y * 3 + r[u].z * 5 + r[u].w * 7;
    }
    sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

// Each timed launch reads one of NBUF copies in turn (4 x 256 MB: none is
// still in the 256-MB MALL when it is read again), events around each launch.
constexpr int NBUF = 4;
template <class F>
static void timeit(const char *name, F launch, double bytes) {
    hipEvent_t ev[2];
    CK(hipEventCreate(&ev[0]));
    CK(hipEventCreate(&ev[1]));
    for (int i = 0; i < NBUF; ++i) launch(i);
    const int reps = 32;
    double tot = 0;
    for (int i = 0; i < reps; ++i) {
        CK(hipEventRecord(ev[0]));
        launch(i % NBUF);
        CK(hipEventRecord(ev[1]));
        CK(hipEventSynchronize(ev[1]));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, ev[0], ev[1]));
        tot += ms;
    }
    const double us = tot * 1e3 / reps;
    printf("%-34s %8.2f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
}

int main() {
    const int P = 1 << 20;
    const size_t n = (size_t)P * S;
    int *buf[NBUF], *sink;
    for (int i = 0; i < NBUF; ++i) CK(hipMalloc(&buf[i], n * 4));
    CK(hipMalloc(&sink, (size_t)64 << 20));
    std::vector<int> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (int)(i * 2654435761u);
    for (int i = 0; i < NBUF; ++i) CK(hipMemcpy(buf[i], h.data(), n * 4, hipMemcpyHostToDevice));
    const double bytes = (double)n * 4;
    auto g = [&](int pb) { return (unsigned)(((P + pb - 1) / pb + 7) / 8 * 8); };
    timeit("A walk1 2048 pods / 512 thr", [&](int i) { walk1<2048, 512><<<g(2048), 512>>>(buf[i], P, sink); }, bytes);
    timeit("A walk1 4096 pods / 1024 thr", [&](int i) { walk1<4096, 1024><<<g(4096), 1024>>>(buf[i], P, sink); }, bytes);
    timeit("A walk1 1024 pods / 256 thr", [&](int i) { walk1<1024, 256><<<g(1024), 256>>>(buf[i], P, sink); }, bytes);
    timeit("B walk4 2048 pods / 512 thr", [&](int i) { walk4<2048, 512><<<g(2048), 512>>>(buf[i], P, sink); }, bytes);
    timeit("B walk4 4096 pods / 1024 thr", [&](int i) { walk4<4096, 1024><<<g(4096), 1024>>>(buf[i], P, sink); }, bytes);
    timeit("B walk4 1024 pods / 256 thr", [&](int i) { walk4<1024, 256><<<g(1024), 256>>>(buf[i], P, sink); }, bytes);
    timeit("B walk4 512 pods / 128 thr", [&](int i) { walk4<512, 128><<<g(512), 128>>>(buf[i], P, sink); }, bytes);
    for (int grid : {1024, 2048, 4096, 8192})
        timeit(grid == 1024 ? "C flat4 grid 1024" : grid == 2048 ? "C flat4 grid 2048" : grid == 4096 ? "C flat4 grid 4096" : "C flat4 grid 8192",
               [&](int i) { flat4<<<grid, 256>>>(reinterpret_cast<const v4i *>(buf[i]), n / 4, sink); }, bytes);
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
