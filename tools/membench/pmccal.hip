// pmccal — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE / TCC counters on
// gfx950 for the CAR tile kernel's access widths (the microarch guide's x2
// correction is measured for 16-B-per-lane reads only).  Each kernel moves a
// known byte count, once per launch, in the tile kernel's pattern:
//   read4   P rows x S scenarios of int32, 4 B per lane: a wave reads one
//           256-B segment (64 scenarios) of a shuffled pod row at a time
//   write4  the same segments written (the target stores)
//   read16  the same bytes, 16 B per lane (the calibrated width)
//   gather2 2-B code gathers code[node * S + s] from an N x S u16 table
//           (5000 x 4096 = 41 MB: the tile kernel's code lines)
// usage: pmccal  (prints the algorithmic bytes of each kernel)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int kRows = 16;  // rows per wave

__global__ __launch_bounds__(256) void read4(const int *__restrict__ src, int P, int S, const int *__restrict__ perm,
                                             int *__restrict__ sink) {
    const int nch = S / 64, w = (int)(blockIdx.x * 4 + (threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int c = w % nch, r0 = (w / nch) * kRows;
    if (r0 >= P) return;
    int acc = 0;
#pragma unroll
    for (int u = 0; u < kRows; ++u) {
        const int q = perm[min(r0 + u, P - 1)];
        acc ^= __builtin_nontemporal_load(&src[(size_t)q * S + c * 64 + lane]);
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ __launch_bounds__(256) void write4(int *__restrict__ dst, int P, int S, const int *__restrict__ perm) {
    const int nch = S / 64, w = (int)(blockIdx.x * 4 + (threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int c = w % nch, r0 = (w / nch) * kRows;
    if (r0 >= P) return;
#pragma unroll
    for (int u = 0; u < kRows; ++u) {
        const int q = perm[min(r0 + u, P - 1)];
        __builtin_nontemporal_store(q ^ lane, &dst[(size_t)q * S + c * 64 + lane]);
    }
}

__global__ __launch_bounds__(256) void read16(const int4 *__restrict__ src, size_t n4, int *__restrict__ sink) {
    int acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const int4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x7fffffff) sink[0] = acc;
}

__global__ __launch_bounds__(256) void gather2(const unsigned short *__restrict__ code, int P, int S, int N,
                                               int *__restrict__ sink) {
    const int nch = S / 64, w = (int)(blockIdx.x * 4 + (threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int c = w % nch, r0 = (w / nch) * kRows;
    if (r0 >= P) return;
    unsigned acc = 0;
#pragma unroll
    for (int u = 0; u < kRows; ++u) {
        const unsigned node = ((unsigned)(r0 + u) * 2654435761u) % (unsigned)N;
        acc ^= code[(size_t)node * S + c * 64 + lane];
    }
    if (acc == 0x7fffffffu) sink[0] = (int)acc;
}

int main() {
    const int P = 100000, S = 4096, N = 5000;
    const size_t n = (size_t)P * S;
    int *src, *dst, *perm, *sink;
    unsigned short *code;
    CK(hipMalloc(&src, n * 4));
    CK(hipMalloc(&dst, n * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&code, (size_t)N * S * 2));
    CK(hipMemset(src, 1, n * 4));
    CK(hipMemset(code, 1, (size_t)N * S * 2));
    std::vector<int> ph(P);
    for (int i = 0; i < P; ++i) ph[i] = i;
    srand(1);
    for (int i = P - 1; i > 0; --i) std::swap(ph[i], ph[rand() % (i + 1)]);
    CK(hipMalloc(&perm, P * 4));
    CK(hipMemcpy(perm, ph.data(), P * 4, hipMemcpyHostToDevice));
    const int waves = ((P + kRows - 1) / kRows) * (S / 64), grid = (waves + 3) / 4;
    for (int rep = 0; rep < 3; ++rep) {
        read4<<<grid, 256>>>(src, P, S, perm, sink);
        write4<<<grid, 256>>>(dst, P, S, perm);
        read16<<<4096, 256>>>(reinterpret_cast<const int4 *>(src), n / 4, sink);
        gather2<<<grid, 256>>>(code, P, S, N, sink);
    }
    CK(hipDeviceSynchronize());
    printf("read4   %zu B read per launch (4 B/lane, 256-B segments of shuffled rows)\n", n * 4);
    printf("write4  %zu B written per launch\n", n * 4);
    printf("read16  %zu B read per launch (16 B/lane, streaming)\n", n * 4);
    printf("gather2 %zu B gathered per launch (2 B/lane from a %zu-B table)\n", n * 2, (size_t)N * S * 2);
    return 0;
}
