// membench — achievable HBM rate of the CAR tile access pattern on gfx950.
// Copies src[P][S] -> dst[P][S] (int32, scenario-minor rows of S*4 bytes) in
// segments of SEG scenarios: work item = (pod block of 128 rows, chunk c);
// lanes = scenarios; each wave-instruction moves 64 lanes * 4 B.
// Orders: chunk-major (all pods' chunk c, then c+1: the tile kernel's order)
// or pod-major.  Variants: read only, write only, copy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

template <int SEG, int MODE>  // MODE 0 copy, 1 read, 2 write
__global__ __launch_bounds__(256) void k_tile(const int *__restrict__ src, int *__restrict__ dst, int P, int S, int nblk,
                                              int chunk_major, const int *__restrict__ perm, int *__restrict__ sink) {
    const int nchunk = S / SEG;
    const int bid = blockIdx.x;
    const int blk = chunk_major ? bid % nblk : bid / nchunk;
    const int c = chunk_major ? bid / nblk : bid % nchunk;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int RPW = 64 / SEG;  // rows per wave-instruction
    int acc = 0;
#pragma unroll 4
    for (int r0 = wave * RPW; r0 < 128; r0 += 4 * RPW) {
        const int r = r0 + lane / SEG;
        const int row = blk * 128 + r;
        const int q = perm[min(row, P - 1)];
        const size_t o = (size_t)q * S + c * SEG + (lane % SEG);
        if (MODE == 0) dst[o] = src[o];
        else if (MODE == 1) acc += src[o];
        else dst[o] = row;
    }
    if (MODE == 1 && acc == 0x7fffffff) sink[0] = acc;
}

// CH consecutive 256-B segments of a row per work item (chunk of 64 * CH
// scenarios): a wave moves one row's CH segments back to back, so the
// requests of one row reach DRAM together (512 B / 1 KB per row visit).
template <int CH, int MODE>
__global__ __launch_bounds__(256) void k_tile_wide(const int *__restrict__ src, int *__restrict__ dst, int P, int S,
                                                   int nblk, int chunk_major, const int *__restrict__ perm,
                                                   int *__restrict__ sink) {
    const int nchunk = S / (64 * CH);
    const int bid = blockIdx.x;
    const int blk = chunk_major ? bid % nblk : bid / nchunk;
    const int c = chunk_major ? bid / nblk : bid % nchunk;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int acc = 0;
#pragma unroll 2
    for (int r = wave; r < 128; r += 4) {
        const int row = blk * 128 + r;
        const int q = perm[min(row, P - 1)];
        const size_t o = (size_t)q * S + (size_t)c * 64 * CH + lane;
#pragma unroll
        for (int h = 0; h < CH; ++h) {
            if (MODE == 0) dst[o + 64 * h] = src[o + 64 * h];
            else if (MODE == 1) acc += src[o + 64 * h];
            else dst[o + 64 * h] = row;
        }
    }
    if (MODE == 1 && acc == 0x7fffffff) sink[0] = acc;
}

int main(int argc, char **argv) {
    const int P = 100000, S = 4096;
    const size_t n = (size_t)P * S;
    int *src, *dst, *perm, *sink;
    CK(hipMalloc(&src, n * 4));
    CK(hipMalloc(&dst, n * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 1, n * 4));
    CK(hipMemset(dst, 0, n * 4));
    std::vector<int> ph(P);
    for (int i = 0; i < P; ++i) ph[i] = i;
    const bool shuffle = argc > 1 && atoi(argv[1]);
    if (shuffle) { srand(1); for (int i = P - 1; i > 0; --i) std::swap(ph[i], ph[rand() % (i + 1)]); }
    CK(hipMalloc(&perm, P * 4));
    CK(hipMemcpy(perm, ph.data(), P * 4, hipMemcpyHostToDevice));
    const int nblk = (P + 127) / 128;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](auto kern, int seg, const char *name, int cm, double bytes_mult) {
        const int grid = nblk * (S / seg);
        for (int w = 0; w < 3; ++w) kern<<<grid, 256>>>(src, dst, P, S, nblk, cm, perm, sink);
        CK(hipEventRecord(a));
        const int it = 10;
        for (int w = 0; w < it; ++w) kern<<<grid, 256>>>(src, dst, P, S, nblk, cm, perm, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= it;
        printf("%-6s seg=%2d %s perm=%d: %.3f ms  %.2f TB/s\n", name, seg, cm ? "chunk-major" : "pod-major  ", (int)shuffle, ms,
               bytes_mult * n * 4 / (ms * 1e-3) / 1e12);
    };
    run(k_tile_wide<1, 0>, 64, "copyW1", 1, 2);
    run(k_tile_wide<2, 0>, 128, "copyW2", 1, 2);
    run(k_tile_wide<4, 0>, 256, "copyW4", 1, 2);
    run(k_tile_wide<1, 1>, 64, "readW1", 1, 1);
    run(k_tile_wide<2, 1>, 128, "readW2", 1, 1);
    run(k_tile_wide<1, 2>, 64, "writW1", 1, 1);
    run(k_tile_wide<2, 2>, 128, "writW2", 1, 1);
    for (int cm = 1; cm >= 0; --cm) {
        run(k_tile<16, 0>, 16, "copy", cm, 2);
        run(k_tile<32, 0>, 32, "copy", cm, 2);
        run(k_tile<64, 0>, 64, "copy", cm, 2);
        run(k_tile<32, 1>, 32, "read", cm, 1);
        run(k_tile<64, 1>, 64, "read", cm, 1);
        run(k_tile<32, 2>, 32, "write", cm, 1);
        run(k_tile<64, 2>, 64, "write", cm, 1);
    }
    return 0;
}
