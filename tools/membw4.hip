// Encode-shape store-pattern sweep (not part of the product): 16 u16 rows
// of a stripe in, 64 rows out (cfg2), 4 B (2 columns) per lane per row.
// A wave is split into NQ lane groups on the same columns; group h stores
// the rows of pass v = h (NQ = 4) or v in {h, h + 2} (NQ = 2), so one store
// instruction writes NQ rows x (256 / NQ) bytes.  NQ = 1 is the product's
// pass order (rows 4u + v, 16 per pass).  Also RO 0 (rows in order).
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/membw4.hip -o build/membw4
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHECK(x)                                                             \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);          \
            exit(1);                                                         \
        }                                                                    \
    } while (0)
constexpr long P = 32768;  // u16 words per row
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                             (int)bytes, 0x00020000);
}
// NQ lane groups per wave; RO 1: a group's passes in order (rows 4u + v),
// RO 0: (NQ = 1 only) rows 0..63 in order
template <int NQ, int RO, int AUXS>
__global__ __launch_bounds__(256) void enc(const uint16_t* in, uint16_t* out, int S, int tiles)
{
    const int b = blockIdx.x;
    const int xcd = b & 7, j = b >> 3;
    const int s = (j / tiles) * 8 + xcd;
    const int tile = j % tiles;
    constexpr int LPG = 64 / NQ;  // lanes per group
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, h = l / LPG;
    // a block covers 4 waves x LPG lanes x 2 columns
    const uint32_t voff = (tile * 4 * LPG + w * LPG + (l % LPG)) * 4;
    auto ri = rsrc(in + (long)s * 16 * P, 16 * P * 2);
    auto ro = rsrc(out + (long)s * 64 * P, 64 * P * 2);
    uint32_t x[16];
#pragma unroll
    for (int t = 0; t < 16; t++)
        x[t] = __builtin_amdgcn_raw_buffer_load_b32(ri, voff, t * P * 2, 0);
    constexpr int NP = 4 / NQ;  // passes per lane
#pragma unroll
    for (int pp = 0; pp < NP; pp++)
#pragma unroll
        for (int u = 0; u < 16; u++) {
            int row;
            if constexpr (RO == 0)
                row = 16 * pp + u;
            else
                row = 4 * u + h + NQ * pp;
            __builtin_amdgcn_raw_buffer_store_b32(x[u] ^ ((u + 16 * pp) * 0x9E3779B9u), ro, voff,
                                                  row * P * 2, AUXS);
        }
}
template <typename F>
float timeit(F f, int reps)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; r++)
        f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}
int main(int argc, char** argv)
{
    const int S = argc > 1 ? atoi(argv[1]) : 4096;
    const int reps = 10;
    uint16_t *a, *b;
    const size_t ab = (size_t)S * 16 * P * 2, bb = (size_t)S * 64 * P * 2;
    CHECK(hipMalloc(&a, ab));
    CHECK(hipMalloc(&b, bb));
    CHECK(hipMemset(a, 1, ab));
    CHECK(hipMemset(b, 2, bb));
    const double eb = ab + bb;
#define RUN(NQ, RO, SA)                                                                    \
    {                                                                                      \
        const int tiles = P / (2 * 4 * (64 / NQ));                                         \
        float ms = timeit([&] { enc<NQ, RO, SA><<<tiles * S, 256>>>(a, b, S, tiles); }, reps); \
        printf("enc NQ%d ro%d S%2d %7.3f ms %7.1f GB/s\n", NQ, RO, SA, ms, eb / ms / 1e6);  \
    }
    for (int rep = 0; rep < 3; rep++) {
        printf("--- rep %d\n", rep);
        RUN(1, 1, 18)
        RUN(1, 0, 18)
        RUN(2, 1, 18)
        RUN(4, 1, 18)
        RUN(2, 1, 0)
        RUN(4, 1, 0)
        RUN(2, 1, 2)
        RUN(4, 1, 2)
    }
    return 0;
}
