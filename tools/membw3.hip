// Encode-shape memory-pattern sweep (not part of the product): 16 u16 rows of
// a stripe in, 64 rows out, 4 B per lane per row, varying the block width,
// the block -> (stripe, tile) order, the row order of the stores and the
// cache-policy aux bits, to find the best HBM pattern for encode_fnt_kernel.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/membw3.hip -o build/membw3
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

// BT threads per block, each lane 4 B of a row; ORD 0: stripe-major tiles,
// 1: tile-major (consecutive blocks in different stripes), 2: XCD-grouped
// (the 8 blocks dispatched round-robin to the 8 XCDs get 8 consecutive tiles
// of one stripe each... i.e. each XCD walks a contiguous run of tiles);
// RO 0: rows 0..63 in order, 1: pass order (4u + v).
template <int BT, int ORD, int RO, int AUXL, int AUXS, int PADB = 0>
__global__ __launch_bounds__(BT) void enc(const uint16_t* in, uint16_t* out, int S,
                                          int tiles)
{
    const int b = blockIdx.x;
    int s, tile;
    if constexpr (ORD == 0) {
        s = b / tiles;
        tile = b % tiles;
    } else if constexpr (ORD == 1) {
        s = b % S;
        tile = b / S;
    } else if constexpr (ORD == 3) {
        // whole stripes per XCD, interleaved: XCD x walks stripes x, x+8, ...
        const int xcd = b & 7, j = b >> 3;
        s = (j / tiles) * 8 + xcd;
        tile = j % tiles;
    } else if constexpr (ORD == 4) {
        // XCD-contiguous runs of 4 stripes: lin = xcd-run of (4 * tiles) blocks
        const int xcd = b & 7, j = b >> 3;
        const int run = 4 * tiles;
        const int lin = (j / run) * run * 8 + xcd * run + (j % run);
        s = lin / tiles;
        tile = lin % tiles;
    } else {
        const int nb = S * tiles;
        const int xcd = b & 7, j = b >> 3;
        const int lin = xcd * (nb >> 3) + j;
        s = lin / tiles;
        tile = lin % tiles;
    }
    const uint32_t voff = (tile * BT + threadIdx.x) * 4;
    auto ri = rsrc(in + (long)s * 16 * P, 16 * P * 2);
    constexpr long RS = P * 2 + PADB;
    auto ro = rsrc((char*)out + (long)s * 64 * RS, 64 * RS);
    uint32_t x[16];
#pragma unroll
    for (int t = 0; t < 16; t++)
        x[t] = __builtin_amdgcn_raw_buffer_load_b32(ri, voff, t * P * 2, AUXL);
#pragma unroll
    for (int u = 0; u < 64; u++) {
        int row;
        if constexpr (RO == 0)
            row = u;
        else if constexpr (RO == 1)
            row = 4 * (u % 16) + u / 16;
        else if constexpr (RO == 2)  // pass pairs: 0,1,4,5,...,2,3,6,7,...
            row = 4 * ((u / 2) % 16) + 2 * (u / 32) + (u & 1);
        else if constexpr (RO == 3)  // pass order rotated per wave
            row = 4 * (u % 16) + ((u / 16 + (threadIdx.x >> 6)) & 3);
        else  // pass order rotated per block
            row = 4 * (u % 16) + ((u / 16 + b) & 3);
        __builtin_amdgcn_raw_buffer_store_b32(x[u % 16] ^ (u * 0x9E3779B9u), ro, voff,
                                              row * RS, AUXS);
    }
}



// encode shape with half-wave pass split: a block covers 256 columns (each
// column read by 2 lanes); lanes 0-31 of a wave store row 4u+v, lanes 32-63
// row 4u+v+1 (v even), 4 B per lane: every store instruction writes 128 B of
// two rows whose 64 KiB address bit differs
template <int ORD, int AUXS>
__global__ __launch_bounds__(256) void enc_split(const uint16_t* in, uint16_t* out, int S,
                                                 int tiles)
{
    const int b = blockIdx.x;
    int s, tile;
    if constexpr (ORD == 0) {
        s = b / tiles;
        tile = b % tiles;
    } else {
        const int xcd = b & 7, j = b >> 3;
        s = (j / tiles) * 8 + xcd;
        tile = j % tiles;
    }
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63, h = l >> 5;
    const uint32_t voff = (tile * 128 + w * 32 + (l & 31)) * 4;
    auto ri = rsrc(in + (long)s * 16 * P, 16 * P * 2);
    auto ro = rsrc(out + (long)s * 64 * P, 64 * P * 2);
    uint32_t x[16];
#pragma unroll
    for (int t = 0; t < 16; t++)
        x[t] = __builtin_amdgcn_raw_buffer_load_b32(ri, voff, t * P * 2, 0);
    const uint32_t vo = voff + h * P * 2;
#pragma unroll
    for (int pp = 0; pp < 2; pp++)
#pragma unroll
        for (int u = 0; u < 16; u++)
            __builtin_amdgcn_raw_buffer_store_b32(x[u] ^ (u * 0x9E3779B9u), ro, vo,
                                                  (4 * u + 2 * pp) * P * 2, AUXS);
}

// decode shape: 16 of a stripe's 64 rows in (8 B per lane), 16 rows out
template <int ORD, int AUXL, int AUXS>
__global__ __launch_bounds__(256) void dec(const uint16_t* in, uint16_t* out, int S, int tiles)
{
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    const int b = blockIdx.x;
    int s, tile;
    if constexpr (ORD == 0) {
        s = b / tiles;
        tile = b % tiles;
    } else {
        const int xcd = b & 7, j = b >> 3;
        s = (j / tiles) * 8 + xcd;
        tile = j % tiles;
    }
    const uint32_t voff = (tile * 256 + threadIdx.x) * 8;
    auto ri = rsrc(in + (long)s * 64 * P, 64 * P * 2);
    auto ro = rsrc(out + (long)s * 16 * P, 16 * P * 2);
    u2 x[16];
#pragma unroll
    for (int t = 0; t < 16; t++) {
        const int row = (t * 4 + ((s * 7 + t) & 3));
        x[t] = __builtin_amdgcn_raw_buffer_load_b64(ri, voff, row * P * 2, AUXL);
    }
#pragma unroll
    for (int u = 0; u < 16; u++) {
        u2 v = x[u] ^ x[(u + 1) & 15];
        __builtin_amdgcn_raw_buffer_store_b64(v, ro, voff, u * P * 2, AUXS);
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
    CHECK(hipMalloc(&b, bb + (size_t)S * 64 * 4096));
    CHECK(hipMemset(a, 1, ab));
    CHECK(hipMemset(b, 2, bb));
    const double eb = ab + bb;
#define RUNP(BT, ORD, RO, L, SA, PB)                                                  \
    {                                                                            \
        const int tiles = P / (2 * BT);                                          \
        float ms = timeit([&] { enc<BT, ORD, RO, L, SA, PB><<<tiles * S, BT>>>(a, b, S, tiles); }, reps); \
        printf("enc BT%4d ord%d ro%d L%2d S%2d pad%4d %7.3f ms %7.1f GB/s\n", BT, ORD, RO, L, SA, PB, ms, \
               eb / ms / 1e6);                                                   \
    }
#define RUN(BT, ORD, RO, L, SA) RUNP(BT, ORD, RO, L, SA, 0)
    for (int rep = 0; rep < 3; rep++) {
    printf("--- rep %d\n", rep);
    RUN(256, 0, 1, 0, 2)
    RUN(256, 3, 1, 0, 18)
    RUN(512, 3, 1, 0, 18)
    RUN(1024, 3, 1, 0, 18)
    RUN(512, 3, 2, 0, 18)
    RUN(1024, 3, 2, 0, 18)
#define SPLIT(ORD, SA)                                                            \
    {                                                                             \
        const int tiles = P / 128;                                                \
        float ms = timeit([&] { enc_split<ORD, SA><<<tiles * S, 256>>>(a, b, S, tiles); }, reps); \
        printf("enc split ord%d S%2d        %7.3f ms %7.1f GB/s\n", ORD, SA, ms, eb / ms / 1e6); \
    }
    SPLIT(0, 2)
    SPLIT(3, 18)
    SPLIT(3, 2)
#define DEC(ORD, L, SA)                                                              \
    {                                                                                \
        const int tiles = P / 1024;                                                  \
        float ms = timeit([&] { dec<ORD, L, SA><<<tiles * S, 256>>>(b, a, S, tiles); }, reps); \
        printf("dec ord%d L%2d S%2d  %7.3f ms %7.1f GB/s\n", ORD, L, SA, ms, 2.0 * ab / ms / 1e6); \
    }
    DEC(0, 2, 2)
    DEC(3, 2, 2)
    DEC(3, 2, 18)
    DEC(3, 18, 18)
    DEC(3, 0, 18)
    DEC(3, 16, 18)
    DEC(3, 2, 26)
    }
    return 0;
}
