// cfg3-decode memory-shape sweep (not part of the product): the pattern of
// matrix_os_kernel<4,4,1> alone -- 1024 stripes, 64 received rows in and 64
// data rows out, 4 KiB each; one block of 512 threads per stripe walks its
// columns in tiles of TW columns, rows of tile + D - 1 in flight while tile
// is stored (D = 2: the product's DEEP prefetch).  A tile moves 64 rows x 2 TW
// bytes each way; a store instruction writes 8 rows x 128 B (the product's
// whole-line shape).  Reports GB/s of reads + writes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/membw6.hip -o build/membw6
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
constexpr long P = 2048;  // u16 words per row
constexpr int KIN = 64, NOUT = 64;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes,
                                             0x00020000);
}
// TW columns per tile; loads: 4 columns (b64) per lane, TW / 4 lanes per
// row, 512 / (TW / 4) rows per pass, RPT passes; stores: TW / 64 super
// tiles x 64 rows = 8 waves x NSW super-tile rows, 2 b128 per (super tile,
// 16-row block)
template <int TW, int D, int AUX, int ROT>
__global__ __launch_bounds__(512) void dec(const uint16_t* in, uint16_t* out, int tiles,
                                           int blocks_per_stripe)
{
    constexpr int TPR = TW / 4, RPP = 512 / TPR, RPT = KIN / RPP;
    const int s = blockIdx.x / blocks_per_stripe;
    const int part = blockIdx.x % blocks_per_stripe;
    const int t0 = part * tiles / blocks_per_stripe, t1 = (part + 1) * tiles / blocks_per_stripe;
    auto ri = rsrc(in + (long)s * KIN * P, KIN * P * 2);
    auto ro = rsrc(out + (long)s * NOUT * P, NOUT * P * 2);
    const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
    const int rg = tid / TPR, cl = (tid % TPR) * 4;
    v2u w[D][RPT];
    const int nt = t1 - t0;
    const int rot = ROT ? (int)((blockIdx.x * 5u) % (unsigned)nt) : 0;
    auto phys = [&](int tile) { int i = tile - t0 + rot; return t0 + (i >= nt ? i - nt : i); };
    auto issue = [&](int tile, v2u (&r)[RPT]) {
        const uint32_t oob = tile < t1 ? 0u : 0x80000000u;
        tile = tile < t1 ? phys(tile) : tile;
#pragma unroll
        for (int i = 0; i < RPT; i++)
            r[i] = __builtin_bit_cast(
                v2u, __builtin_amdgcn_raw_buffer_load_b64(
                         ri, (int)(((RPP * i + rg) * P * 2 + (cl + tile * TW) * 2) | oob), 0, 2));
    };
    uint32_t acc = 0;
#pragma unroll
    for (int d = 0; d < D - 1; d++)
        issue(t0 + d, w[d]);
    // stores: 64 rows x TW columns = 4 row blocks x TW / 64 super tiles;
    // wave wv takes (row block, super tile) pairs wv, wv + 8, ...
    constexpr int NST = TW / 64, PAIRS = 4 * NST;
    for (int tile = t0; tile < t1; tile += D) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            const int tt = tile + d;
            if (tt >= t1)
                break;
            issue(tt + D - 1, w[(d + D - 1) % D]);
#pragma unroll
            for (int i = 0; i < RPT; i++)
                acc ^= w[d][i].x + w[d][i].y;
            for (int pp = wv; pp < PAIRS; pp += 8) {
                const int rb = pp % 4, st = pp / 4;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int row = 16 * rb + 8 * h + (l >> 3), c = l & 7;
                    v4u v = {acc, acc + 1, acc + 2, acc + (uint32_t)row};
                    const uint32_t vo = row * P * 2 + (phys(tt) * TW + 64 * st + 8 * c) * 2;
                    __builtin_amdgcn_raw_buffer_store_b128(v, ro, vo, 0, AUX);
                }
            }
            __syncthreads();
        }
    }
}
static void* g_flush = nullptr;  // non-null: a 1 GiB write before every timed launch
template <typename F>
float timeit(F f, int reps)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    float tot = 0;
    if (g_flush) {
        for (int r = 0; r < reps; r++) {
            CHECK(hipMemsetAsync(g_flush, r, 1u << 30));
            CHECK(hipEventRecord(a));
            f();
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            tot += ms;
        }
        return tot / reps;
    }
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
    const int S = argc > 1 ? atoi(argv[1]) : 1024;
    const int reps = 20;
    if (argc > 2 && atoi(argv[2]))
        CHECK(hipMalloc(&g_flush, 1u << 30));
    uint16_t *a, *b;
    const size_t ab = (size_t)S * KIN * P * 2, bb = (size_t)S * NOUT * P * 2;
    CHECK(hipMalloc(&a, ab));
    CHECK(hipMalloc(&b, bb));
    CHECK(hipMemset(a, 1, ab));
    CHECK(hipMemset(b, 2, bb));
    const double eb = ab + bb;
#define RUN(TW, D, AUX, BPS, LDS, ROT)                                                                \
    {                                                                                             \
        const int tiles = P / TW;                                                                 \
        float ms = timeit(                                                                        \
            [&] { dec<TW, D, AUX, ROT><<<S * BPS, 512, LDS * 1024>>>(a, b, tiles, BPS); }, reps);       \
        printf("cfg3dec TW%4d D%d aux%2d bps%d lds%3dK rot%d %7.1f us %7.1f GB/s\n", TW, D, AUX, BPS, \
               LDS, ROT, ms * 1e3, eb / ms / 1e6);                                                     \
    }
    for (int rep = 0; rep < 2; rep++) {
        printf("--- rep %d%s\n", rep, g_flush ? " (1 GiB write before each launch)" : "");
        RUN(128, 2, 18, 1, 57, 0)
        RUN(128, 2, 18, 1, 57, 1)
        RUN(128, 2, 18, 2, 57, 0)
        RUN(128, 2, 18, 2, 57, 1)
        RUN(128, 2, 0, 1, 57, 0)
        RUN(128, 2, 0, 1, 57, 1)
        RUN(128, 2, 0, 2, 57, 1)
        RUN(256, 2, 18, 1, 76, 1)
        RUN(256, 2, 0, 1, 76, 1)
    }
    return 0;
}
