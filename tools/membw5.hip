// cfg3-encode store-pattern sweep (not part of the product): the memory
// shape of matrix_mfma_kernel<4,8,4,true> alone -- 1024 stripes, 64 input
// rows and 1024 output rows of 4 KiB, a block of 4 waves on 512 columns of
// one stripe (XCD-grouped block map), each wave walking its 16 row blocks of
// 16 rows.  A store instruction writes RPI rows x (1024 / RPI) bytes:
// RPI = 8 is the product's shape (8 rows x 128 B per 64-column super tile);
// smaller RPI needs 8 / RPI super tiles held before the store.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/membw5.hip -o build/membw5
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
constexpr long P = 2048;     // u16 words per row
constexpr int KIN = 64, NOUT = 1024, TW = 512;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                             (int)bytes, 0x00020000);
}
// RPI rows per store instruction; RBO 0: wave w takes row blocks w + 4 j,
// 1: row blocks 16 w + j; AUX store policy
template <int RPI, int RBO, int AUX, int ROT = 0>
__global__ __launch_bounds__(256) void enc(const uint16_t* in, uint16_t* out, int tiles)
{
    const int b = blockIdx.x;
    const int j = b >> 3;
    const int g = j / tiles;
    const int s = g * 8 + (b & 7);
    const int tile = j - g * tiles;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    auto ri = rsrc(in + (long)s * KIN * P, KIN * P * 2);
    auto ro = rsrc(out + (long)s * NOUT * P, NOUT * P * 2);
    // input: 128 lanes per row (4 columns, b64), 2 row groups, 32 rows each
    const uint32_t voff = (tile * TW + (threadIdx.x & 127) * 4) * 2;
    const int rg = threadIdx.x >> 7;
    uint32_t acc = 0;
#pragma unroll
    for (int r = 0; r < KIN / 2; r++) {
        auto v = __builtin_amdgcn_raw_buffer_load_b64(ri, voff, (2 * r + rg) * P * 2, 2);
        acc ^= v[0] + v[1];
    }
    // store lane map: RPI rows x (64 / RPI) lanes of 16 B
    constexpr int LPR = 64 / RPI;  // lanes per row
    const int lr = l / LPR, lc = l % LPR;
    constexpr int NI = 8 / RPI;  // instructions per 16-row x 64 / ... group
#pragma unroll 1
    for (int j0 = 0; j0 < 16; j0++) {
        // ROT: the row-block walk starts at a per-stripe offset
        const int jj = ROT ? (j0 + ROT * s) & 15 : j0;
        const int rb = RBO == 0 ? w + 4 * jj : 16 * w + jj;
        // 16 rows x 1 KB = 16 instructions of 1 KB
#pragma unroll
        for (int it = 0; it < 16; it++) {
            // it -> (row group of RPI rows, column piece)
            const int pieces = 8 / RPI * 1;  // column pieces of 128 RPI... per row
            (void)pieces;
            int row, cbyte;
            if constexpr (RPI == 8) {
                // super tile st = it / 2, half h = it % 2
                row = 8 * (it & 1) + lr;
                cbyte = 128 * (it >> 1) + 16 * lc;
            } else {
                // RPI rows x (1024 / RPI) bytes; 16 / RPI row groups
                constexpr int NG = 16 / RPI;
                const int rgp = it % NG, cp = it / NG;  // row group, column piece
                row = RPI * rgp + lr;
                cbyte = (1024 / RPI) * cp * 0 + 16 * lc + cp * (1024 / RPI) * 0;
                // pieces per row = RPI (1024 B / (1024 / RPI)); cp < RPI
                cbyte = cp * (1024 / RPI) + 16 * lc;
            }
            v4u v = {acc + it, acc ^ it, acc + rb, acc};
            const uint32_t vo = (16 * rb + row) * P * 2 + tile * TW * 2 + cbyte;
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, vo, 0, AUX);
        }
    }
    (void)NI;
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
    const int S = argc > 1 ? atoi(argv[1]) : 1024;
    const int reps = 10;
    uint16_t *a, *b;
    const size_t ab = (size_t)S * KIN * P * 2, bb = (size_t)S * NOUT * P * 2;
    CHECK(hipMalloc(&a, ab));
    CHECK(hipMalloc(&b, bb));
    CHECK(hipMemset(a, 1, ab));
    CHECK(hipMemset(b, 2, bb));
    const double eb = ab + bb;
    const int tiles = P / TW;
#define RUN(RPI, RBO, AUX, ROT)                                                                   \
    {                                                                                        \
        float ms = timeit([&] { enc<RPI, RBO, AUX, ROT><<<tiles * S, 256, 80 * 1024>>>(a, b, tiles); }, \
                          reps);                                                             \
        printf("cfg3enc RPI%d rbo%d aux%2d rot%d %7.3f ms %7.1f GB/s\n", RPI, RBO, AUX, ROT, ms,         \
               eb / ms / 1e6);                                                               \
    }
    for (int rep = 0; rep < 2; rep++) {
        printf("--- rep %d\n", rep);
        RUN(8, 0, 18, 0)
        RUN(8, 0, 18, 1)
        RUN(8, 0, 18, 5)
        RUN(8, 0, 18, 7)
        RUN(8, 0, 0, 0)
        RUN(8, 0, 0, 5)
        RUN(4, 0, 18, 5)
    }
    return 0;
}
