// Memory-pattern ceilings for the two RS-FNT kernels on MI355X (not part of
// the product): buffer-resource loads/stores with the kernels' widths and
// cache-policy variants.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/membw2.hip -o build/membw2
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

// encode shape: read 16 rows, write 64 rows, 4 B per lane; AUXL/AUXS policy
template <int AUXL, int AUXS>
__global__ __launch_bounds__(256) void enc_shape(const uint16_t* in, uint16_t* out,
                                                 int tiles)
{
    const int b = blockIdx.x;
    const int s = b / tiles, tile = b % tiles;
    const uint32_t voff = (tile * 256 + threadIdx.x) * 4;
    auto ri = rsrc(in + (long)s * 16 * P, 16 * P * 2);
    auto ro = rsrc(out + (long)s * 64 * P, 64 * P * 2);
    uint32_t x[16];
#pragma unroll
    for (int t = 0; t < 16; t++)
        x[t] = __builtin_amdgcn_raw_buffer_load_b32(ri, voff, t * P * 2, AUXL);
#pragma unroll
    for (int u = 0; u < 64; u++)
        __builtin_amdgcn_raw_buffer_store_b32(x[u % 16] ^ (u * 0x9E3779B9u), ro, voff,
                                              u * P * 2, AUXS);
}

// decode shape: read 16 of 64 rows (per-stripe pseudo-random), write 16 rows,
// 8 B per lane
template <int AUXL, int AUXS>
__global__ __launch_bounds__(256) void dec_shape(const uint16_t* in, uint16_t* out,
                                                 int tiles)
{
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    const int b = blockIdx.x;
    const int s = b / tiles, tile = b % tiles;
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

// pure streaming write / read of the coded-row footprint, 4 B per lane
template <int AUX>
__global__ __launch_bounds__(256) void wr_only(uint16_t* out, int tiles)
{
    const int b = blockIdx.x;
    const int s = b / tiles, tile = b % tiles;
    const uint32_t voff = (tile * 256 + threadIdx.x) * 4;
    auto ro = rsrc(out + (long)s * 64 * P, 64 * P * 2);
#pragma unroll
    for (int u = 0; u < 64; u++)
        __builtin_amdgcn_raw_buffer_store_b32(voff ^ u, ro, voff, u * P * 2, AUX);
}

__global__ __launch_bounds__(256) void rd_only(const uint16_t* in, uint32_t* sink,
                                               int tiles)
{
    const int b = blockIdx.x;
    const int s = b / tiles, tile = b % tiles;
    const uint32_t voff = (tile * 256 + threadIdx.x) * 4;
    auto ri = rsrc(in + (long)s * 64 * P, 64 * P * 2);
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < 64; u++)
        acc ^= __builtin_amdgcn_raw_buffer_load_b32(ri, voff, u * P * 2, 0);
    if (acc == 0x12345678u)
        sink[0] = acc;
}


// streaming write with W-byte stores per lane (W = 4, 8, 16)
template <int W, int AUX>
__global__ __launch_bounds__(256) void wr_wide(uint16_t* out, int tiles)
{
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    const int b = blockIdx.x;
    const int s = b / tiles, tile = b % tiles;
    const uint32_t voff = (tile * 256 + threadIdx.x) * W;
    auto ro = rsrc(out + (long)s * 64 * P, 64 * P * 2);
#pragma unroll
    for (int u = 0; u < 64; u++) {
        if constexpr (W == 16)
            __builtin_amdgcn_raw_buffer_store_b128(u4{voff ^ u, voff, (unsigned)u, 1u}, ro, voff, u * P * 2, AUX);
        else if constexpr (W == 8)
            __builtin_amdgcn_raw_buffer_store_b64(u2{voff ^ u, voff}, ro, voff, u * P * 2, AUX);
        else
            __builtin_amdgcn_raw_buffer_store_b32(voff ^ u, ro, voff, u * P * 2, AUX);
    }
}

// plain contiguous copy, 16 B per lane (the guide's copy-kernel ceiling)
__global__ __launch_bounds__(256) void copy16(const uint4* in, uint4* out, long n)
{
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    const long stride = (long)gridDim.x * 256;
    for (; i < n; i += stride)
        out[i] = in[i];
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
    const int et = P / 512, dt = P / 1024;
    const double eb = ab + bb, db = 2.0 * ab;
#define ENC(L, S_)                                                              \
    {                                                                           \
        float ms = timeit([&] { enc_shape<L, S_><<<et * S, 256>>>(a, b, et); }, reps); \
        printf("enc shape aux L%d S%d  %7.3f ms %7.1f GB/s\n", L, S_, ms, eb / ms / 1e6); \
    }
#define DEC(L, S_)                                                              \
    {                                                                           \
        float ms = timeit([&] { dec_shape<L, S_><<<dt * S, 256>>>(b, a, dt); }, reps); \
        printf("dec shape aux L%d S%d  %7.3f ms %7.1f GB/s\n", L, S_, ms, db / ms / 1e6); \
    }
    {
        float ms = timeit([&] { wr_only<0><<<et * S, 256>>>(b, et); }, reps);
        printf("write-only 4B        %7.3f ms %7.1f GB/s\n", ms, bb / ms / 1e6);
        ms = timeit([&] { wr_only<2><<<et * S, 256>>>(b, et); }, reps);
        printf("write-only 4B nt     %7.3f ms %7.1f GB/s\n", ms, bb / ms / 1e6);
        ms = timeit([&] { rd_only<<<et * S, 256>>>(b, reinterpret_cast<uint32_t*>(a), et); }, reps);
        printf("read-only 4B         %7.3f ms %7.1f GB/s\n", ms, bb / ms / 1e6);
    }

    {
        float ms = timeit([&] { wr_wide<8, 0><<<(P / 1024) * S, 256>>>(b, P / 1024); }, reps);
        printf("write-only 8B        %7.3f ms %7.1f GB/s\n", ms, bb / ms / 1e6);
        ms = timeit([&] { wr_wide<16, 0><<<(P / 2048) * S, 256>>>(b, P / 2048); }, reps);
        printf("write-only 16B       %7.3f ms %7.1f GB/s\n", ms, bb / ms / 1e6);
        ms = timeit([&] { wr_wide<16, 2><<<(P / 2048) * S, 256>>>(b, P / 2048); }, reps);
        printf("write-only 16B nt    %7.3f ms %7.1f GB/s\n", ms, bb / ms / 1e6);
        const long n16 = (long)ab / 16;
        ms = timeit([&] { copy16<<<256 * 8 * 4, 256>>>((const uint4*)a, (uint4*)b, n16); }, reps);
        printf("copy 16B (r+w)       %7.3f ms %7.1f GB/s\n", ms, 2.0 * ab / ms / 1e6);
    }
    ENC(0, 0) ENC(0, 1) ENC(0, 2) ENC(0, 3) ENC(2, 0) ENC(2, 2)
    DEC(0, 0) DEC(0, 1) DEC(0, 2) DEC(0, 3) DEC(2, 0) DEC(2, 2)
    return 0;
}
