// Memory-pattern microbenchmark for the RS-FNT encode shape on MI355X:
// per stripe read KIN rows, write KOUT rows of 64 KiB, at 4/8/16 B per lane,
// plus a 16 B/lane copy baseline.  Not part of the product; used to size the
// kernels' access width.
//   hipcc --offload-arch=gfx950 -O3 tools/membw.hip -o build/membw
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

constexpr int KIN = 16, KOUT = 64;
constexpr long P = 32768;  // words per row

template <typename V>
__global__ __launch_bounds__(256) void shape_kernel(const uint16_t* in,
                                                    uint16_t* out, int tiles)
{
    constexpr int C = sizeof(V) / 2;  // columns per lane
    const int b = blockIdx.x;
    const int s = b / tiles, tile = b % tiles;
    const long col = (static_cast<long>(tile) * 256 + threadIdx.x) * C;
    const uint16_t* src = in + s * KIN * P + col;
    uint16_t* dst = out + s * KOUT * P + col;
    V acc[KIN];
#pragma unroll
    for (int t = 0; t < KIN; t++)
        acc[t] = *reinterpret_cast<const V*>(src + t * P);
#pragma unroll
    for (int u = 0; u < KOUT; u++) {
        V v = acc[u % KIN];
        // cheap mixing so nothing is dead
        uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
        for (int j = 0; j < static_cast<int>(sizeof(V) / 4); j++)
            w[j] ^= static_cast<uint32_t>(u * 0x9E3779B9u);
        *reinterpret_cast<V*>(dst + u * P) = v;
    }
}

__global__ __launch_bounds__(256) void copy_kernel(const uint4* in, uint4* out,
                                                   long n)
{
    long i = static_cast<long>(blockIdx.x) * 256 + threadIdx.x;
    const long stride = static_cast<long>(gridDim.x) * 256;
    for (; i < n; i += stride)
        out[i] = in[i];
}

template <typename V>
float run_shape(const uint16_t* in, uint16_t* out, int S, int reps)
{
    constexpr int C = sizeof(V) / 2;
    const int tiles = static_cast<int>(P / (256 * C));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    shape_kernel<V><<<tiles * S, 256>>>(in, out, tiles);
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; r++)
        shape_kernel<V><<<tiles * S, 256>>>(in, out, tiles);
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
    uint16_t *in, *out;
    const size_t inb = static_cast<size_t>(S) * KIN * P * 2;
    const size_t outb = static_cast<size_t>(S) * KOUT * P * 2;
    CHECK(hipMalloc(&in, inb));
    CHECK(hipMalloc(&out, outb));
    CHECK(hipMemset(in, 1, inb));
    CHECK(hipMemset(out, 0, outb));
    const double bytes = static_cast<double>(inb + outb);
    struct {
        const char* name;
        float ms;
    } r[3] = {{"4B/lane", run_shape<uint32_t>(in, out, S, reps)},
              {"8B/lane", run_shape<uint2>(in, out, S, reps)},
              {"16B/lane", run_shape<uint4>(in, out, S, reps)}};
    for (auto& x : r)
        printf("shape %-9s %8.3f ms  %8.1f GB/s\n", x.name, x.ms,
               bytes / (x.ms * 1e-3) / 1e9);
    // copy baseline over the same total footprint
    const long n = static_cast<long>(outb / 16);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    copy_kernel<<<8192, 256>>>(reinterpret_cast<uint4*>(out),
                               reinterpret_cast<uint4*>(in), n / 4);
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; i++)
        copy_kernel<<<8192, 256>>>(reinterpret_cast<uint4*>(out),
                                   reinterpret_cast<uint4*>(in), n / 4);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("copy 16B/lane %8.3f ms  %8.1f GB/s (read+write)\n", ms,
           2.0 * (n / 4) * 16 / (ms * 1e-3) / 1e9);
    return 0;
}
