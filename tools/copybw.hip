// Measured copy ceiling of the box (not part of the product): a streaming
// device-to-device copy, b128 per lane, grid-stride, at a few sizes and
// store policies, plus hipMemcpyAsync.  GB/s counts read + write bytes (the
// bench's algorithmic-byte convention).  DESIGN.md section 5 reports the best
// beside the 8 TB/s spec.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/copybw.hip -o build/copybw
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
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// UNROLL independent b128 loads per lane in flight, then their stores
template <int UNROLL, int AUX>
__global__ __launch_bounds__(256) void copy_k(const v4u* __restrict__ in, v4u* __restrict__ out,
                                              size_t n)
{
    const size_t stride = static_cast<size_t>(gridDim.x) * 256 * UNROLL;
    for (size_t base = static_cast<size_t>(blockIdx.x) * 256 * UNROLL + threadIdx.x; base < n;
         base += stride) {
        v4u v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
            const size_t i = base + static_cast<size_t>(u) * 256;
            v[u] = i < n ? in[i] : v4u{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
            const size_t i = base + static_cast<size_t>(u) * 256;
            if (i < n) {
                if constexpr (AUX)
                    __builtin_nontemporal_store(v[u], out + i);
                else
                    out[i] = v[u];
            }
        }
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

int main()
{
    const size_t maxb = size_t(4) << 30;
    void *a, *b;
    CHECK(hipMalloc(&a, maxb));
    CHECK(hipMalloc(&b, maxb));
    CHECK(hipMemset(a, 1, maxb));
    CHECK(hipMemset(b, 2, maxb));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    double best = 0;
    for (size_t gib : {size_t(1), size_t(2), size_t(4)}) {
        const size_t bytes = gib << 30, n = bytes / 16;
        const double moved = 2.0 * bytes;
#define RUN(U, AUX, WPC)                                                                      \
    {                                                                                         \
        const int grid = cus * (WPC);                                                         \
        float ms = timeit([&] { copy_k<U, AUX><<<grid, 256>>>((const v4u*)a, (v4u*)b, n); }, \
                          10);                                                                \
        const double gbs = moved / ms / 1e6;                                                  \
        best = gbs > best ? gbs : best;                                                       \
        printf("copy %zu GiB unroll %d nt %d blocks/CU %2d: %7.3f ms %7.1f GB/s\n", gib, U,   \
               AUX, WPC, ms, gbs);                                                            \
    }
        RUN(4, 0, 8)
        RUN(4, 1, 8)
        RUN(8, 0, 8)
        RUN(8, 1, 8)
        RUN(4, 0, 16)
        RUN(4, 1, 16)
        {
            float ms = timeit([&] { CHECK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice)); },
                              10);
            const double gbs = moved / ms / 1e6;
            best = gbs > best ? gbs : best;
            printf("copy %zu GiB hipMemcpyAsync D2D:         %7.3f ms %7.1f GB/s\n", gib, ms, gbs);
        }
    }
    printf("best copy %.1f GB/s (read + write)\n", best);
    return 0;
}
