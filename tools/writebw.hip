// Write ceiling of the box (not part of the product): how
// fast can HBM absorb the encodes' output bytes alone?  Write-only fills of
// the cfg3 coded batch (1024 stripes x 1024 rows x 4 KiB = 4.29 GB) and the
// cfg2 coded batch (4096 stripes x 64 rows x 64 KiB = 17.18 GB), b128 per
// lane, whole 128-byte lines per 8 lanes, in three orders:
//   lin    grid-stride over the whole buffer (the easiest order for HBM)
//   stripe one block per (stripe, 64 KiB piece), blocks dealt over the XCDs as
//          the product's block_map (XCD x walks stripe 8g + x)
//   rows   as stripe, but each block writes 16 rows x 4 KiB (a 1024-column
//          tile of 16 output rows, the cfg3 generator kernel's store shape)
// under the store policies default / nt / sc1 / nt|sc1 (buffer stores, aux
// 0 / 2 / 16 / 18), plus the encodes' full memory shape without math (read
// the k data rows once, write the coded rows) for reference.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/writebw.hip -o build/writebw
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
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void* base, unsigned bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
}

template <int AUX>
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, unsigned off, v4i v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, AUX);
}

// lin: grid-stride, 8 b128 stores per lane per iteration, over `chunks` of
// 1 GiB (buffer resources address 32 bits)
template <int AUX>
__global__ __launch_bounds__(256) void fill_lin(char* base, size_t bytes)
{
    const v4i v = {int(threadIdx.x), int(blockIdx.x), 7, 9};
    const size_t step = static_cast<size_t>(gridDim.x) * 256 * 16 * 8;
    for (size_t o = (static_cast<size_t>(blockIdx.x) * 256 * 8 + threadIdx.x) * 16; o < bytes;
         o += step) {
        const size_t g = o >> 30;  // 1 GiB window
        __amdgpu_buffer_rsrc_t r = rsrc(base + (g << 30), 1u << 30);
        const unsigned lo = static_cast<unsigned>(o - (g << 30));
#pragma unroll
        for (int u = 0; u < 8; u++)
            st16<AUX>(r, lo + u * 256 * 16, v);
    }
}

// stripe: block b -> (stripe, piece of PIECE bytes); XCD-aware map as the
// product (block b runs on XCD b % 8; XCD x walks the pieces of stripe 8g + x)
template <int AUX, int PIECE>
__global__ __launch_bounds__(256) void fill_stripe(char* base, size_t stripe_bytes, int S)
{
    const int per = static_cast<int>(stripe_bytes / PIECE);
    const int b = blockIdx.x, x = b & 7, j = b >> 3;
    const int grp = j / per, pc = j - grp * per;
    const int s = grp * 8 + x;
    if (s >= S)
        return;
    char* sb = base + static_cast<size_t>(s) * stripe_bytes + static_cast<size_t>(pc) * PIECE;
    __amdgpu_buffer_rsrc_t r = rsrc(sb, PIECE);
    const v4i v = {int(threadIdx.x), s, pc, 9};
#pragma unroll 8
    for (unsigned o = threadIdx.x * 16; o < PIECE; o += 256 * 16)
        st16<AUX>(r, o, v);
}

// rows: block b -> (stripe, tile of 16 rows x ROWB bytes at row pitch
// `pitch`); the 16 rows of a tile are consecutive rows of the coded stripe
template <int AUX, int ROWB>
__global__ __launch_bounds__(256) void fill_rows(char* base, size_t stripe_bytes, int S,
                                                 unsigned pitch, int rows)
{
    const int tiles = rows / 16;
    const int b = blockIdx.x, x = b & 7, j = b >> 3;
    const int grp = j / tiles, tl = j - grp * tiles;
    const int s = grp * 8 + x;
    if (s >= S)
        return;
    char* sb = base + static_cast<size_t>(s) * stripe_bytes;
    __amdgpu_buffer_rsrc_t r = rsrc(sb, static_cast<unsigned>(stripe_bytes));
    const v4i v = {int(threadIdx.x), s, tl, 9};
    constexpr int kLanesPerRow = ROWB / 16;
    for (int e = threadIdx.x; e < 16 * kLanesPerRow; e += 256) {
        const int row = tl * 16 + e / kLanesPerRow, c = e % kLanesPerRow;
        st16<AUX>(r, row * pitch + c * 16, v);
    }
}

// the cfg3 generator encode's store ORDER without its loads or math
// (1024 stripes x 1024 rows x 4 KiB): block = (stripe, column tile of CT
// columns), 4 waves, wave w walks row blocks w, w + 4, ... (16 rows each);
//   MODE 0: per 64-column super tile two store instructions of 8 rows x
//           128 B (the product's LDS-transposed epilogue, gen_mfma_kernel)
//   MODE 1: per row of the row block, CT * 2 bytes as 1 KiB instructions
//           (each instruction one contiguous run of one row)
template <int AUX, int CT, int MODE, int NW = 4>
__global__ __launch_bounds__(64 * NW) void fill_tiles(char* base, int S)
{
    constexpr int NT = 2048 / CT;  // column tiles per stripe
    const int b = blockIdx.x, x = b & 7, j = b >> 3;
    const int grp = j / NT, ct = j - grp * NT;
    const int s = grp * 8 + x;
    if (s >= S)
        return;
    __amdgpu_buffer_rsrc_t r = rsrc(base + static_cast<size_t>(s) * (1024u * 4096u),
                                    1024u * 4096u);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const v4i v = {l, s, ct, 9};
    const unsigned c0 = ct * CT * 2;
    for (int rb = w; rb < 64; rb += NW) {
        if constexpr (MODE == 0) {
#pragma unroll
            for (int st = 0; st < CT / 64; st++)
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int row = 16 * rb + 8 * h + (l >> 3);
                    st16<AUX>(r, row * 4096u + c0 + st * 128 + 16 * (l & 7), v);
                }
        } else {
#pragma unroll
            for (int rr = 0; rr < 16; rr++)
#pragma unroll
                for (int q = 0; q < CT * 2 / 1024; q++)
                    st16<AUX>(r, (16 * rb + rr) * 4096u + c0 + q * 1024 + 16 * l, v);
        }
    }
}

// the encode's memory shape without math: read K rows of a stripe's data
// (RB bytes each), write N rows (RB bytes each); one block per (stripe,
// 4 KiB column piece), the block's loads first, then its stores
template <int AUX, int K, int N>
__global__ __launch_bounds__(256) void enc_shape(const char* in, char* out, size_t in_sb,
                                                 size_t out_sb, unsigned rowb, int S)
{
    const int per = rowb / 4096;
    const int b = blockIdx.x, x = b & 7, j = b >> 3;
    const int grp = j / per, pc = j - grp * per;
    const int s = grp * 8 + x;
    if (s >= S)
        return;
    __amdgpu_buffer_rsrc_t ri = rsrc(const_cast<char*>(in) + s * in_sb, static_cast<unsigned>(in_sb));
    __amdgpu_buffer_rsrc_t ro = rsrc(out + s * out_sb, static_cast<unsigned>(out_sb));
    const unsigned c0 = pc * 4096 + threadIdx.x * 16;
    v4i acc = {0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < K; t++)
        acc += __builtin_amdgcn_raw_buffer_load_b128(ri, t * rowb + c0, 0, 0);
#pragma unroll 8
    for (int t = 0; t < N; t++)
        st16<AUX>(ro, t * rowb + c0, acc + v4i{t, 0, 0, 0});
}

template <typename F>
float timeit(F f, int reps)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int w = 0; w < 20; w++)  // the clock ramps over the first tens of ms
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
    const size_t cfg3_sb = 1024ull * 4096, cfg2_sb = 64ull * 65536;
    const int S3 = 1024, S2 = 4096;
    const size_t b3 = cfg3_sb * S3, b2 = cfg2_sb * S2;  // 4.29 GB, 17.18 GB
    char *out, *in;
    CHECK(hipMalloc(&out, b2));
    CHECK(hipMalloc(&in, 16ull * 65536 * S2));
    CHECK(hipMemset(out, 1, b2));
    CHECK(hipMemset(in, 2, 16ull * 65536 * S2));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto rep = [](const char* what, size_t bytes, float ms) {
        printf("%-44s %8.3f ms %7.1f GB/s\n", what, ms, bytes / ms / 1e6);
    };
#define LIN(AUX, NAME, B)                                                                      \
    rep("fill lin " NAME " " #B, B, timeit([&] { fill_lin<AUX><<<cus * 8, 256>>>(out, B); }, 10));
#define STRIPE(AUX, NAME, SB, S)                                                               \
    rep("fill stripe 64KiB pieces " NAME " " #SB, SB * S, timeit([&] {                         \
            fill_stripe<AUX, 65536><<<S * (SB / 65536), 256>>>(out, SB, S);                     \
        }, 10));
    if (getenv("WRITEBW_ORDER")) {
        // the cfg3 generator's store order (fill_tiles), 2 passes
        for (int pass = 0; pass < 2; pass++) {
            printf("-- order pass %d\n", pass);
#define TIL(AUX, CT, MODE, NAME)                                                            \
    rep("tiles CT " #CT " " NAME " aux " #AUX, b3, timeit([&] {                               \
            fill_tiles<AUX, CT, MODE><<<S3 * (2048 / CT), 256>>>(out, S3);                    \
        }, 10));
            TIL(0, 512, 0, "8 rows x 128 B") TIL(18, 512, 0, "8 rows x 128 B")
            TIL(0, 512, 1, "row runs 1 KiB") TIL(18, 512, 1, "row runs 1 KiB")
            TIL(0, 1024, 0, "8 rows x 128 B") TIL(18, 1024, 0, "8 rows x 128 B")
            TIL(0, 1024, 1, "row runs 1 KiB") TIL(18, 1024, 1, "row runs 1 KiB")
            TIL(0, 2048, 0, "8 rows x 128 B") TIL(18, 2048, 0, "8 rows x 128 B")
            TIL(0, 2048, 1, "row runs 1 KiB") TIL(18, 2048, 1, "row runs 1 KiB")
            // occupancy: the product's LDS footprint (77 KB: 2 blocks of 4
            // waves per CU) or half of it, and 8-wave blocks
            for (int lds : {77 * 1024, 38 * 1024, 19 * 1024}) {
                CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fill_tiles<18, 512, 0, 4>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, lds));
                CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&fill_tiles<18, 512, 0, 8>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, lds));
                char nm[96];
                snprintf(nm, sizeof nm, "tiles CT 512 aux 18, 4 waves, LDS %d KB", lds >> 10);
                rep(nm, b3, timeit([&] { fill_tiles<18, 512, 0, 4><<<S3 * 4, 256, lds>>>(out, S3); }, 10));
                snprintf(nm, sizeof nm, "tiles CT 512 aux 18, 8 waves, LDS %d KB", lds >> 10);
                rep(nm, b3, timeit([&] { fill_tiles<18, 512, 0, 8><<<S3 * 4, 512, lds>>>(out, S3); }, 10));
            }
        }
        return 0;
    }
    for (int pass = 0; pass < 2; pass++) {
        printf("-- pass %d\n", pass);
        LIN(0, "default", b3) LIN(2, "nt", b3) LIN(16, "sc1", b3) LIN(18, "nt|sc1", b3)
        STRIPE(0, "default", cfg3_sb, S3) STRIPE(18, "nt|sc1", cfg3_sb, S3)
        rep("fill rows 16x4KiB tiles default cfg3", b3, timeit([&] {
                fill_rows<0, 4096><<<S3 * 64, 256>>>(out, cfg3_sb, S3, 4096, 1024);
            }, 10));
        rep("fill rows 16x4KiB tiles nt|sc1 cfg3", b3, timeit([&] {
                fill_rows<18, 4096><<<S3 * 64, 256>>>(out, cfg3_sb, S3, 4096, 1024);
            }, 10));
        rep("enc shape cfg3 (read 64 rows, write 1024) nt|sc1", b3 + 64ull * 4096 * S3,
            timeit([&] {
                enc_shape<18, 64, 1024><<<S3 * 1, 256>>>(in, out, 64ull * 4096, cfg3_sb, 4096, S3);
            }, 10));
        LIN(0, "default", b2) LIN(2, "nt", b2) LIN(18, "nt|sc1", b2)
        STRIPE(0, "default", cfg2_sb, S2) STRIPE(18, "nt|sc1", cfg2_sb, S2)
        rep("enc shape cfg2 (read 16 rows, write 64) nt|sc1", b2 + 16ull * 65536 * S2,
            timeit([&] {
                enc_shape<18, 16, 64><<<S2 * 16, 256>>>(in, out, 16ull * 65536, cfg2_sb, 65536, S2);
            }, 10));
    }
    return 0;
}
