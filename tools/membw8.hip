// cfg3-encode probe (not part of the product; round 6): does the encode lose
// its time waiting for each block's input rows?  tools/writebw.hip measures
// the generator encode's store order alone at 0.71 ms and tools/membw7.hip's
// L0 (the same stores after each block's 64 row loads) at 0.90 ms.  Here the
// blocks are persistent (2 per CU) and walk their units (stripe, 512-column
// tile) in order; the next unit's row loads are issued while this unit's
// stores run:
//   P0  loads + stores only (membw7 L0, persistent, prefetch one unit ahead)
//   P3  + the per-row-block operand loads (L2), OPS row blocks ahead; the
//       next unit's rows are issued behind the first OPS row blocks' operand
//       loads (vector loads return in order: a wait for a later load waits
//       for the prefetch too)
//   P5  + the LDS image, the MFMAs and the epilogue math (membw7 L5)
// and the non-persistent L0 / L5 for reference.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/membw8.hip -o build/membw8
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../quadiron_amd/csrc/gf65537.h"
#define CHECK(x)                                                             \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);          \
            exit(1);                                                         \
        }                                                                    \
    } while (0)
constexpr long P = 2048;
constexpr int KIN = 64, NOUT = 1024, TW = 512;
constexpr int RSB = TW + 16;
constexpr int IMG = 2 * KIN * RSB;
constexpr int STGP = 144, STG = 16 * STGP;
constexpr int LDS = IMG + 2048 + 16 + 4 * STG;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes,
                                             0x00020000);
}
__device__ __forceinline__ void epilogue(const v4i (&a4)[4][3], v4u& o0, v4u& o1)
{
    int32_t y[16];
#pragma unroll
    for (int T = 0; T < 4; T++)
#pragma unroll
        for (int j = 0; j < 4; j++)
            y[4 * T + j] = qi::fold(qi::fold((a4[T][2][j] << 8) + a4[T][1][j] - a4[T][0][j]));
    uint32_t bad = 0;
#pragma unroll
    for (int c = 0; c < 16; c++)
        bad |= static_cast<uint32_t>(y[c]);
    if (__builtin_expect(__builtin_amdgcn_ballot_w64((bad >> 16) != 0) != 0, 0)) {
#pragma unroll
        for (int c = 0; c < 16; c++)
            if (static_cast<uint32_t>(y[c]) > 65535u)
                y[c] = 0;
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
        o0[c] = __builtin_amdgcn_perm(static_cast<uint32_t>(y[2 * c + 1]),
                                      static_cast<uint32_t>(y[2 * c]), 0x05040100u);
        o1[c] = __builtin_amdgcn_perm(static_cast<uint32_t>(y[8 + 2 * c + 1]),
                                      static_cast<uint32_t>(y[8 + 2 * c]), 0x05040100u);
    }
}

struct Ops {
    v4i b0, b1;
    int kt;
};

// LV 0: loads + stores; 3: + operand loads; 5: + image, MFMAs, epilogue.
// PERS: persistent blocks (grid = units / U) walking units b, b + grid, ...
template <int LV, bool PERS, int OPS>
__global__ __launch_bounds__(256) void enc(const uint16_t* in, uint16_t* out, const int* gen,
                                           int tiles, int units)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int tl = l & 15, gq = l >> 4;
    const uint32_t cl = threadIdx.x * 2;
    auto unit_of = [&](int u, int& s, int& tile) {
        const int j = u >> 3, g8 = j / tiles;
        s = g8 * 8 + (u & 7);
        tile = j - g8 * tiles;
    };
    uint32_t wv[KIN];
    auto issue = [&](int u) {
        int s, tile;
        unit_of(u < units ? u : units - 1, s, tile);
        auto ri = rsrc(in + (long)s * KIN * P, KIN * P * 2);
        const uint32_t voff = (tile * TW + cl) * 2 + (u < units ? 0u : 0x80000000u);
#pragma unroll
        for (int r = 0; r < KIN; r++)
            wv[r] = __builtin_amdgcn_raw_buffer_load_b32(ri, voff, r * P * 2, 2);
    };
    const uint32_t lpos = 64 * (cl / 64) + 16 * ((cl % 16) / 4) + 4 * ((cl % 64) / 16) + cl % 4;
    auto stage = [&]() -> uint32_t {
        if constexpr (LV < 5) {
            uint32_t acc = 0;
#pragma unroll
            for (int r = 0; r < KIN; r++)
                acc ^= wv[r];
            return acc;
        } else {
#pragma unroll
            for (int r = 0; r < KIN; r++) {
                const uint32_t hi = __builtin_amdgcn_perm(0u, wv[r], 0x0c0c0301u) ^ 0x8080u;
                const uint32_t lo = __builtin_amdgcn_perm(0u, wv[r], 0x0c0c0200u) ^ 0x8080u;
                *reinterpret_cast<uint16_t*>(lds + r * RSB + lpos) = (uint16_t)hi;
                *reinterpret_cast<uint16_t*>(lds + (KIN + r) * RSB + lpos) = (uint16_t)lo;
            }
            return 0u;
        }
    };
    auto load_ops = [&](int rb, Ops& o) {
        rb = rb < 63 ? rb : 63;
        auto ld2 = [&](int ks, int ty) {
            return *reinterpret_cast<const v2i*>(gen + ((rb * 4 + ks) * 3 + ty) * 128 + l * 2);
        };
        const v2i x0 = ld2(0, 0), x1 = ld2(1, 0), y0 = ld2(2, 1), y1 = ld2(3, 1);
        o.b0 = v4i{x0.x, x0.y, x1.x, x1.y};
        o.b1 = v4i{y0.x, y0.y, y1.x, y1.y};
        o.kt = gen[64 * 4 * 3 * 128 + 16 * rb + tl];
    };
    auto* ldsa = (__attribute__((address_space(3))) uint8_t*)lds;
    const uint32_t abase = (uint32_t)((8 * gq + ((l & 15) >> 1)) * RSB + 8 * (l & 1));
    uint8_t* stg = lds + IMG + 2048 + 16 + w * STG;
    const int step = PERS ? gridDim.x : units;
    int u = blockIdx.x;
    if (u >= units)
        return;
    issue(u);
    for (; u < units; u += step) {
        int s, tile;
        unit_of(u, s, tile);
        auto ro = rsrc(out + (long)s * NOUT * P, NOUT * P * 2);
        if constexpr (LV >= 5)
            __syncthreads();  // every wave is done with the previous unit's image
        const uint32_t acc = stage();
        if constexpr (LV >= 5)
            __syncthreads();
        Ops ops[OPS];
        if constexpr (LV >= 3) {
#pragma unroll
            for (int i = 0; i < OPS; i++)
                load_ops(w + 4 * i, ops[i]);
        }
        if (PERS && u + step < units)  // behind the first operand loads
            issue(u + step);
#pragma unroll 1
        for (int jj = 0; jj < 16; jj += OPS) {
#pragma unroll
            for (int i = 0; i < OPS; i++) {
                const int rb = w + 4 * (jj + i);
                const Ops o = ops[i];
                if constexpr (LV >= 3)
                    load_ops(rb + 4 * OPS, ops[i]);
                uint32_t x = acc;
                if constexpr (LV >= 3 && LV < 5)
                    x ^= (uint32_t)(o.b0.x ^ o.b1.y ^ o.kt);
#pragma unroll 1
                for (int st = 0; st < 8; st++) {
                    v4u o0 = {x + st, x ^ st, x + rb, x}, o1 = {x ^ rb, x + 7, x, x ^ st};
                    if constexpr (LV >= 5) {
                        v4i a4[4][3];
                        const v4i ktv{o.kt, o.kt, o.kt, o.kt};
#pragma unroll
                        for (int T = 0; T < 4; T++) {
                            auto rd = [&](int k2) {
                                auto* pa = (__attribute__((address_space(3))) v2i*)(
                                    ldsa + abase + 32 * k2 * RSB + (4 * st + T) * 16);
                                return __builtin_amdgcn_ds_read_tr8_b64_v2i32(pa);
                            };
                            const v2i h0 = rd(0), h1 = rd(1), l0 = rd(2), l1 = rd(3);
                            const v4i ah{h0.x, h0.y, h1.x, h1.y}, al{l0.x, l0.y, l1.x, l1.y};
                            a4[T][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, o.b0, v4i{0, 0, 0, 0}, 0, 0, 0);
                            a4[T][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, o.b1, ktv, 0, 0, 0);
                            a4[T][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, o.b1, v4i{0, 0, 0, 0}, 0, 0, 0);
                            a4[T][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, o.b0, a4[T][2], 0, 0, 0);
                        }
                        epilogue(a4, o0, o1);
                        *reinterpret_cast<v4u*>(stg + tl * STGP + 32 * gq) = o0;
                        *reinterpret_cast<v4u*>(stg + tl * STGP + 32 * gq + 16) = o1;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const int orow = 8 * h + (l >> 3), c = l & 7;
                        v4u v = h ? o1 : o0;
                        if constexpr (LV >= 5)
                            v = *reinterpret_cast<const v4u*>(stg + orow * STGP + 16 * c);
                        const uint32_t vo = (16 * rb + orow) * P * 2 + tile * TW * 2 + 128 * st + 16 * c;
                        __builtin_amdgcn_raw_buffer_store_b128(v, ro, vo, 0, 18);
                    }
                    if constexpr (LV >= 5) {
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                    }
                }
            }
        }
        if (!PERS)
            break;
    }
}

template <typename F>
float timeit(F f, int reps)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 20; i++)
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
    uint16_t *a, *b;
    int* gen;
    const size_t ab = (size_t)S * KIN * P * 2, bb = (size_t)S * NOUT * P * 2;
    const size_t gb = (64 * 4 * 3 * 128 + 4096) * 4;
    CHECK(hipMalloc(&a, ab));
    CHECK(hipMalloc(&b, bb));
    CHECK(hipMalloc(&gen, gb));
    {
        std::vector<uint32_t> h(ab / 4);
        uint64_t x = 0x9E3779B97F4A7C15ull;
        for (auto& v : h) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            v = static_cast<uint32_t>(x);
        }
        CHECK(hipMemcpy(a, h.data(), ab, hipMemcpyHostToDevice));
        std::vector<uint32_t> hg(gb / 4);
        for (size_t i = 0; i < hg.size(); i++) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            hg[i] = i < 64 * 4 * 3 * 128 ? static_cast<uint32_t>(x) : static_cast<uint32_t>(x & 1023);
        }
        CHECK(hipMemcpy(gen, hg.data(), gb, hipMemcpyHostToDevice));
    }
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const double eb = ab + bb;
    const int tiles = P / TW, units = tiles * S;
#define RUN(LV, PERS, OPS, GRID)                                                              \
    {                                                                                         \
        CHECK(hipFuncSetAttribute((const void*)enc<LV, PERS, OPS>,                           \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS));          \
        const int grid = GRID;                                                                \
        float ms = timeit([&] { enc<LV, PERS, OPS><<<grid, 256, LDS>>>(a, b, gen, tiles, units); }, \
                          10);                                                                \
        CHECK(hipGetLastError());                                                             \
        printf("cfg3 L%d %s ops%d grid %5d %7.3f ms %7.1f GB/s\n", LV, PERS ? "persistent" : "per-unit  ", \
               OPS, grid, ms, eb / ms / 1e6);                                                 \
    }
    for (int rep = 0; rep < 2; rep++) {
        printf("--- rep %d\n", rep);
        RUN(0, false, 2, units)
        RUN(0, true, 2, 2 * cus)
        RUN(3, false, 2, units)
        RUN(3, true, 2, 2 * cus)
        RUN(3, true, 4, 2 * cus)
        RUN(5, false, 2, units)
        RUN(5, true, 2, 2 * cus)
        RUN(5, true, 4, 2 * cus)
    }
    return 0;
}
