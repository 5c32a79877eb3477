// cfg3-encode probe ladder (not part of the product): the memory shape of
// matrix_mfma_kernel<4,8,4,true> (1024 stripes, 64 input rows and 1024 output
// rows of 4 KiB, a block of 4 waves on 512 columns of one stripe, XCD-grouped
// block map, stores of 8 rows x 128 B) with the kernel's other phases added
// one at a time, to attribute the gap between the bare store shape and the
// kernel without its epilogue math:
//   L0  row loads to registers, then every store (tools/membw5.hip RPI 8)
//   L1  + the rows staged in LDS as byte planes (perm + xor, the product's
//       column permutation) and a block barrier
//   L2  + each 16 x 64 output tile transposed through the wave's LDS staging
//       tile (2 ds_write_b128, wave barrier, 2 ds_read_b128) before its stores
//   L3  + the operand tiles of each row block loaded from a 256 KB generator
//       (L2-resident), one row block ahead in ping-pong, as the product
//   L4  + 16 ds_read_b64_tr_b8 + 16 v_mfma_i32_16x16x64_i8 per output tile
//   L5  + the epilogue's element math (the product's kernel without its
//       mark / row-scale paths and the pipelined pair loop)
// and enc_as, the A-stationary alternative (below).
// RS > 1: a block covers 1024 / RS output rows (RS blocks per column tile,
// consecutive on one XCD, re-staging the same input through L2).
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/membw7.hip -o build/membw7
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
constexpr long P = 2048;     // u16 words per row
constexpr int KIN = 64, NOUT = 1024, TW = 512;
constexpr int RSB = TW + 16;                     // image row pitch (bytes)
constexpr int IMG = 2 * KIN * RSB;               // 67,584 B
constexpr int STGP = 144, STG = 16 * STGP;       // per-wave staging tile
constexpr int LDS = IMG + 2048 + 16 + 4 * STG;   // the product's footprint
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0,
                                             (int)bytes, 0x00020000);
}
// the product's epilogue element math of one 16 x 64 tile (y = 256 D2 +
// D1 - D0 folded twice, the OOR test, packing) into o0 / o1
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

template <int LV, int RS>
__global__ __launch_bounds__(256) void enc(const uint16_t* in, uint16_t* out,
                                           const int* gen, int tiles)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    // XCD-grouped map over (stripe, tile, row part): XCD x walks all column
    // tiles and row parts of stripe 8 g + x
    const int b = blockIdx.x;
    const int j = b >> 3;
    const int per = tiles * RS;
    const int g8 = j / per;
    const int s = g8 * 8 + (b & 7);
    const int rem = j - g8 * per;
    const int tile = rem / RS, part = rem % RS;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int tl = l & 15, gq = l >> 4;
    auto ri = rsrc(in + (long)s * KIN * P, KIN * P * 2);
    auto ro = rsrc(out + (long)s * NOUT * P, NOUT * P * 2);
    // staging: thread t loads 2 columns (b32) of all 64 rows
    const uint32_t cl = threadIdx.x * 2;
    const uint32_t voff = (tile * TW + cl) * 2;
    uint32_t wv[KIN];
#pragma unroll
    for (int r = 0; r < KIN; r++)
        wv[r] = __builtin_amdgcn_raw_buffer_load_b32(ri, voff, r * P * 2, 2);
    uint32_t acc = 0;
    if constexpr (LV == 0) {
#pragma unroll
        for (int r = 0; r < KIN; r++)
            acc ^= wv[r];
    } else {
        const uint32_t lpos = 64 * (cl / 64) + 16 * ((cl % 16) / 4) +
                              4 * ((cl % 64) / 16) + cl % 4;
#pragma unroll
        for (int r = 0; r < KIN; r++) {
            const uint32_t hi = __builtin_amdgcn_perm(0u, wv[r], 0x0c0c0301u) ^ 0x8080u;
            const uint32_t lo = __builtin_amdgcn_perm(0u, wv[r], 0x0c0c0200u) ^ 0x8080u;
            *reinterpret_cast<uint16_t*>(lds + r * RSB + lpos) = (uint16_t)hi;
            *reinterpret_cast<uint16_t*>(lds + (KIN + r) * RSB + lpos) = (uint16_t)lo;
        }
        __syncthreads();
        acc = *reinterpret_cast<const uint32_t*>(lds + l * 4);
    }
    // operands (L3+): the product's load_ops per row block
    auto load_ops = [&](int rb, v2i (&bo)[4][3], int (&sc)[5]) {
        rb = rb < 63 ? rb : 63;  // the clamped prefetch past the last row block
#pragma unroll
        for (int ks = 0; ks < 4; ks++)
#pragma unroll
            for (int ty = 0; ty < 2; ty++)
                bo[ks][ty] = *reinterpret_cast<const v2i*>(gen + ((rb * 4 + ks) * 3 + ty) * 128 + l * 2);
#pragma unroll
        for (int ks = 0; ks < 4; ks++)
            bo[ks][2] = ks < 2 ? bo[ks + 2][1] : bo[ks - 2][0];
        const int t = 16 * rb + tl;
        const int* tail = gen + 64 * 4 * 3 * 128;
        sc[0] = tail[t];
        sc[1] = tail[1024 + t];
        sc[2] = tail[2048 + t];
        sc[3] = tail[2048 + 16 * rb + (l >> 3)];
        sc[4] = tail[2048 + 16 * rb + 8 + (l >> 3)];
    };
    auto* ldsa = (__attribute__((address_space(3))) uint8_t*)lds;
    const uint32_t abase = (uint32_t)((8 * gq + ((l & 15) >> 1)) * RSB + 8 * (l & 1));
    uint8_t* stg = lds + IMG + 2048 + 16 + w * STG;
    constexpr int NRB = 16 / RS;  // row blocks per wave
    auto rb_body = [&](int rb, const v2i (&bo)[4][3], const int (&sc)[5]) {
        uint32_t x = acc;
        if constexpr (LV >= 3)
            x ^= (uint32_t)(bo[0][0].x ^ bo[3][1].y ^ sc[0] ^ sc[1] ^ sc[2]);
#pragma unroll 1
        for (int st = 0; st < 8; st++) {
            v4u o0 = {x + st, x ^ st, x + rb, x}, o1 = {x ^ rb, x + 7, x, x ^ st};
            if constexpr (LV >= 4) {
                v4i a4[4][3];
#pragma unroll
                for (int T = 0; T < 4; T++) {
                    a4[T][0] = v4i{0, 0, 0, 0};
                    a4[T][1] = v4i{sc[0], sc[0], sc[0], sc[0]};
                    a4[T][2] = v4i{0, 0, 0, 0};
#pragma unroll
                    for (int ks = 0; ks < 4; ks += 2) {
                        auto rd = [&](int k2) {
                            auto* pa = (__attribute__((address_space(3))) v2i*)(
                                ldsa + abase + 32 * k2 * RSB + (4 * st + T) * 16);
                            return __builtin_amdgcn_ds_read_tr8_b64_v2i32(pa);
                        };
                        const v2i p0 = rd(ks), p1 = rd(ks + 1);
                        const v4i a{p0.x, p0.y, p1.x, p1.y};
#pragma unroll
                        for (int ty = 0; ty < 3; ty++) {
                            if ((ty == 0 && ks >= 2) || (ty == 1 && ks + 1 < 2))
                                continue;
                            const v4i bb{bo[ks][ty].x, bo[ks][ty].y, bo[ks + 1][ty].x,
                                         bo[ks + 1][ty].y};
                            a4[T][ty] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, bb, a4[T][ty], 0, 0, 0);
                        }
                    }
                }
                if constexpr (LV >= 5) {
                    epilogue(a4, o0, o1);
                } else {
#pragma unroll
                    for (int T = 0; T < 4; T++) {
                        o0[T] ^= (uint32_t)(a4[T][0][0] + a4[T][1][1] + a4[T][2][2]);
                        o1[T] ^= (uint32_t)(a4[T][0][3] + a4[T][1][2] + a4[T][2][1]);
                    }
                }
            }
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int orow = 8 * h + (l >> 3), c = l & 7;
                v4u v = h ? o1 : o0;
                if constexpr (LV >= 2) {
                    if (h == 0) {
                        *reinterpret_cast<v4u*>(stg + tl * STGP + 32 * gq) = o0;
                        *reinterpret_cast<v4u*>(stg + tl * STGP + 32 * gq + 16) = o1;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    }
                    v = *reinterpret_cast<const v4u*>(stg + orow * STGP + 16 * c);
                }
                const int row = 16 * rb + orow;
                int rowo = row;
                if constexpr (LV >= 3)
                    rowo = (sc[3 + h] & 0) + row;  // the rowmap's value, identity
                const uint32_t vo = rowo * P * 2 + tile * TW * 2 + 128 * st + 16 * c;
                __builtin_amdgcn_raw_buffer_store_b128(v, ro, vo, 0, 18);
            }
            if constexpr (LV >= 2) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
            }
        }
    };
    const int rbase = part * (64 / RS);
    v2i bA[4][3], bB[4][3];
    int sA[5], sB[5];
    if constexpr (LV >= 3)
        load_ops(rbase + w, bA, sA);
    for (int jj = 0; jj < NRB; jj += 2) {
        const int rb = rbase + w + 4 * jj;
        if constexpr (LV >= 3)
            load_ops(rb + 4, bB, sB);
        rb_body(rb, bA, sA);
        if (jj + 1 >= NRB)
            break;
        if constexpr (LV >= 3)
            load_ops(jj + 2 < NRB ? rb + 8 : rb + 4, bA, sA);
        rb_body(rb + 4, bB, sB);
    }
}
// A-stationary geometry: a block of 4 waves on 256 columns of one stripe,
// wave w owns super tile w (its A operand -- 64 columns x 128 byte-plane
// rows, 8 v4i -- read once from the staged image into registers) and walks
// all 64 row blocks, the generator's operand tiles of each row block loaded
// (L2) one row block ahead.  The image is dead after the A reads and holds
// the waves' output staging tiles; 35 KB of LDS: 4 blocks (16 waves) per CU.
// EPI: the product's epilogue math (else a stand-in xor)
constexpr int TWA = 256, RSBA = TWA + 16, IMGA = 2 * KIN * RSBA;
template <bool EPI>
__global__ __launch_bounds__(256) void enc_as(const uint16_t* in, uint16_t* out, const int* gen,
                                              int tiles)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int b = blockIdx.x;
    const int j = b >> 3;
    const int g8 = j / tiles;
    const int s = g8 * 8 + (b & 7);
    const int tile = j - g8 * tiles;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int tl = l & 15, gq = l >> 4;
    auto ri = rsrc(in + (long)s * KIN * P, KIN * P * 2);
    auto ro = rsrc(out + (long)s * NOUT * P, NOUT * P * 2);
    // staging: lane l of wave w loads 4 columns (b64) of rows w + 4 r
    const uint32_t cl = l * 4;
    const uint32_t voff = (tile * TWA + cl) * 2;
    uint32_t wv[16][2];
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(ri, voff, (4 * r + w) * P * 2, 2);
        wv[r][0] = v[0];
        wv[r][1] = v[1];
    }
    const uint32_t lpos = 64 * (cl / 64) + 16 * ((cl % 16) / 4) + 4 * ((cl % 64) / 16);
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int i = 4 * r + w;
        const uint32_t hi = __builtin_amdgcn_perm(wv[r][1], wv[r][0], 0x07050301u) ^ 0x80808080u;
        const uint32_t lo = __builtin_amdgcn_perm(wv[r][1], wv[r][0], 0x06040200u) ^ 0x80808080u;
        *reinterpret_cast<uint32_t*>(lds + i * RSBA + lpos) = hi;
        *reinterpret_cast<uint32_t*>(lds + (KIN + i) * RSBA + lpos) = lo;
    }
    __syncthreads();
    auto* ldsa = (__attribute__((address_space(3))) uint8_t*)lds;
    const uint32_t abase = (uint32_t)((8 * gq + ((l & 15) >> 1)) * RSBA + 8 * (l & 1));
    v4i av[4][2];
#pragma unroll
    for (int T = 0; T < 4; T++)
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
            auto rd = [&](int ks) {
                auto* pa = (__attribute__((address_space(3))) v2i*)(ldsa + abase + 32 * ks * RSBA +
                                                                   (4 * w + T) * 16);
                return __builtin_amdgcn_ds_read_tr8_b64_v2i32(pa);
            };
            const v2i p0 = rd(2 * kk), p1 = rd(2 * kk + 1);
            av[T][kk] = v4i{p0.x, p0.y, p1.x, p1.y};
        }
    __syncthreads();  // the image is dead: it holds the staging tiles now
    uint8_t* stg = lds + w * STG;
    const int* tail = gen + 64 * 4 * 3 * 128;
    auto ld_b = [&](int rb, v4i& b0, v4i& b1, int& kt) {
        auto ld2 = [&](int ks, int ty) {
            return *reinterpret_cast<const v2i*>(gen + ((rb * 4 + ks) * 3 + ty) * 128 + l * 2);
        };
        const v2i x0 = ld2(0, 0), x1 = ld2(1, 0), y0 = ld2(2, 1), y1 = ld2(3, 1);
        b0 = v4i{x0.x, x0.y, x1.x, x1.y};
        b1 = v4i{y0.x, y0.y, y1.x, y1.y};
        kt = tail[16 * rb + tl];
    };
    v4i bA0, bA1, bB0, bB1;
    int ktA, ktB;
    ld_b(0, bA0, bA1, ktA);
    auto rb_body = [&](int rb, const v4i& b0, const v4i& b1, int kt) {
        v4i a4[4][3];
#pragma unroll
        for (int T = 0; T < 4; T++) {
            a4[T][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[T][0], b0, v4i{0, 0, 0, 0}, 0, 0, 0);
            a4[T][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[T][1], b1, v4i{kt, kt, kt, kt}, 0, 0, 0);
            a4[T][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[T][0], b1, v4i{0, 0, 0, 0}, 0, 0, 0);
            a4[T][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[T][1], b0, a4[T][2], 0, 0, 0);
        }
        v4u o0, o1;
        if constexpr (EPI) {
            epilogue(a4, o0, o1);
        } else {
#pragma unroll
            for (int T = 0; T < 4; T++) {
                o0[T] = (uint32_t)(a4[T][0][0] + a4[T][1][1] + a4[T][2][2]);
                o1[T] = (uint32_t)(a4[T][0][3] + a4[T][1][2] + a4[T][2][1]);
            }
        }
        *reinterpret_cast<v4u*>(stg + tl * STGP + 32 * gq) = o0;
        *reinterpret_cast<v4u*>(stg + tl * STGP + 32 * gq + 16) = o1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int orow = 8 * h + (l >> 3), c = l & 7;
            const v4u v = *reinterpret_cast<const v4u*>(stg + orow * STGP + 16 * c);
            const uint32_t vo = (16 * rb + orow) * P * 2 + (tile * TWA + 64 * w) * 2 + 16 * c;
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, vo, 0, 18);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    };
#pragma unroll 1
    for (int rb = 0; rb < 64; rb += 2) {
        ld_b(rb + 1, bB0, bB1, ktB);
        rb_body(rb, bA0, bA1, ktA);
        ld_b(rb + 2 < 64 ? rb + 2 : 63, bA0, bA1, ktA);
        rb_body(rb + 1, bB0, bB1, ktB);
    }
}

// Half-line output stores (no LDS transpose): lane (g, t) holds row t,
// columns {8g .. 8g+7} (o0) and {32+8g .. 32+8g+7} (o1) of a super tile (an
// image column order that puts them there), so a store instruction of o0
// writes 16 rows x 64 contiguous bytes, and o1 the other half of each line.
// NW waves per block on 512 columns, wave w takes row blocks w + NW j; no
// staging tiles: 70 KB of LDS, so 2 blocks of 8 waves (4 waves per SIMD)
// fit a CU.  MATH: the kernel's A reads, MFMAs and epilogue (else only the
// stores).  AUX: store policy.
template <int NW, bool MATH, int AUX>
__global__ __launch_bounds__(64 * NW) void enc_h(const uint16_t* in, uint16_t* out, const int* gen,
                                                int tiles)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int b = blockIdx.x;
    const int j = b >> 3;
    const int g8 = j / tiles;
    const int s = g8 * 8 + (b & 7);
    const int tile = j - g8 * tiles;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int tl = l & 15, gq = l >> 4;
    auto ri = rsrc(in + (long)s * KIN * P, KIN * P * 2);
    auto ro = rsrc(out + (long)s * NOUT * P, NOUT * P * 2);
    // staging: 256 lanes per row pass (2 columns, b32), NW / 4 row groups
    constexpr int RG = NW / 4, RPT = KIN / RG;
    const int rg = threadIdx.x / 256;
    const uint32_t cl = (threadIdx.x % 256) * 2;
    const uint32_t voff = (tile * TW + cl) * 2;
    uint32_t wv[RPT];
#pragma unroll
    for (int r = 0; r < RPT; r++)
        wv[r] = __builtin_amdgcn_raw_buffer_load_b32(ri, voff, (RG * r + rg) * P * 2, 2);
    const uint32_t lpos = 64 * (cl / 64) + 16 * ((cl % 16) / 4) + 4 * ((cl % 64) / 16) + cl % 4;
#pragma unroll
    for (int r = 0; r < RPT; r++) {
        const int i = RG * r + rg;
        const uint32_t hi = __builtin_amdgcn_perm(0u, wv[r], 0x0c0c0301u) ^ 0x8080u;
        const uint32_t lo = __builtin_amdgcn_perm(0u, wv[r], 0x0c0c0200u) ^ 0x8080u;
        *reinterpret_cast<uint16_t*>(lds + i * RSB + lpos) = (uint16_t)hi;
        *reinterpret_cast<uint16_t*>(lds + (KIN + i) * RSB + lpos) = (uint16_t)lo;
    }
    __syncthreads();
    uint32_t acc = *reinterpret_cast<const uint32_t*>(lds + l * 4);
    auto* ldsa = (__attribute__((address_space(3))) uint8_t*)lds;
    const uint32_t abase = (uint32_t)((8 * gq + ((l & 15) >> 1)) * RSB + 8 * (l & 1));
    const int* tail = gen + 64 * 4 * 3 * 128;
    auto ld_b = [&](int rb, v4i& b0, v4i& b1, int& kt) {
        auto ld2 = [&](int ks, int ty) {
            return *reinterpret_cast<const v2i*>(gen + ((rb * 4 + ks) * 3 + ty) * 128 + l * 2);
        };
        const v2i x0 = ld2(0, 0), x1 = ld2(1, 0), y0 = ld2(2, 1), y1 = ld2(3, 1);
        b0 = v4i{x0.x, x0.y, x1.x, x1.y};
        b1 = v4i{y0.x, y0.y, y1.x, y1.y};
        kt = tail[16 * rb + tl];
    };
    auto rb_body = [&](int rb, const v4i& b0, const v4i& b1, int kt) {
#pragma unroll 1
        for (int st = 0; st < 8; st++) {
            v4u o0 = {acc + st, acc ^ st, acc + rb, acc}, o1 = {acc ^ rb, acc + 7, acc, acc ^ st};
            if constexpr (MATH) {
                v4i a4[4][3];
#pragma unroll
                for (int T = 0; T < 4; T++) {
                    auto rd = [&](int ks) {
                        auto* pa = (__attribute__((address_space(3))) v2i*)(
                            ldsa + abase + 32 * ks * RSB + (4 * st + T) * 16);
                        return __builtin_amdgcn_ds_read_tr8_b64_v2i32(pa);
                    };
                    const v2i p0 = rd(0), p1 = rd(1), p2 = rd(2), p3 = rd(3);
                    const v4i h{p0.x, p0.y, p1.x, p1.y}, lo{p2.x, p2.y, p3.x, p3.y};
                    a4[T][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(h, b0, v4i{0, 0, 0, 0}, 0, 0, 0);
                    a4[T][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(lo, b1, v4i{kt, kt, kt, kt}, 0, 0, 0);
                    a4[T][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(h, b1, v4i{0, 0, 0, 0}, 0, 0, 0);
                    a4[T][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(lo, b0, a4[T][2], 0, 0, 0);
                }
                epilogue(a4, o0, o1);
            }
            const uint32_t rowb = (16 * rb + tl) * P * 2 + tile * TW * 2 + 128 * st + 16 * gq;
            __builtin_amdgcn_raw_buffer_store_b128(o0, ro, rowb, 0, AUX);
            __builtin_amdgcn_raw_buffer_store_b128(o1, ro, rowb + 64, 0, AUX);
        }
    };
    v4i bA0, bA1, bB0, bB1;
    int ktA, ktB;
    ld_b(w, bA0, bA1, ktA);
    constexpr int NRB = 64 / NW;
#pragma unroll 1
    for (int jj = 0; jj < NRB; jj += 2) {
        const int rb = w + NW * jj;
        ld_b(rb + NW, bB0, bB1, ktB);
        rb_body(rb, bA0, bA1, ktA);
        ld_b(jj + 2 < NRB ? rb + 2 * NW : rb + NW, bA0, bA1, ktA);
        rb_body(rb + NW, bB0, bB1, ktB);
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
    if (g_flush) {
        float tot = 0;
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
    const int reps = 10;
    uint16_t *a, *b;
    int* gen;
    const size_t ab = (size_t)S * KIN * P * 2, bb = (size_t)S * NOUT * P * 2;
    const size_t gb = (64 * 4 * 3 * 128 + 4096) * 4;
    CHECK(hipMalloc(&a, ab));
    CHECK(hipMalloc(&b, bb));
    CHECK(hipMalloc(&gen, gb));
    CHECK(hipMemset(b, 2, bb));
    // random data and operand tiles (argv[2] = "zero": the trivial fills;
    // MFMAs on random operands draw more power and clock lower)
    const bool zero = argc > 2 && argv[2][0] == 'z';
    {
        std::vector<uint32_t> h(ab / 4);
        uint64_t x = 0x9E3779B97F4A7C15ull;
        for (auto& v : h) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            v = zero ? 0x01010101u : static_cast<uint32_t>(x);
        }
        CHECK(hipMemcpy(a, h.data(), ab, hipMemcpyHostToDevice));
        std::vector<uint32_t> hg(gb / 4);
        for (size_t i = 0; i < hg.size(); i++) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            // operand bytes in [-128, 127]; the tail (kt, rowmap) small
            hg[i] = zero ? 0u : i < 64 * 4 * 3 * 128 ? static_cast<uint32_t>(x) : static_cast<uint32_t>(x & 1023);
        }
        CHECK(hipMemcpy(gen, hg.data(), gb, hipMemcpyHostToDevice));
    }
    printf("data: %s\n", zero ? "trivial fills" : "random");
    // argv[3] = "flush": caches flushed (a 1 GiB write) before every launch,
    // as the encode meets them in the bench step (after the decode)
    if (argc > 3 && argv[3][0] == 'f') {
        CHECK(hipMalloc(&g_flush, 1u << 30));
        printf("1 GiB write before each timed launch\n");
    }
    const double eb = ab + bb;
    const int tiles = P / TW;
#define RUN(LV, RS)                                                                        \
    {                                                                                      \
        CHECK(hipFuncSetAttribute((const void*)enc<LV, RS>,                               \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDS));       \
        float ms = timeit([&] { enc<LV, RS><<<tiles * S * RS, 256, LDS>>>(a, b, gen, tiles); }, \
                          reps);                                                           \
        CHECK(hipGetLastError());                                                          \
        printf("cfg3 ladder L%d RS%d %7.3f ms %7.1f GB/s\n", LV, RS, ms, eb / ms / 1e6);  \
    }
#define RUNAS(EPI)                                                                         \
    {                                                                                      \
        float ms = timeit([&] { enc_as<EPI><<<(P / TWA) * S, 256, IMGA>>>(a, b, gen, P / TWA); }, \
                          reps);                                                           \
        CHECK(hipGetLastError());                                                          \
        printf("cfg3 A-stationary epi%d  %7.3f ms %7.1f GB/s\n", EPI, ms, eb / ms / 1e6);  \
    }
    constexpr int LDSH = IMG + 2048 + 16;
#define RUNH(NW, MATH, AUX)                                                                \
    {                                                                                      \
        CHECK(hipFuncSetAttribute((const void*)enc_h<NW, MATH, AUX>,                      \
                                  hipFuncAttributeMaxDynamicSharedMemorySize, LDSH));      \
        float ms = timeit([&] { enc_h<NW, MATH, AUX><<<tiles * S, 64 * NW, LDSH>>>(a, b, gen, tiles); }, \
                          reps);                                                           \
        CHECK(hipGetLastError());                                                          \
        printf("cfg3 half-line NW%d math%d aux%2d %7.3f ms %7.1f GB/s\n", NW, MATH, AUX, ms, \
               eb / ms / 1e6);                                                             \
    }
    for (int rep = 0; rep < 2; rep++) {
        printf("--- rep %d\n", rep);
        RUNH(4, false, 0)
        RUNH(4, false, 18)
        RUNH(8, false, 0)
        RUNH(8, false, 18)
        RUNH(8, true, 0)
        RUNH(8, true, 18)
        RUNH(4, true, 0)
        RUN(0, 1)
        RUN(1, 1)
        RUN(2, 1)
        RUN(3, 1)
        RUN(4, 1)
        RUN(5, 1)
        RUN(0, 4)
        RUN(4, 4)
        RUN(5, 4)
        RUNAS(false)
        RUNAS(true)
    }
    return 0;
}
