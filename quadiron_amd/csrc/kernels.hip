// HIP kernels for RS-FNT over GF(65537) on CDNA4 (gfx950).
//
// Layout: every fragment row is a contiguous run of u16 symbols ("words");
// a stripe is the set of rows sharing a column index range.  One lane owns
// COLS adjacent columns of one stripe, so every global access of a wave is a
// contiguous 64*COLS*2-byte segment of one row (coalesced), and every column
// -- an independent RS codeword read "vertically" across the fragments
// (src/fec_base.h:1103-1150) -- is transformed entirely in VGPRs.
//
// Addressing: a stripe's rows are reached through a buffer resource (SGPR
// base + 32-bit extent) with the row offset in an SGPR (soffset) and the
// column offset in one VGPR (voffset), so no per-lane 64-bit address math is
// spent per load/store.  Stripes whose extent does not fit 32 bits use the
// BUF=false instantiation (flat global addressing).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <utility>

#include "fnt_codelets.h"
#include "gf65537.h"
#include "matrix_pack.h"
#include "qi_internal.h"


namespace qi {

constexpr int kBlock = 256;

__device__ __forceinline__ void record_oor(const Oor& o, int s, int slot,
                                           long long col)
{
    const uint32_t e =
        atomicAdd(&o.counts[static_cast<long long>(s) * o.slots + slot], 1u);
    if (e < static_cast<uint32_t>(o.cap))
        o.entries[(static_cast<long long>(s) * o.slots + slot) * o.cap + e] =
            static_cast<uint32_t>(col);
}

// T-range value -> stored u16: 65536 and its alias -1 are stored as 0 (the
// truncation of vec::unpack src/vec_cast.h:133-163).
__device__ __forceinline__ uint32_t fix16(int32_t y)
{
    return static_cast<uint32_t>(y) > 65535u ? 0u : static_cast<uint32_t>(y);
}

// canonical residue of a V-range value [-2, 65537]
__device__ __forceinline__ uint32_t canon_v(int32_t y)
{
    const int32_t c = y < 0 ? y + 65537 : y;
    return static_cast<uint32_t>(c >= 65537 ? c - 65537 : c);
}

constexpr long long kTwLo = -32767, kTwHi = 98303;
static_assert(fold_rng(join(mul_rng(Rng{0, 65535}, 32768),
                            mul_rng(Rng{0, 65535}, -32768))).lo == kTwLo &&
                  fold_rng(join(mul_rng(Rng{0, 65535}, 32768),
                                mul_rng(Rng{0, 65535}, -32768))).hi == kTwHi,
              "twist output range");

// x * c for a T-range x and a balanced row scale |c| <= 32766 as ONE
// v_mul_i32_i24 (written out: the compiler cannot see that the lazily
// reduced x fits 24 bits and emitted the quarter-rate v_mul_lo_u32)
__device__ __forceinline__ int32_t mul_rs(int32_t x, int32_t c)
{
    int32_t r;
    asm("v_mul_i32_i24 %0, %1, %2" : "=v"(r) : "v"(x), "v"(c));
    return r;
}

// pack the low halves of two dwords: [a.lo, b.lo] (one v_perm_b32)
__device__ __forceinline__ uint32_t pack_lo(uint32_t a, uint32_t b)
{
    return __builtin_amdgcn_perm(b, a, 0x05040100u);
}

// A stripe region: buffer resource (BUF) or flat base pointer.
template <bool BUF>
struct Region {
    __amdgpu_buffer_rsrc_t r;
    char* p;
    __device__ __forceinline__ Region(const void* base, uint32_t bytes)
    {
        p = static_cast<char*>(const_cast<void*>(base));
        if constexpr (BUF)
            r = __builtin_amdgcn_make_buffer_rsrc(p, static_cast<short>(0),
                                                  static_cast<int>(bytes),
                                                  0x00020000);
    }
};

// Cache policy of the streamed rows (buffer-op aux bits on gfx950: 1 = sc0,
// 2 = nt, 16 = sc1).  Measured with tools/membw2.hip / membw3.hip on the
// kernels' own shapes (profiles/r1_membw.txt): nt|sc1 stores (device scope,
// written through the XCD's L2) +5 % on both the encode shape (16 rows in,
// 64 out) and the decode shape (16 of 64 rows in, 16 out); nt loads +5 % on
// the decode shape, but slow the encode shape down (its inputs stay plain).
// The matrix-core kernel's whole-line output stores keep nt|sc1 as well:
// default, nt and sc1 alone measured 1-7 % slower
// (profiles/r1_ab_mfma_store_policy.txt).
constexpr int kAuxLd = 2;
constexpr int kAuxSt = 18;
constexpr int kAuxStMf = 18;
// matrix_os_kernel's row loads: default policy (its G row-block groups read
// the same tiles through their XCD's L2; nt measured the same at k200 /
// k256 / cfg3, gpurun_out ab_aux)
constexpr int kAuxLdOs = 0;

// XCD-aware block -> (stripe, tile) map.  Workgroups are dispatched
// round-robin over the 8 XCDs (block b runs on XCD b % 8), so with the plain
// stripe-major order the 8 adjacent tiles of one stripe land on 8 different
// XCDs.  Instead, each group of 8 consecutive stripes is split so that XCD x
// walks all tiles of stripe 8g + x: +4-6 % HBM throughput on both kernel
// shapes (membw3 "ord3").  A trailing partial group (S % 8 stripes) keeps
// the stripe-major order.
__device__ __forceinline__ void block_map(int b, int tiles, int& s, int& tile)
{
    const int n_stripes = static_cast<int>(gridDim.x) / tiles;
    const int grouped = (n_stripes & ~7) * tiles;  // blocks in full groups
    if (b < grouped) {
        const int j = b >> 3;
        const int g = j / tiles;
        s = g * 8 + (b & 7);
        tile = j - g * tiles;
        return;
    }
    s = b / tiles;
    tile = b - s * tiles;
}

// NDW (1 or 2) dwords per lane of the row at byte offset `row`
template <int NDW, bool BUF, int AUX = 0>
__device__ __forceinline__ void ld_dw(const Region<BUF>& g, uint32_t row,
                                      uint32_t voff, uint32_t (&w)[NDW])
{
    static_assert(NDW == 1 || NDW == 2, "dword count");
    if constexpr (NDW == 1) {
        if constexpr (BUF)
            w[0] = __builtin_amdgcn_raw_buffer_load_b32(
                g.r, static_cast<int>(voff), static_cast<int>(row), AUX);
        else
            w[0] = *reinterpret_cast<const uint32_t*>(g.p + row + voff);
    } else {
        if constexpr (BUF) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(
                g.r, static_cast<int>(voff), static_cast<int>(row), AUX);
            w[0] = v[0];
            w[1] = v[1];
        } else {
            const uint2 v = *reinterpret_cast<const uint2*>(g.p + row + voff);
            w[0] = v.x;
            w[1] = v.y;
        }
    }
}

template <int NDW, bool BUF, int AUX = 0>
__device__ __forceinline__ void st_dw(const Region<BUF>& g, uint32_t row,
                                      uint32_t voff, const uint32_t (&w)[NDW])
{
    static_assert(NDW == 1 || NDW == 2, "dword count");
    if constexpr (NDW == 1) {
        if constexpr (BUF)
            __builtin_amdgcn_raw_buffer_store_b32(w[0], g.r, static_cast<int>(voff),
                                                  static_cast<int>(row), AUX);
        else
            *reinterpret_cast<uint32_t*>(g.p + row + voff) = w[0];
    } else {
        if constexpr (BUF) {
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
            u32x2 v;
            v[0] = w[0];
            v[1] = w[1];
            __builtin_amdgcn_raw_buffer_store_b64(v, g.r, static_cast<int>(voff),
                                                  static_cast<int>(row), AUX);
        } else {
            *reinterpret_cast<uint2*>(g.p + row + voff) = make_uint2(w[0], w[1]);
        }
    }
}

// COLS adjacent u16 columns of the row at byte offset `row` (wave-uniform).
// FULL: COLS/2 dwords per lane (COLS 2 or 4); otherwise one u16 per column
// and columns past `avail` are 0.
template <int COLS, bool FULL, bool BUF, int AUX = 0>
__device__ __forceinline__ void ld(const Region<BUF>& g, uint32_t row,
                                   uint32_t voff, long long avail, int32_t* v)
{
    if constexpr (FULL && COLS % 2 == 0) {
        uint32_t w[COLS / 2];
        ld_dw<COLS / 2, BUF, AUX>(g, row, voff, w);
#pragma unroll
        for (int d = 0; d < COLS / 2; d++) {
            v[2 * d] = w[d] & 0xffff;
            v[2 * d + 1] = w[d] >> 16;
        }
    } else {
#pragma unroll
        for (int c = 0; c < COLS; c++) {
            if (FULL || c < avail) {
                if constexpr (BUF)
                    v[c] = __builtin_amdgcn_raw_buffer_load_b16(
                        g.r, static_cast<int>(voff + 2 * c),
                        static_cast<int>(row), AUX);
                else
                    v[c] = *reinterpret_cast<const uint16_t*>(g.p + row + voff +
                                                              2 * c);
            } else {
                v[c] = 0;
            }
        }
    }
}

template <int COLS, bool FULL, bool BUF, int AUX = 0>
__device__ __forceinline__ void st(const Region<BUF>& g, uint32_t row,
                                   uint32_t voff, long long avail,
                                   const uint32_t* v)
{
    if constexpr (FULL && COLS % 2 == 0) {
        uint32_t w[COLS / 2];
#pragma unroll
        for (int d = 0; d < COLS / 2; d++)
            w[d] = pack_lo(v[2 * d], v[2 * d + 1]);
        st_dw<COLS / 2, BUF, AUX>(g, row, voff, w);
    } else {
#pragma unroll
        for (int c = 0; c < COLS; c++) {
            if (FULL || c < avail) {
                if constexpr (BUF)
                    __builtin_amdgcn_raw_buffer_store_b16(
                        static_cast<uint16_t>(v[c]), g.r,
                        static_cast<int>(voff + 2 * c), static_cast<int>(row), AUX);
                else
                    *reinterpret_cast<uint16_t*>(g.p + row + voff + 2 * c) =
                        static_cast<uint16_t>(v[c]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Non-systematic encode (src/fec_rs_fnt.h:236-251 NON_SYSTEMATIC branch ==
// Radix2::fft of the zero-padded column, src/fft_2n.h:360-407).
//
// The n-point transform of a column with K = ceil2(k) live inputs is split
// into n/K twisted K-point transforms:
//     out[(n/K) u + v] = sum_{t<K} (d_t w^{vt}) wK^{ut}
// so a lane keeps only 2K values per column live, and pass v writes the K
// output rows {(n/K)u + v}.  All loads of a lane are issued back to back
// (branch-free), outputs are stored as soon as a pass is done, and the rare
// out-of-range outputs (value 65536, src/fec_rs_fnt.h:253-269) are found by
// one OR-reduction per pass and fixed up off the fast path.
// KEQ: k == K (no zero-padded inputs to mask).
// ---------------------------------------------------------------------------
// cfg2 encode passes in store-interleaved pairs (3.675 -> 3.627 ms)
static constexpr bool kEncPair = true;

template <int K, int COLS, bool FULL, bool KEQ, bool BUF>
__device__ __forceinline__ void encode_body(
    int k, int n, int n_out, const int32_t* __restrict__ twist,
    const Region<BUF>& gi, uint32_t irs, const Region<BUF>& go, uint32_t ors,
    uint32_t voff, long long col, long long avail, int s, const Oor& oor)
{
    // RELOAD (K = 32): re-read the K input rows every pass (L2 hits after
    // the first) instead of keeping them live next to the pass's outputs:
    // 141 -> 105 VGPRs, 3 -> 4 waves/SIMD.  K = 64 stays resident (its DFT64
    // codelet alone needs ~180 VGPRs, so reloading gains no occupancy).
    // Holding two passes to interleave their stores (the 64 KiB address bit
    // alternating, +7 % on the bare store pattern) measured 3 % slower on
    // the real kernel (16 more VGPRs + unpacks), so passes store alone.
    constexpr bool RELOAD = K == 32;
    const int passes = n / K;

    constexpr bool PAIR_ = kEncPair && K == 16 && COLS == 2 && FULL;
    int32_t x[COLS][K];
    auto load_x = [&](uint32_t vo) {
#pragma unroll
        for (int t = 0; t < K; t++) {
            const int row = KEQ ? t : (t < k ? t : k - 1);  // clamp, then mask
            int32_t v[COLS];
            ld<COLS, FULL, BUF>(gi, static_cast<uint32_t>(row) * irs, vo, avail, v);
#pragma unroll
            for (int c = 0; c < COLS; c++)
                x[c][t] = (KEQ || t < k) ? v[c] : 0;
        }
    };
    if constexpr (!RELOAD && !PAIR_)
        load_x(voff);

    // pass v: y[c][u] = output row passes*u + v of column c, in V = [-2, 65537]
    auto compute = [&](int v, int32_t (&y)[COLS][K]) {
        if constexpr (RELOAD) {
            uint32_t vo = voff;
            asm volatile("" : "+v"(vo));  // keep the loads inside the loop
            load_x(vo);
        }
        if (v == 0) {
#pragma unroll
            for (int c = 0; c < COLS; c++) {
#pragma unroll
                for (int t = 0; t < K; t++)
                    y[c][t] = x[c][t];
                dft<K, 0, 65535>(y[c]);
            }
        } else {
            // twist by w^{vt}: |x*c| < 2^31 for x < 2^16, |c| <= 2^15, and
            // one fold leaves [-32767, 98303] (kTwLo/kTwHi), which the
            // codelet plan accepts as its input range
            const int32_t* tw = twist + v * K;
#pragma unroll
            for (int t = 0; t < K; t++) {
                const int32_t cb = tw[t];
#pragma unroll
                for (int c = 0; c < COLS; c++)
                    y[c][t] = t == 0 ? x[c][t] : fold(mul_i24_s(x[c][t], cb));
            }
#pragma unroll
            for (int c = 0; c < COLS; c++)
                dft<K, kTwLo, kTwHi>(y[c]);
        }
    };
    // the stored word is the low 16 bits; any output outside [0, 65535] (the
    // true OOR symbol 65536 or a non-canonical alias) sends the pass through
    // the rare fix-up: canonicalise in place, then record the OOR marks from
    // a bitmask (keeps the atomics out of the unrolled code)
    // The wave takes the fix-up when any of its lanes has such an output
    // (about 64 x 2K x 4 / 65537 = 12 % of the passes at K = 16), so the
    // fix-up is per element and wave-uniform: one compare + ballot per
    // output, and only the elements some lane has out of range are
    // canonicalised (the earlier whole-pass canonicalisation with a 64-bit
    // mark mask cost ~400 instructions per taken pass)
    auto fixup = [&](int v, int32_t (&y)[COLS][K]) {
        uint32_t bad = 0;
#pragma unroll
        for (int u = 0; u < K; u++)
#pragma unroll
            for (int c = 0; c < COLS; c++)
                bad |= static_cast<uint32_t>(y[c][u]);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64((bad >> 16) != 0) != 0, 0)) {
#pragma unroll
            for (int u = 0; u < K; u++) {
#pragma unroll
                for (int c = 0; c < COLS; c++) {
                    if (__builtin_amdgcn_ballot_w64(static_cast<uint32_t>(y[c][u]) > 65535u)) {
                        const uint32_t cv = canon_v(y[c][u]);
                        y[c][u] = static_cast<int32_t>(cv & 0xffffu);
                        const int row = passes * u + v;
                        if (cv == 65536u && oor.counts && (FULL || c < avail) && row < n_out)
                            record_oor(oor, s, row, col + c);
                    }
                }
            }
        }
    };
    // CHK: some rows >= n_out are not wanted (uniform per launch; the
    // checks become a scalar branch around every store, so the common
    // all-rows case gets its own branch-free copy)
    auto run = [&](auto chk) {
        for (int v = 0; v < passes; v++) {
            int32_t y[COLS][K];
            compute(v, y);
            fixup(v, y);
#pragma unroll
            for (int u = 0; u < K; u++) {
                const int row = passes * u + v;
                uint32_t o[COLS];
#pragma unroll
                for (int c = 0; c < COLS; c++)
                    o[c] = static_cast<uint32_t>(y[c][u]);
                if (!decltype(chk)::value || row < n_out)
                    st<COLS, FULL, BUF, kAuxSt>(go, static_cast<uint32_t>(row) * ors,
                                                voff, avail, o);
            }
        }
    };
    // PAIR (K = 16, 2 columns per lane, whole tiles: the cfg2 shape): the
    // passes run in pairs (v, v + 1) and their stores interleave, rows
    // 4u + v, 4u + v + 1, ..., so consecutive 256-byte row stores of a wave
    // alternate the 64 KiB address bit (the pass-order pattern, all 16 rows
    // of a pass in a row, measured 3.61 ms vs 3.34-3.41 ms for row order /
    // pass pairs on the bare store pattern, profiles/r1_membw3.txt,
    // r3_membw4.txt).  The even pass is held packed (16 VGPRs); the inputs
    // stay packed too (16 VGPRs instead of 32: the twist multiplies read a
    // column's 16-bit half with SDWA), so the kernel keeps 4 waves per SIMD.
    auto run_pairs = [&](auto chk) {
        uint32_t xw[K];
#pragma unroll
        for (int t = 0; t < K; t++) {
            const int row = KEQ ? t : (t < k ? t : k - 1);
            uint32_t w[1];
            ld_dw<1, BUF>(gi, static_cast<uint32_t>(row) * irs, voff, w);
            xw[t] = (KEQ || t < k) ? w[0] : 0u;
        }
        auto compute_p = [&](int v, int32_t (&y)[COLS][K]) {
#pragma unroll
            for (int t = 0; t < K; t++) {
                y[0][t] = static_cast<int32_t>(xw[t] & 0xffffu);
                y[1][t] = static_cast<int32_t>(xw[t] >> 16);
            }
            if (v == 0) {
#pragma unroll
                for (int c = 0; c < COLS; c++)
                    dft<K, 0, 65535>(y[c]);
            } else {
                const int32_t* tw = twist + v * K;
#pragma unroll
                for (int t = 1; t < K; t++) {
                    const int32_t cb = tw[t];
                    y[0][t] = fold(mul_i24_lo16(xw[t], cb));
                    y[1][t] = fold(mul_i24_hi16(xw[t], cb));
                }
#pragma unroll
                for (int c = 0; c < COLS; c++)
                    dft<K, kTwLo, kTwHi>(y[c]);
            }
        };
        auto packed = [&](int v, uint32_t (&o)[K]) {
            int32_t y[COLS][K];
            compute_p(v, y);
            fixup(v, y);
#pragma unroll
            for (int u = 0; u < K; u++)
                o[u] = pack_lo(static_cast<uint32_t>(y[0][u]), static_cast<uint32_t>(y[1][u]));
        };
        auto store = [&](int row, uint32_t o) {
            if (!decltype(chk)::value || row < n_out) {
                const uint32_t w[1] = {o};
                st_dw<1, BUF, kAuxSt>(go, static_cast<uint32_t>(row) * ors, voff, w);
            }
        };
        int v = 0;
        for (; v + 1 < passes; v += 2) {
            uint32_t o0[K], o1[K];
            packed(v, o0);
            packed(v + 1, o1);
#pragma unroll
            for (int u = 0; u < K; u++) {
                store(passes * u + v, o0[u]);
                store(passes * u + v + 1, o1[u]);
            }
        }
        if (v < passes) {
            uint32_t o0[K];
            packed(v, o0);
#pragma unroll
            for (int u = 0; u < K; u++)
                store(passes * u + v, o0[u]);
        }
    };
    constexpr bool PAIR = kEncPair && K == 16 && COLS == 2 && FULL;
    if constexpr (PAIR) {
        if (n_out >= n)
            run_pairs(std::integral_constant<bool, false>{});
        else
            run_pairs(std::integral_constant<bool, true>{});
    } else {
        if (n_out >= n)
            run(std::integral_constant<bool, false>{});
        else
            run(std::integral_constant<bool, true>{});
    }
}

template <int K, int COLS, bool KEQ, bool BUF>
// 4 waves per SIMD: the K=16, COLS=2 body fits 128 VGPRs without spills or
// extra instructions (3 waves at the compiler's default 130).  K = 64: 2
// waves (3 waves = 168 VGPRs spilled and ran 20 % slower,
// profiles/r1_ab_k64_encode.txt)
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(K >= 64 ? 2 : 4))) void
encode_fnt_kernel(
    int k, int n, int n_out, const int32_t* __restrict__ twist,
    const uint16_t* __restrict__ data, long long dss, uint32_t irs,
    uint32_t iext, uint16_t* __restrict__ out, long long oss, uint32_t ors,
    uint32_t oext, long long words, int tiles, Oor oor)
{
    int s, tile;
    block_map(blockIdx.x, tiles, s, tile);
    const long long col0 = static_cast<long long>(tile) * kBlock * COLS;
    const long long col = col0 + static_cast<long long>(threadIdx.x) * COLS;
    const Region<BUF> gi(data + s * dss, iext);
    const Region<BUF> go(out + s * oss, oext);
    const uint32_t voff = static_cast<uint32_t>(col * 2);
    if (col0 + kBlock * COLS <= words) {  // block-uniform
        encode_body<K, COLS, true, KEQ, BUF>(k, n, n_out, twist, gi, irs, go,
                                             ors, voff, col, COLS, s, oor);
    } else {
        if (col >= words)
            return;
        encode_body<K, COLS, false, KEQ, BUF>(k, n, n_out, twist, gi, irs, go,
                                              ors, voff, col, words - col, s,
                                              oor);
    }
}

// ---------------------------------------------------------------------------
// Matrix apply: out[t] = sum_i M[t][i] * in[i] over GF(65537) with
// v_dot2_i32_i16 (two 16x16 products + accumulate per instruction).
// Used for decode (M = interpolation matrix of the received ids: the linear
// map computed by FecCode::decode_apply, src/fec_base.h:1418-1448, restated
// as one k x k product), systematic decode and systematic encode.
// ---------------------------------------------------------------------------
constexpr int kMaxTileOor = 256;
typedef short qi_short2 __attribute__((ext_vector_type(2)));

// launch geometry of a matrix kernel: byte extents of the stripe regions it
// touches and its first column (a tail launch starts past the columns the
// matrix-core kernel covered)
struct MatExt {
    uint32_t e0, e1, eo;
    long long c0;
};

// everything a matrix launch needs (one kernel argument block)
struct MatArgs {
    MatLayout L;
    const int32_t* mat;  // per-stripe matrix blocks, ms words apart (0: shared)
    long long ms;
    const int32_t* ids;  // per-stripe int32 ids, is apart (nullptr: identity)
    long long is;
    RowSrc src;
    RowDst dst;
    MatExt ext;
    long long words;
    int tiles;
    Oor in_oor;  // input marks (counts nullptr: none)
    int slot_base;
    Oor out_oor;  // output marks recorded (counts nullptr: none)
    // output row of matrix row t (the plan groups a shared generator's
    // row-scaled rows into as few 16-row blocks as possible); identity for
    // decode matrices
    const int32_t* rowmap;
    const uint32_t* route;
    long long rstride;
    SlowList slow;
    uint32_t* err;
};

// Where the OOR marks of the received rows (decode_prepare's restore of
// 65536, src/fec_base.h:1361-1404) come from in a matrix launch.  A tile
// normally takes them from the context's route table or from one scan of
// the buckets into LDS (kMaxTileOor entries); a tile holding more marks
// than that (adversarial data) sets `slow` and every epilogue walks the
// buckets directly -- slower, but with no limit, as the reference has none.
struct OorScan {
    Oor in;
    const int32_t* sid;  // per-stripe ids (nullptr = identity)
    int by_pos, slot_base, kin, s;
    bool slow;
};

// A tile with more than kMaxTileOor marks (adversarial data; the reference
// has no such limit): the matrix kernels applied only the first
// kMaxTileOor of them and appended the tile to its stripe's slow list (in
// the decode context); matrix_redo_kernel, launched right after them on the
// same stream, recomputes every column of the tile that holds a mark from
// scratch -- all marks of the column restored, plain canonical arithmetic
// -- and stores it again.  Only decodes carry input marks, and their
// outputs are data symbols (< 65536), so nothing is recorded as OOR here.
// Keeping this out of the hot kernels keeps their registers: inlined at
// their end it held the bucket and row pointers live across the MFMA loop
// (SGPR spills, 2x slower decode).
__device__ __forceinline__ void push_slow_tile(const SlowList& sl, int s, long long col0,
                                               int width)
{
    // width: a power-of-two multiple of kSlowGrain (64 .. 1024 columns)
    uint32_t* l = sl.base + s * sl.stride;
    const uint32_t idx = atomicAdd(l, 1u);
    l[1 + idx] = static_cast<uint32_t>(col0 / kSlowGrain) << 3 |
                 static_cast<uint32_t>(ilog2c(static_cast<uint32_t>(width / kSlowGrain)));
}

// One block per stripe at a time; a slow tile is redone in chunks of
// kRedoCols columns: the chunk's received symbols (u16) and a bitmap of
// their marks staged in LDS (every mark of every received row, from the
// buckets), then lane c of wave wv recomputes column c for the output rows
// wv, wv + 4, ... (the coefficient, read back from the operand tiles by
// mf_entry, is wave-uniform: scalar loads) -- only in columns that hold a
// mark.  Work per chunk is
// R * kin * 64 multiply-adds whatever the mark density (walking the marks
// per (mark, row, input) was quadratic in the density).  The stripe's list
// is emptied afterwards (a context can serve several decodes).
constexpr int kRedoCols = 64;

// Recompute, from scratch, every column of stripe s's columns [t0c, t1c)
// that holds a mark (all marks of the column restored, plain canonical
// arithmetic) and store it again: NT threads, LDS scratch xs (kin x
// kRedoCols u16), mk (kin x kRedoCols / 32 u32), colmk (kRedoCols / 32 u32).
// The caller has waited for its own stores of these columns.  Only the
// output rows of row blocks gq, gq + G, gq + 2G, ... (16 rows each) are
// recomputed: a block of matrix_os_kernel redoes just the rows it stored
// itself (G row-block groups share a column range), so no two blocks write
// the same outputs; other callers pass gq = 0, G = 1 (every row).
template <int NT>
__device__ void redo_columns(const MatArgs& a, int s, long long t0c, long long t1c,
                             uint16_t* xs, uint32_t* mk, uint32_t* colmk, int gq = 0,
                             int G = 1)
{
    const MatLayout L = a.L;
    const int kin = L.kin;
    const RowSrc& src = a.src;
    const RowDst& dst = a.dst;
    const Oor& in = a.in_oor;
    const int tid = threadIdx.x, c = tid & 63, wv = tid >> 6;
    const int32_t* M = a.mat + s * a.ms;
    const int32_t* sid = a.ids ? a.ids + s * a.is : nullptr;
    const int32_t* rscale = M + L.rscale();
    const int32_t* mf = M + L.mf();
    auto id_of = [&](int i) { return src.by_pos ? i : (sid ? sid[i] : i); };
    for (long long c0 = t0c; c0 < t1c; c0 += kRedoCols) {
        for (int j = tid; j < kin * (kRedoCols / 32); j += NT)
            mk[j] = 0;
        if (tid < kRedoCols / 32)
            colmk[tid] = 0;
        // the chunk's received symbols, one row of 64 per wave pass
        for (int i = wv; i < kin; i += NT / 64) {
            const int id = id_of(i);
            const uint16_t* row = id < src.split
                                      ? src.base0 + s * src.ss0 + id * src.rs0
                                      : src.base1 + s * src.ss1 + (id - src.split) * src.rs1;
            xs[i * kRedoCols + c] = c0 + c < t1c ? row[c0 + c] : 0;
        }
        __syncthreads();
        // every mark of every received row inside the chunk
        for (int i = tid; i < kin; i += NT) {
            const int slot = (src.by_pos ? i : id_of(i)) - a.slot_base;
            if (slot < 0)
                continue;  // systematic data row: no marks
            const long long bk = static_cast<long long>(s) * in.slots + slot;
            const uint32_t cnt = min(in.counts[bk], static_cast<uint32_t>(in.cap));
            for (uint32_t f = 0; f < cnt; f++) {
                const long long w = in.entries[bk * in.cap + f];
                if (w >= c0 && w < c0 + kRedoCols && w < t1c) {
                    const int cc = static_cast<int>(w - c0);
                    atomicOr(&mk[i * (kRedoCols / 32) + cc / 32], 1u << (cc % 32));
                    atomicOr(&colmk[cc / 32], 1u << (cc % 32));
                }
            }
        }
        __syncthreads();
        if ((colmk[c / 32] >> (c % 32)) & 1u) {
            const int nrows = 16 * ((L.RB() - gq + G - 1) / G);
            for (int it = wv; it < nrows; it += NT / 64) {
                const int t = 16 * (gq + G * (it >> 4)) + (it & 15);
                if (t >= L.R)
                    continue;
                uint64_t acc = 0;
                for (int j = 0; j < kin; j++) {
                    const uint32_t x = (mk[j * (kRedoCols / 32) + c / 32] >> (c % 32)) & 1u
                                           ? 65536u
                                           : xs[j * kRedoCols + c];
                    acc += static_cast<uint64_t>(mf_entry(L, mf, t, j)) * x;
                }
                uint32_t y = static_cast<uint32_t>(acc % 65537u);
                const int32_t rs = rscale[t];
                if (rs != 1)
                    y = static_cast<uint32_t>(static_cast<uint64_t>(y) *
                                              static_cast<uint32_t>(rs < 0 ? rs + kQ : rs) %
                                              65537u);
                dst.base[s * dst.ss + a.rowmap[t] * dst.rs + c0 + c] =
                    static_cast<uint16_t>(y == 65536u ? 0u : y);
            }
        }
        __syncthreads();
    }
}

// A block's slow tiles (see push_slow_tile), redone by the block itself at
// its end, after its waves' stores: the separate redo launch cost 4-5 us per
// decode even with nothing to redo.  Waits for this wave's outstanding
// memory operations (stores included), then the block barrier.
__device__ __forceinline__ void drain_block_stores()
{
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
    __syncthreads();
}

// The dot2 kernel's slow tiles (column tails, unaligned rows): kept in the
// context's slow list and redone by this launch after it.  A block checks
// the lists of kRedoSpan stripes at once (one lane each) and walks only the
// stripes holding slow tiles.
constexpr int kRedoSpan = 64;

__global__ __launch_bounds__(kBlock) void matrix_redo_kernel(MatArgs a, int n_stripes)
{
    // (the dot2 tails' slow tiles: k <= 256; the operand-stationary kernel
    // redoes its own in its dynamic LDS)
    __shared__ uint16_t xs[kMatGenMaxKin * kRedoCols];  // [input i][column]
    __shared__ uint32_t mk[kMatGenMaxKin * (kRedoCols / 32)];
    __shared__ uint32_t colmk[kRedoCols / 32];
    const int tid = threadIdx.x, c = tid & 63, wv = tid >> 6;
    // this block's stripes with a non-empty list (wave 0, one lane each;
    // broadcast to the block through LDS)
    __shared__ uint64_t todo;
    const int s0 = blockIdx.x * kRedoSpan;
    if (wv == 0) {
        const int sl = s0 + c;
        const uint32_t nl = sl < n_stripes
                                ? __hip_atomic_load(a.slow.base + sl * a.slow.stride,
                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                : 0u;
        const uint64_t m = __builtin_amdgcn_ballot_w64(nl != 0);
        if (c == 0)
            todo = m;
    }
    __syncthreads();
    uint64_t pend = todo;
    while (pend) {
        const int s = s0 + __builtin_ctzll(pend);  // block-uniform
        pend &= pend - 1;
        uint32_t* l = a.slow.base + s * a.slow.stride;
        const uint32_t n = *l;
        for (uint32_t e = 0; e < n; e++) {
            const uint32_t code = l[1 + e];
            const long long t0 = static_cast<long long>(code >> 3) * kSlowGrain;
            const long long t1 = min(t0 + (static_cast<long long>(kSlowGrain) << (code & 7)),
                                     a.words);
            redo_columns<kBlock>(a, s, t0, t1, xs, mk, colmk);
        }
        __syncthreads();
        if (tid == 0)
            *l = 0;
    }
}

// the context's routed marks of this tile (count <= kRouteCap, entries
// pos << 16 | column in the kRouteTile tile) into the LDS list (s_i, s_col)
__device__ __forceinline__ void stage_route_marks(const uint32_t* rm, int n_rm,
                                                  long long col0, int* s_i,
                                                  uint32_t* s_col)
{
    if (static_cast<int>(threadIdx.x) < n_rm) {
        const uint32_t v = rm[threadIdx.x];
        s_i[threadIdx.x] = static_cast<int>(v >> 16);
        s_col[threadIdx.x] =
            static_cast<uint32_t>(col0 / kRouteTile * kRouteTile + (v & 0xffffu));
    }
}

// The same from the route-table entry rt (count + kRouteCap entries), the
// count by a scalar load (constant address space).  VEC: the entries by the
// lanes that stage one, with a vector load; otherwise all 16 dwords by
// scalar loads (round 5: a vector load is ordered with the kernel's
// streaming stores and row prefetch in vmcnt, and waiting for it drained
// both every tile).  The callers stage a route tile's list once per mark
// buffer, and only wave 0 issues the vector load; the 16 SGPRs of the
// scalar form had pushed the KS = 4 kernel to ~75 SGPR spills (VEC there:
// cfg3 decode -2 us, k200 / k300 -1 %; at KS = 8 the scalar form measured
// 1.5 % faster, k128).  Returns the count, or -1 when the tile overflowed
// the table (scan the buckets).
template <bool VEC>
__device__ __forceinline__ int stage_route_marks_s(const uint32_t* rt, long long col0, int* s_i,
                                                   uint32_t* s_col)
{
    using CU = const __attribute__((address_space(4))) uint32_t;
    CU* c = (CU*)rt;
    if constexpr (!VEC) {
        uint32_t e[kRouteStride];
#pragma unroll
        for (int i = 0; i < kRouteStride; i++)
            e[i] = c[i];
        const uint32_t rc = e[0];
        if (rc > static_cast<uint32_t>(kRouteCap))
            return -1;
        const int tid = static_cast<int>(threadIdx.x);
        if (tid < static_cast<int>(rc)) {
            uint32_t v = 0;
#pragma unroll
            for (int i = 0; i < kRouteCap; i++)
                v = tid == i ? e[1 + i] : v;
            s_i[tid] = static_cast<int>(v >> 16);
            s_col[tid] = static_cast<uint32_t>(col0 / kRouteTile * kRouteTile + (v & 0xffffu));
        }
        return static_cast<int>(rc);
    }
    const uint32_t rc = c[0];
    if (rc > static_cast<uint32_t>(kRouteCap))
        return -1;
    const int tid = static_cast<int>(threadIdx.x);
    if (tid < static_cast<int>(rc)) {
        const uint32_t v = rt[1 + tid];
        s_i[tid] = static_cast<int>(v >> 16);
        s_col[tid] = static_cast<uint32_t>(col0 / kRouteTile * kRouteTile + (v & 0xffffu));
    }
    return static_cast<int>(rc);
}

// block-wide scan of the buckets into the LDS list (s_i, s_col) of the
// marks inside columns [col0, col1); returns the number of marks found
// (> kMaxTileOor: the list is incomplete, use the slow path)
__device__ __forceinline__ int scan_tile_marks(const OorScan& sc, long long col0,
                                               long long col1, long long words,
                                               int* s_cnt, int* s_i, uint32_t* s_col,
                                               uint32_t* err)
{
    if (threadIdx.x == 0)
        *s_cnt = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < sc.kin; i += blockDim.x) {
        const int id = sc.sid ? sc.sid[i] : i;
        const int slot = (sc.by_pos ? i : id) - sc.slot_base;
        if (slot < 0)
            continue;
        const long long bk = static_cast<long long>(sc.s) * sc.in.slots + slot;
        uint32_t c = sc.in.counts[bk];
        if (c > static_cast<uint32_t>(sc.in.cap)) {
            atomicOr(err, kErrOorTruncated);
            c = static_cast<uint32_t>(sc.in.cap);
        }
        for (uint32_t e = 0; e < c; e++) {
            const uint32_t w = sc.in.entries[bk * sc.in.cap + e];
            if (w >= col0 && w < col1 && w < words) {
                const int p = atomicAdd(s_cnt, 1);
                if (p < kMaxTileOor) {
                    s_i[p] = i;
                    s_col[p] = w;
                }
            }
        }
    }
    __syncthreads();
    return *s_cnt;
}

template <int KP, int COLS, bool FULL, bool BUF, class IdOf>
__device__ __forceinline__ void matrix_load(const IdOf& id_of,
                                            const RowSrc& src,
                                            const Region<BUF>& g0,
                                            const Region<BUF>& g1, uint32_t voff,
                                            long long avail,
                                            int32_t (&xp)[COLS][KP])
{
    // every row pair, branch-free, offset to signed 16 bit (x - 32768) and
    // packed [row 2j, row 2j+1] per column for dot2.  Rows past kin load a
    // valid (clamped) row and need no masking: their packed coefficients are
    // 0 and kcorr sums only the real ones (pack_row).
#pragma unroll
    for (int j = 0; j < KP; j++) {
        Region<BUF> g[2] = {g0, g0};
        uint32_t off[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int id = id_of(2 * j + h);
            // branch-free source select (uniform s_cselect): a branch here
            // makes the compiler drain vmcnt after every row load
            const bool lo = id < src.split;
            if constexpr (BUF)
                g[h].r = lo ? g0.r : g1.r;
            g[h].p = lo ? g0.p : g1.p;
            off[h] = static_cast<uint32_t>(lo ? id * src.rs0 * 2
                                              : (id - src.split) * src.rs1 * 2);
        }
        if constexpr (FULL && COLS % 2 == 0) {
            uint32_t w0[COLS / 2], w1[COLS / 2];
            ld_dw<COLS / 2, BUF, kAuxLd>(g[0], off[0], voff, w0);
            ld_dw<COLS / 2, BUF, kAuxLd>(g[1], off[1], voff, w1);
#pragma unroll
            for (int d = 0; d < COLS / 2; d++) {
                xp[2 * d][j] = static_cast<int32_t>(
                    __builtin_amdgcn_perm(w1[d], w0[d], 0x05040100u) ^ 0x80008000u);
                xp[2 * d + 1][j] = static_cast<int32_t>(
                    __builtin_amdgcn_perm(w1[d], w0[d], 0x07060302u) ^ 0x80008000u);
            }
        } else {
            int32_t vv[2][COLS];
            ld<COLS, FULL, BUF, kAuxLd>(g[0], off[0], voff, avail, vv[0]);
            ld<COLS, FULL, BUF, kAuxLd>(g[1], off[1], voff, avail, vv[1]);
#pragma unroll
            for (int c = 0; c < COLS; c++)
                xp[c][j] = static_cast<int32_t>(
                    pack_lo(static_cast<uint32_t>(vv[0][c]),
                            static_cast<uint32_t>(vv[1][c])) ^
                    0x80008000u);
        }
    }
}

template <int KP, int COLS, bool FULL, bool BUF>
__device__ __forceinline__ void matrix_compute(
    const MatLayout& L, const int32_t* __restrict__ M,
    const int32_t (&xp)[COLS][KP], const Region<BUF>& go, uint32_t ors,
    uint32_t voff, long long col, long long col0, long long avail, int s,
    int n_lm, const int* s_i, const uint32_t* s_col, const Oor& out_oor,
    const int32_t* __restrict__ rowmap)
{
    // M: the per-stripe matrix block (wave-uniform: scalar loads)
    const int kin = L.kin;
    const int32_t* kcorr = M + L.kcorr();
    const int32_t* rscale = M + L.rscale();
    const int32_t* plain = M + L.plain();
    const bool rec = out_oor.counts != nullptr;
    for (int t = 0; t < L.R; t++) {
        const int32_t* mrow = M + t * KP;
        int32_t acc[COLS];
#pragma unroll
        for (int c = 0; c < COLS; c++)
            acc[c] = kcorr[t];
#pragma unroll
        for (int j = 0; j < KP; j++) {
            const qi_short2 m2 = __builtin_bit_cast(qi_short2, mrow[j]);
#pragma unroll
            for (int c = 0; c < COLS; c++)
                acc[c] = fold(__builtin_amdgcn_sdot2(
                    __builtin_bit_cast(qi_short2, xp[c][j]), m2, acc[c], false));
        }
        int32_t y[COLS];
#pragma unroll
        for (int c = 0; c < COLS; c++)
            y[c] = fold(acc[c]);  // T-range
        // restored OOR symbols: 65536 == -1 where the stored word is 0
        for (int e = 0; e < n_lm; e++) {
            const int pos = s_i[e];
            const long long w = s_col[e];
            // branch-free per lane, unconditional load consumed at once (see
            // the matrix-core epilogue: a load under a divergent branch made
            // the compiler drain vmcnt(0) after every row)
            const long long d = w - col;
            const int32_t corr = plain[t * kin + pos];
#pragma unroll
            for (int c = 0; c < COLS; c++) {
                const int32_t yc = fold(fold(y[c] - corr));
                y[c] = d == c ? yc : y[c];
            }
        }
        const int32_t rs = rscale[t];
        if (rs != 1) {
#pragma unroll
            for (int c = 0; c < COLS; c++)
                y[c] = fold(fold(mul_rs(y[c], rs)));
        }
        uint32_t o[COLS];
        uint32_t bad = 0;
#pragma unroll
        for (int c = 0; c < COLS; c++) {
            o[c] = static_cast<uint32_t>(y[c]);
            bad |= o[c];
        }
        if (__builtin_expect((bad >> 16) != 0, 0)) {
#pragma unroll
            for (int c = 0; c < COLS; c++) {
                if (static_cast<uint32_t>(y[c]) > 65535u && rec &&
                    (FULL || c < avail))
                    record_oor(out_oor, s, rowmap[t], col + c);
                o[c] = fix16(y[c]);
            }
        }
        st<COLS, FULL, BUF, kAuxSt>(go, static_cast<uint32_t>(rowmap[t]) * ors, voff, avail,
                                    o);
    }
}

template <int KP, int COLS, bool BUF>
__global__ __launch_bounds__(kBlock) void matrix_kernel(MatArgs a)
{
    const MatLayout L = a.L;
    const int32_t* __restrict__ mat = a.mat;
    const long long mat_stride = a.ms;
    const int32_t* __restrict__ ids = a.ids;
    const long long ids_stride = a.is;
    const RowSrc src = a.src;
    const RowDst dst = a.dst;
    const MatExt ext = a.ext;
    const long long words = a.words;
    const int tiles = a.tiles;
    const Oor in_oor = a.in_oor;
    const int slot_base = a.slot_base;
    const Oor out_oor = a.out_oor;
    const uint32_t* __restrict__ route = a.route;
    const long long route_stride = a.rstride;
    const SlowList slow = a.slow;
    uint32_t* err = a.err;
    __shared__ int s_cnt;
    __shared__ int s_i[kMaxTileOor];
    __shared__ uint32_t s_col[kMaxTileOor];

    int s, tile;
    block_map(blockIdx.x, tiles, s, tile);
    const int kin = L.kin;
    const long long col0 = ext.c0 + static_cast<long long>(tile) * kBlock * COLS;
    const long long col1 = col0 + kBlock * COLS;
    const long long col = col0 + static_cast<long long>(threadIdx.x) * COLS;
    const uint32_t voff = static_cast<uint32_t>(col * 2);
    const int32_t* M = mat + s * mat_stride;
    // fragment ids as dwords (scalar loads; a u16 array would need vector
    // loads + readfirstlane, draining vmcnt between the row loads)
    const int32_t* sid = ids ? ids + s * ids_stride : nullptr;
    const bool full = col1 <= words;  // block-uniform
    const Region<BUF> g0(src.base0 + s * src.ss0, ext.e0);
    const Region<BUF> g1(src.base1 ? src.base1 + s * src.ss1 : src.base0,
                         ext.e1);
    const Region<BUF> go(dst.base + s * dst.ss, ext.eo);

    // the OOR marks of the received rows in this tile (decode_prepare,
    // src/fec_base.h:1361-1404): from the context's route table (scalar
    // loads, issued with the row loads), or -- when the table overflowed or
    // is absent -- by scanning the OOR buckets
    int n_rm = 0;
    const uint32_t* rm = nullptr;
    bool scan = in_oor.counts != nullptr;
    if (route) {
        const uint32_t* rt =
            route + s * route_stride + (col0 / kRouteTile) * kRouteStride;
        const uint32_t rc = rt[0];
        if (rc <= static_cast<uint32_t>(kRouteCap)) {
            n_rm = static_cast<int>(rc);
            rm = rt + 1;
            scan = false;
        }
    }

    // source row of input i: its position (by_pos) or its fragment id; rows
    // past kin are clamped to a valid row (their coefficients are 0).
    // KP <= 32: all ids up front in SGPRs (2*KP dwords, the context pads
    // past kin), so the scalar loads batch into a few s_load_dwordxN.
    // KP >= 64 (the column tails of k > 64): 128-256 ids do not fit the
    // SGPRs (they spilled to VGPR lanes and scratch), so lane c of
    // idl[i / 64] holds id i and the row loads read it with v_readlane.
    constexpr int NIL = KP >= 64 ? 2 * KP / 64 : 1;
    constexpr int NIV = KP >= 64 ? 1 : 2 * KP;
    int idl[NIL];
    int idv[NIV];
    if constexpr (KP >= 64) {
        const int ln = static_cast<int>(threadIdx.x & 63);
#pragma unroll
        for (int c = 0; c < NIL; c++) {
            const int i = 64 * c + ln;
            const int ii = i < kin ? i : kin - 1;
            idl[c] = src.by_pos ? ii : (sid ? sid[i < kin ? i : 0] : (i < kin ? i : 0));
        }
        (void)idv;
    } else {
        (void)idl;
        if (sid) {
#pragma unroll
            for (int i = 0; i < 2 * KP; i++)
                idv[i] = sid[i];
        } else {
#pragma unroll
            for (int i = 0; i < 2 * KP; i++)
                idv[i] = i;
        }
#pragma unroll
        for (int i = 0; i < 2 * KP; i++) {
            const int ii = i < kin ? i : kin - 1;
            idv[i] = src.by_pos ? ii : (i < kin ? idv[i] : idv[0]);
        }
    }
    auto id_of = [&](int i) {
        if constexpr (KP >= 64)
            return __builtin_amdgcn_readlane(idl[i / 64], i % 64);
        else
            return idv[i];
    };
    int32_t xp[COLS][KP];
    if (full) {
        matrix_load<KP, COLS, true, BUF>(id_of, src, g0, g1, voff, COLS, xp);
    } else if (col < words) {
        matrix_load<KP, COLS, false, BUF>(id_of, src, g0, g1, voff,
                                          words - col, xp);
    }
    OorScan sc{in_oor, sid, src.by_pos, slot_base, kin, s, false};
    int n_lm = 0;
    if (scan) {  // block-uniform
        const int cnt = scan_tile_marks(sc, col0, col1, words, &s_cnt, s_i, s_col, err);
        sc.slow = cnt > kMaxTileOor;
        n_lm = min(cnt, kMaxTileOor);
    } else if (n_rm > 0) {  // block-uniform: the routed marks into the same list
        stage_route_marks(rm, n_rm, col0, s_i, s_col);
        __syncthreads();
        n_lm = n_rm;
    }
    const uint32_t ors = static_cast<uint32_t>(dst.rs * 2);
    if (full) {
        matrix_compute<KP, COLS, true, BUF>(L, M, xp, go, ors, voff, col, col0,
                                            COLS, s, n_lm, s_i, s_col, out_oor,
                                            a.rowmap);
    } else if (col < words) {
        matrix_compute<KP, COLS, false, BUF>(L, M, xp, go, ors, voff, col, col0,
                                             words - col, s, n_lm, s_i, s_col,
                                             out_oor, a.rowmap);
    }
    if (sc.slow && threadIdx.x == 0)  // rare: see matrix_redo_kernel
        push_slow_tile(slow, s, col0, kBlock * COLS);
}

// ---------------------------------------------------------------------------
// Matrix apply on the matrix cores (v_mfma_i32_16x16x32_i8 at KS = 1,
// v_mfma_i32_16x16x64_i8 above), kin <= 256.
//
// The product of matrix_kernel, out[t] = sum_i M[t][i] x_i mod q, with the
// u16 inputs and the row-scaled coefficients split into signed bytes:
//   x = 256 h' + l' + 32896        h' = (x >> 8) - 128, l' = (x & 255) - 128
//   c = 256 a + b                  a, b in [-128, 127] (split_i8)
// and 2^16 = -1 (mod q):
//   sum_i c x = 256 D2 + D1 - D0 + 32896 sum_i c
//   D0 = sum a h',  D1 = sum b l',  D2 = sum b h' + a l'
// -- three int8 GEMMs over K = [h' rows ; l' rows] against the per-stripe
// operand tiles [a|0], [0|b], [b|a] (matrix_pack.h pack_mf_dword; D1 starts
// at kmf[t] = 32896 sum c).  |D| <= 2 kin 128^2: up to kin = 128 (2^22)
// 256 D2 + D1 - D0 stays inside int32; at KS = 16 (kin <= 256, |D2| <= 2^23)
// the epilogue folds D2 before the shift.  The dot2 kernel's ~19 VALU
// per (output, column) become ~5 of epilogue, so the decode is HBM-bound
// rather than VALU-bound.
//
// Orientation D^T = X^T M^T: the A operand is the tile's byte planes,
// staged in LDS and read with ds_read_b64_tr_b8 (lane 2q+p of a 16-lane
// group addresses row q, bytes 8p..8p+7 of an 8 x 16-byte block; lane i gets
// column i -- profiles/r1_mfma_probe.txt); the B operand is the coefficient
// tile, pre-swizzled in lane order.  A lane's 4 results are 4 adjacent LDS
// columns of ONE output row t = lane & 15.  The LDS image stores column
// u = 16 g + 4 T + j of every 64-column super tile at byte 4 g + j of 16-byte
// chunk T, so after the 4 chunks of a super tile lane (g, t) holds the 16
// contiguous columns 16 g .. 16 g + 15 of row t: two b128 stores.
// Whole kRouteTile column tiles only; launch_matrix sends the tail to
// matrix_kernel.
// ---------------------------------------------------------------------------
typedef int qi_v4i __attribute__((ext_vector_type(4)));
// (The tall KS = 4 generators -- cfg3's 1024 x 64 -- run gen_mfma_kernel;
// this kernel's super-tile loop is plain.  Round 3's pipelined pair loop for
// them, the next tile's MFMAs interleaved with this one's epilogue, measured
// no gain against a plain loop in round 5: profiles/r5_ab_notes.txt.)
typedef int qi_v2i __attribute__((ext_vector_type(2)));
typedef unsigned int qi_v4u __attribute__((ext_vector_type(4)));

// Geometry of a matrix-core block: NST super tiles of 64 columns (the
// block's columns, staged once as the A image), NW waves.  RSPLIT: the waves
// split the row blocks (wave wv takes wv, wv + NW, ...) and each walks every
// super tile, so an operand tile is fetched once per block; otherwise every
// wave takes every row block over its own NST / NW super tiles.
template <int KS, int NST, int NW>
struct MfmaTile {
    static constexpr int kThreads = 64 * NW;
    static constexpr int kCols = 64 * NST;     // columns per block
    static constexpr int kRows = 16 * KS;      // rows per byte plane
    static constexpr int kPitch = kCols + 16;  // LDS row pitch: +4 banks/row
    static constexpr size_t kImg = static_cast<size_t>(2 * kRows) * kPitch;
    // image + OOR scan scratch (s_i, s_col) + s_cnt
    static constexpr size_t kLds = kImg + 2 * 4 * kMaxTileOor + 16;
    // per-wave output staging tile (16 rows x 128 bytes, padded), only
    // allocated when the block has several 16-row output blocks
    static constexpr int kStagePitch = 144;
    static constexpr size_t kStage = 16 * kStagePitch;
    static constexpr size_t kLdsStaged = kLds + NW * kStage;
    // staging loads: CPL columns per lane (b64 or b32), TPR lanes per image
    // row, RG row groups
    // (b64 staging loads at 512-column blocks -- 32 rows per thread
    // instead of 64 -- measured the cfg3 encode 6 % slower, decode equal)
    static constexpr int kCpl = kCols >= 4 * kThreads ? 4 : 2;
    static constexpr int kTpr = kCols / kCpl;
    static constexpr int kRg = kThreads / kTpr;
    static_assert(kRg >= 1 && kThreads % kTpr == 0 && kRows % kRg == 0, "staging");
};

template <int KS, int NST, int NW, bool RSPLIT>
__global__ __launch_bounds__(64 * NW) void matrix_mfma_kernel(MatArgs a)
{
    const MatLayout L = a.L;
    const int32_t* __restrict__ mat = a.mat;
    const long long mat_stride = a.ms;
    const int32_t* __restrict__ ids = a.ids;
    const long long ids_stride = a.is;
    const RowSrc src = a.src;
    const RowDst dst = a.dst;
    const MatExt ext = a.ext;
    const long long words = a.words;
    const int tiles = a.tiles;
    const Oor in_oor = a.in_oor;
    const int slot_base = a.slot_base;
    const Oor out_oor = a.out_oor;
    const uint32_t* __restrict__ route = a.route;
    const long long route_stride = a.rstride;
    uint32_t* err = a.err;
    using G = MfmaTile<KS, NST, NW>;
    constexpr int NCOL = G::kCols, KH = G::kRows, RSB = G::kPitch;
    constexpr int CPL = G::kCpl, RG = G::kRg;
    // one dynamic region (16-byte aligned base: no static LDS in front)
    extern __shared__ __attribute__((aligned(16))) uint8_t qi_lds[];
    uint8_t* img = qi_lds;
    int* s_i = reinterpret_cast<int*>(qi_lds + G::kImg);
    uint32_t* s_col = reinterpret_cast<uint32_t*>(s_i + kMaxTileOor);
    int* s_cnt = reinterpret_cast<int*>(s_col + kMaxTileOor);

    int s, tile;
    block_map(blockIdx.x, tiles, s, tile);
    const int kin = L.kin;
    const long long col0 = static_cast<long long>(tile) * NCOL;
    const long long col1 = col0 + NCOL;
    // staging: this thread's first column and its row group
    const uint32_t cl = (RG == 1 ? threadIdx.x : threadIdx.x % G::kTpr) * CPL;
    const int rg = RG == 1 ? 0 : static_cast<int>(threadIdx.x / G::kTpr);
    const uint32_t voff = static_cast<uint32_t>((col0 + cl) * 2);
    const int32_t* M = mat + s * mat_stride;
    const int32_t* sid = ids ? ids + s * ids_stride : nullptr;
    const Region<true> g0(src.base0 + s * src.ss0, ext.e0);
    const Region<true> g1(src.base1 ? src.base1 + s * src.ss1 : src.base0,
                          ext.e1);
    const Region<true> go(dst.base + s * dst.ss, ext.eo);

    // OOR marks of the received rows in this tile: route table (scalar
    // loads) or bucket scan, as matrix_kernel
    int n_rm = 0;
    const uint32_t* rm = nullptr;
    bool scan = in_oor.counts != nullptr;
    if (route) {
        const uint32_t* rt =
            route + s * route_stride + (col0 / kRouteTile) * kRouteStride;
        const uint32_t rc = rt[0];
        if (rc <= static_cast<uint32_t>(kRouteCap)) {
            n_rm = static_cast<int>(rc);
            rm = rt + 1;
            scan = false;
        }
    }

    // operand tiles of output block 0 (per-lane loads; issued before the row
    // loads so their latency hides behind the staging)
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int g = l >> 4, q = (l & 15) >> 1, p = l & 1, tl = l & 15;
    const int RB = L.RB();
    const int32_t* mf = M + L.mf();
    const int32_t* kmf = M + L.kmf();
    const int32_t* rscale = M + L.rscale_mf();
    const int32_t* __restrict__ rowmap = a.rowmap;
    auto load_ops = [&](int rb, qi_v2i (&b)[KS][3], int32_t& kt, int32_t& rs, int32_t (&pr)[3]) {
        // [b | a] is [0 | b] of the l' half over the h' K-steps and [a | 0]
        // of the h' half over the l' K-steps, lane for lane (the same K
        // offset within the half): from those registers at KS >= 2 (the
        // contexts do not store it); at KS = 1 the halves share a K-step
        // and sit in other lanes, so it is loaded
#pragma unroll
        for (int ks = 0; ks < KS; ks++)
#pragma unroll
            for (int ty = 0; ty < (KS >= 2 ? 2 : 3); ty++)
                b[ks][ty] = *reinterpret_cast<const qi_v2i*>(
                    mf + ((rb * KS + ks) * 3 + ty) * 128 + l * 2);
        if constexpr (KS >= 2) {
#pragma unroll
            for (int ks = 0; ks < KS; ks++)
                b[ks][2] = ks < KS / 2 ? b[ks + KS / 2][1] : b[ks - KS / 2][0];
        }
        // unconditional loads (a clamped row), selected after: an exec-masked
        // load leaves the compiler unsure how many vector-memory ops are in
        // flight, and it then drains vmcnt further than needed
        const int t = 16 * rb + tl, tc = t < L.R ? t : L.R - 1;
        const int32_t k0 = kmf[tc], r0 = rscale[tc];
        kt = t < L.R ? k0 : 0;
        rs = t < L.R ? r0 : 1;
        // output rows: this lane's epilogue row and its two store rows
        pr[0] = rowmap[tc];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int ot = 16 * rb + 8 * h + (l >> 3);
            pr[1 + h] = rowmap[ot < L.R ? ot : L.R - 1];
        }
    };
    // tall matrices (RSPLIT, the encode generators): wave wv takes row
    // blocks wv, wv + NW, ... over all the block's super tiles, so each wave
    // fetches only its own operand tiles (NW x fewer L2 operand reads than
    // every wave walking every row block); otherwise every wave takes every
    // row block over its own super tiles
    constexpr bool rsplit = RSPLIT;
    const int rb0 = rsplit ? wv : 0, rbs = rsplit ? NW : 1;
    constexpr int nst = rsplit ? NST : NST / NW;
    static_assert(rsplit || NST % NW == 0, "super tiles per wave");

    // the first row block's operands, issued ahead of the row loads
    qi_v2i bA[KS][3], bB[KS][3];
    int32_t ktA, rsA, ktB, rsB, prA[3], prB[3];
    const int rlast = RB - 1;
    const bool single = rb0 + rbs >= RB;
    load_ops(min(rb0, rlast), bA, ktA, rsA, prA);

    // stage the tile as byte planes h' (rows 0..KH-1) and l' (rows KH..):
    // this thread's CPL columns of every RG-th row, all row loads issued back
    // to back; rows past kin load a clamped row (their operand bytes are 0)
    uint32_t w[KH / RG][CPL / 2];
    if constexpr (G::kTpr % 64 == 0) {
        // the row group is wave-uniform: every id of the thread's rows in
        // SGPRs first (the scalar loads issue together; loading each id
        // next to its row load made a chain of KH dependent scalar loads,
        // one lgkmcnt(0) per row), then the row loads back to back -- with
        // one source region (every decode but the systematic one, and the
        // encode) a row offset is one scalar multiply
        int idv[KH / RG];
        if (sid && !src.by_pos) {
#pragma unroll
            for (int r = 0; r < KH / RG; r++) {
                const int i = r * RG + rg;
                idv[r] = sid[i < kin ? i : kin - 1];
            }
        } else {
#pragma unroll
            for (int r = 0; r < KH / RG; r++) {
                const int i = r * RG + rg;
                idv[r] = i < kin ? i : kin - 1;
            }
        }
        if (!src.base1) {
            const uint32_t rsb = static_cast<uint32_t>(src.rs0 * 2);
#pragma unroll
            for (int r = 0; r < KH / RG; r++)
                ld_dw<CPL / 2, true, kAuxLd>(g0, static_cast<uint32_t>(idv[r]) * rsb, voff,
                                             w[r]);
        } else {
#pragma unroll
            for (int r = 0; r < KH / RG; r++) {
                const int id = idv[r];
                const bool lo = id < src.split;
                Region<true> g = g0;
                g.r = lo ? g0.r : g1.r;
                const uint32_t off = static_cast<uint32_t>(
                    lo ? id * src.rs0 * 2 : (id - src.split) * src.rs1 * 2);
                ld_dw<CPL / 2, true, kAuxLd>(g, off, voff, w[r]);
            }
        }
    } else {
#pragma unroll
        for (int r = 0; r < KH / RG; r++) {
            const int i = r * RG + rg;
            const int ii = i < kin ? i : kin - 1;
            const int id = src.by_pos ? ii : (sid ? sid[ii] : ii);
            const bool lo = id < src.split;
            Region<true> g = g0;
            g.r = lo ? g0.r : g1.r;
            const uint32_t off = static_cast<uint32_t>(
                lo ? id * src.rs0 * 2 : (id - src.split) * src.rs1 * 2);
            ld_dw<CPL / 2, true, kAuxLd>(g, off, voff, w[r]);
        }
    }
    const uint32_t lpos = 64 * (cl / 64) + 16 * ((cl % 16) / 4) +
                          4 * ((cl % 64) / 16) + cl % 4;
#pragma unroll
    for (int r = 0; r < KH / RG; r++) {
        const int i = r * RG + rg;
        if constexpr (CPL == 4) {
            // [c0 lo, c0 hi, c1 lo, c1 hi] [c2 lo, ...] -> hi / lo planes
            const uint32_t hi =
                __builtin_amdgcn_perm(w[r][1], w[r][0], 0x07050301u) ^ 0x80808080u;
            const uint32_t lo =
                __builtin_amdgcn_perm(w[r][1], w[r][0], 0x06040200u) ^ 0x80808080u;
            *reinterpret_cast<uint32_t*>(img + i * RSB + lpos) = hi;
            *reinterpret_cast<uint32_t*>(img + (KH + i) * RSB + lpos) = lo;
        } else {
            const uint32_t hi =
                __builtin_amdgcn_perm(0u, w[r][0], 0x0c0c0301u) ^ 0x8080u;
            const uint32_t lo =
                __builtin_amdgcn_perm(0u, w[r][0], 0x0c0c0200u) ^ 0x8080u;
            *reinterpret_cast<uint16_t*>(img + i * RSB + lpos) =
                static_cast<uint16_t>(hi);
            *reinterpret_cast<uint16_t*>(img + (KH + i) * RSB + lpos) =
                static_cast<uint16_t>(lo);
        }
    }
    OorScan sc{in_oor, sid, src.by_pos, slot_base, kin, s, false};
    int n_lm = 0;
    if (scan) {  // block-uniform; the scan's barriers also publish the image
        const int cnt = scan_tile_marks(sc, col0, col1, words, s_cnt, s_i, s_col, err);
        sc.slow = cnt > kMaxTileOor;
        n_lm = min(cnt, kMaxTileOor);
    } else {
        // the routed marks into the same LDS list: the epilogue then reads
        // only LDS (no memory loads in the hot loop)
        stage_route_marks(rm, n_rm, col0, s_i, s_col);
        __syncthreads();
        n_lm = n_rm;
    }

    // matrix cores: wave wv covers nst super tiles of 64 columns, for each
    // block of 16 output rows in turn (the next block's operands prefetched)
    const bool rec = out_oor.counts != nullptr;
    const uint32_t ors = static_cast<uint32_t>(dst.rs * 2);
    // generic -> LDS address space (C-style cast: reinterpret_cast cannot
    // change the address space)
    auto* lds = (__attribute__((address_space(3))) uint8_t*)img;
    const uint32_t abase = static_cast<uint32_t>((8 * g + q) * RSB + 8 * p);
    // One row block: every super tile's MFMAs, epilogue and stores, with
    // the block's operand tiles b / kt / rs.
    auto rb_body = [&](int rb, const qi_v2i (&bop)[KS][3], const int32_t kt,
                       const int32_t rs, const int32_t (&pr)[3]) {
        const int t = 16 * rb + tl;
        const bool trow = t < L.R;
        // MFMAs of super tile ST into acc
        auto tile_mfma = [&](const int ST, qi_v4i (&acc)[4][3]) {
#pragma unroll
            for (int T = 0; T < 4; T++) {
                acc[T][0] = qi_v4i{0, 0, 0, 0};
                acc[T][1] = qi_v4i{kt, kt, kt, kt};
                acc[T][2] = qi_v4i{0, 0, 0, 0};
                auto rd_a = [&](int ks) {
                    auto* pa = (__attribute__((address_space(3))) qi_v2i*)(
                        lds + abase + 32 * ks * RSB + (4 * ST + T) * 16);
                    return __builtin_amdgcn_ds_read_tr8_b64_v2i32(pa);
                };
                if constexpr (KS == 1) {
                    const long a = __builtin_bit_cast(long, rd_a(0));
#pragma unroll
                    for (int ty = 0; ty < 3; ty++)
                        acc[T][ty] = __builtin_amdgcn_mfma_i32_16x16x32_i8(
                            a, __builtin_bit_cast(long, bop[0][ty]), acc[T][ty], 0,
                            0, 0);
                } else {
                    // two K-steps per v_mfma_i32_16x16x64_i8 (CDNA4: the
                    // cycles of 16x16x32_i8 at twice the K).  Lane l holds
                    // the 8 A bytes of steps ks and ks + 1 (and the same
                    // two B halves): A and B share their lane/byte -> K
                    // map, so the 64-K product is the sum of the two
                    // 32-K products whatever that map is
#pragma unroll
                    for (int ks = 0; ks < KS; ks += 2) {
                        const qi_v2i a0 = rd_a(ks), a1 = rd_a(ks + 1);
                        const qi_v4i a{a0.x, a0.y, a1.x, a1.y};
#pragma unroll
                        for (int ty = 0; ty < 3; ty++) {
                            // [a | 0] is zero over the l' half of K and
                            // [0 | b] over the h' half: skip the pairs
                            // that lie in a zero half (KS = 4)
                            if ((ty == 0 && ks >= KS / 2) ||
                                (ty == 1 && ks + 1 < KS / 2))
                                continue;
                            const qi_v4i b{bop[ks][ty].x, bop[ks][ty].y,
                                           bop[ks + 1][ty].x, bop[ks + 1][ty].y};
                            acc[T][ty] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                                a, b, acc[T][ty], 0, 0, 0);
                        }
                    }
                }
            }
        };
        // epilogue element math of one super tile: lane (g, t) holds row t,
        // columns 16 g .. 16 g + 15 of the super tile; result j of chunk T is
        // LDS byte 4 g + j = column 16 g + 4 T + j (straight-line VALU, so
        // it can share a scheduling region with the next tile's MFMAs)
        auto tile_y = [&](const qi_v4i (&acc)[4][3], int32_t (&y)[16]) {
#pragma unroll
            for (int T = 0; T < 4; T++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    y[4 * T + j] =
                        fold(fold(((KS >= 16 ? fold(acc[T][2][j]) : acc[T][2][j]) << 8) +
                                  acc[T][1][j] - acc[T][0][j]));
        };
        // the rest of the epilogue + stores of super tile ST
        auto tile_fin = [&](const int ST, int32_t (&y)[16]) {
            const long long cb = col0 + 64 * ST + 16 * g;
            // restored OOR symbols of the received rows: 65536 == -1 where
            // the stored word is 0 (decode_prepare, src/fec_base.h:1361-1404)
            // Branch-free per lane: the marks come from LDS and the
            // coefficient load is unconditional and consumed at once.  A gather load under a lane-divergent branch left a
            // possibly pending load into a reused VGPR at the loop exit,
            // and the compiler then drained vmcnt(0) -- every outstanding
            // store and operand prefetch -- after every super tile, with or
            // without marks (cfg3 encode: wait_any 34 % of wave cycles).
            // (One loop body, no lambda: as a lambda the compiler indexed
            // y[] dynamically and moved it to scratch memory.)
            // Only the marks inside this super tile's 64 columns are applied
            // (a wave-uniform test on the LDS list: the list holds the route
            // tile's marks, 1024 columns, so without it every super tile
            // paid 80 VALU per mark of its whole route tile).
            const uint32_t st0 = static_cast<uint32_t>(col0 + 64 * ST);
            for (int e = 0; e < n_lm; e++) {
                const uint32_t wcu = __builtin_amdgcn_readfirstlane(s_col[e]);
                if (wcu - st0 >= 64u)
                    continue;
                const int pos = __builtin_amdgcn_readfirstlane(s_i[e]);
                const long long wc = wcu;
                const long long d = wc - cb;
                // from the operand tile in registers (bop[ks][2] = [b | a])
                const int32_t corr = coef_from_tiles<KS>(
                    [&](int idx) {
                        int32_t r = 0;
#pragma unroll
                        for (int q = 0; q < 2 * KS; q++)
                            r = idx == q ? bop[q >> 1][2][q & 1] : r;
                        return r;
                    },
                    pos, l);
#pragma unroll
                for (int c = 0; c < 16; c++) {
                    const int32_t yc = fold(fold(y[c] - corr));
                    y[c] = (trow && d == c) ? yc : y[c];
                }
            }
            if (__builtin_amdgcn_ballot_w64(rs != 1)) {
                // every lane (rs = 1 keeps its value's residue: y is in
                // [-1, 65536] either way): no per-element exec masking
#pragma unroll
                for (int c = 0; c < 16; c++)
                    y[c] = fold(fold(mul_rs(y[c], rs)));
            }
            uint32_t bad = 0;
#pragma unroll
            for (int c = 0; c < 16; c++)
                bad |= static_cast<uint32_t>(y[c]);
            if (__builtin_expect(__builtin_amdgcn_ballot_w64((bad >> 16) != 0) != 0, 0)) {
#pragma unroll
                for (int c = 0; c < 16; c++) {
                    if (static_cast<uint32_t>(y[c]) > 65535u) {
                        if (rec && trow)
                            record_oor(out_oor, s, pr[0], cb + c);
                        y[c] = 0;  // 65536 (or its alias -1) is stored as 0
                    }
                }
            }
            qi_v4u o0, o1;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                o0[c] = pack_lo(static_cast<uint32_t>(y[2 * c]),
                                static_cast<uint32_t>(y[2 * c + 1]));
                o1[c] = pack_lo(static_cast<uint32_t>(y[8 + 2 * c]),
                                static_cast<uint32_t>(y[8 + 2 * c + 1]));
            }
            // the 16 x 64 output tile is transposed through LDS and stored
            // as 8 whole 128-byte lines per instruction, which can stream
            // (nt|sc1).  One block of output rows: through this super
            // tile's input bytes, dead once its MFMAs are done (row t at
            // image rows 2t, 2t+1, bytes 64 ST..); several: through the
            // wave's own staging tile behind the image (144-byte rows).
            uint8_t* stg;
            int pitch, half;
            if (RB == 1) {
                stg = img + 64 * ST;
                pitch = 2 * RSB;
                half = RSB - 64;  // bytes 64..127 of a row sit one image row down
            } else {
                stg = qi_lds + G::kLds + wv * G::kStage;
                pitch = G::kStagePitch;
                half = 0;
            }
            auto at = [&](int row, int byte) {
                return stg + row * pitch + byte + (byte >= 64 ? half : 0);
            };
            *reinterpret_cast<qi_v4u*>(at(tl, 32 * g)) = o0;
            *reinterpret_cast<qi_v4u*>(at(tl, 32 * g + 16)) = o1;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int orow = 8 * h + (l >> 3), c = l & 7;
                const qi_v4u v = *reinterpret_cast<const qi_v4u*>(at(orow, 16 * c));
                // rows >= R get an offset past the buffer resource's extent
                // (< 2^31): the hardware drops those stores.  Unconditional,
                // so the compiler keeps an exact count of the stores in flight
                const int ot = 16 * rb + orow;
                const uint32_t vo =
                    ot < L.R ? static_cast<uint32_t>(pr[1 + h]) * ors +
                                   static_cast<uint32_t>((col0 + 64 * ST + 8 * c) * 2)
                             : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b128(v, go.r, static_cast<int>(vo), 0,
                                                       kAuxStMf);
            }
            // the staging tile is rewritten by the next (ST, rb): keep this
            // iteration's reads ahead of those writes
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        };
        auto st_of = [&](int st) { return rsplit ? st : wv * nst + st; };
#pragma unroll 1
        for (int st = 0; st < nst; st++) {
            qi_v4i acc[4][3];
            int32_t y[16];
            tile_mfma(st_of(st), acc);
            tile_y(acc, y);
            tile_fin(st_of(st), y);
        }
    };
    // Row blocks in ping-pong over two operand buffers, each prefetch one row
    // block ahead and unconditional (a clamped row block past the end).  On
    // gfx9 loads and stores share the in-order vmcnt: copying a prefetched
    // buffer (or a conditional prefetch) made the compiler drain vmcnt(0) at
    // every row block -- i.e. wait for all the previous block's streaming
    // stores before the next MFMA could issue.
    if (single) {
        // one row block for this wave (every decode up to k = 64): its
        // operands were loaded before the row loads, nothing to prefetch
        if (rb0 < RB)
            rb_body(rb0, bA, ktA, rsA, prA);
    } else {
        for (int rb = rb0; rb < RB; rb += 2 * rbs) {
            load_ops(min(rb + rbs, rlast), bB, ktB, rsB, prB);
            rb_body(rb, bA, ktA, rsA, prA);
            if (rb + rbs >= RB)
                break;
            load_ops(min(rb + 2 * rbs, rlast), bA, ktA, rsA, prA);
            rb_body(rb + rbs, bB, ktB, rsB, prB);
        }
    }
    if (sc.slow) {
        // rare (block-uniform): more marks than the LDS list held; this
        // block redoes its columns once its stores are done, with the image
        // as scratch (kin x 136 bytes <= the image)
        drain_block_stores();
        redo_columns<64 * NW>(a, s, col0, col1, reinterpret_cast<uint16_t*>(qi_lds),
                              reinterpret_cast<uint32_t*>(qi_lds + kin * 2 * kRedoCols),
                              reinterpret_cast<uint32_t*>(qi_lds + kin * (2 * kRedoCols + 8)));
    }
}

// ---------------------------------------------------------------------------
// Tall-generator encode at KS = 4 (33 <= k <= 64 and at least 64 output rows:
// cfg3's 1024 x 64 generator).  matrix_mfma_kernel<4, 8, 4, true>'s geometry
// and arithmetic -- a block of 4 waves stages 512 columns of the stripe's k
// data rows as the byte-plane image, wave wv walks row blocks wv, wv + 4, ...
// over all 8 super tiles, each 16 x 64 output tile transposed through the
// wave's LDS tile into whole-line stores -- without what an encode never
// meets: no input marks (no route tables, bucket scans, per-mark epilogue
// loop or slow-tile list), no received ids, one source region.  Its OOR
// outputs (value 65536) go to an LDS list recorded at the end of the block:
// recording one in the epilogue (a returning global atomic) waited for every
// store the wave had in flight.  A row block's operands come one row block
// ahead; the super-tile loop stays plain (the pipelined pair loop measured
// no gain).  The probe ladder of tools/membw7.hip (profiles/r5_ab_notes.txt)
// puts this structure at the store shape's time.
// ---------------------------------------------------------------------------
template <int NST, int NW>
__global__ __launch_bounds__(64 * NW) void gen_mfma_kernel(MatArgs a)
{
    constexpr int KS = 4;
    using G = MfmaTile<KS, NST, NW>;
    constexpr int NCOL = G::kCols, KH = G::kRows, RSB = G::kPitch;
    constexpr int CPL = G::kCpl, RG = G::kRg;
    static_assert(G::kTpr % 64 == 0, "row groups are wave-uniform");
    extern __shared__ __attribute__((aligned(16))) uint8_t qi_lds[];
    uint8_t* img = qi_lds;
    int* s_i = reinterpret_cast<int*>(qi_lds + G::kImg);
    uint32_t* s_col = reinterpret_cast<uint32_t*>(s_i + kMaxTileOor);
    int* s_cnt = reinterpret_cast<int*>(s_col + kMaxTileOor);
    const MatLayout L = a.L;
    const Oor out_oor = a.out_oor;
    const bool rec = out_oor.counts != nullptr;

    int s, tile;
    block_map(blockIdx.x, a.tiles, s, tile);
    const int kin = L.kin;
    const long long col0 = static_cast<long long>(tile) * NCOL;
    const uint32_t cl = (RG == 1 ? threadIdx.x : threadIdx.x % G::kTpr) * CPL;
    const int rg = RG == 1 ? 0 : static_cast<int>(threadIdx.x / G::kTpr);
    const uint32_t voff = static_cast<uint32_t>((col0 + cl) * 2);
    const int32_t* M = a.mat + s * a.ms;
    const Region<true> g0(a.src.base0 + s * a.src.ss0, a.ext.e0);
    const Region<true> go(a.dst.base + s * a.dst.ss, a.ext.eo);
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int g = l >> 4, q = (l & 15) >> 1, p = l & 1, tl = l & 15;
    const int RB = L.RB();
    const int32_t* mf = M + L.mf();
    const int32_t* kmf = M + L.kmf();
    const int32_t* rscale = M + L.rscale_mf();
    const int32_t* __restrict__ rowmap = a.rowmap;

    // a row block's operands: [a|0] over the h' K-steps (b0) and [0|b] over
    // the l' K-steps (b1), as x64 pairs; [b|a] is b1 over the h' half and b0
    // over the l' half, lane for lane (see matrix_mfma_kernel's load_ops)
    struct Ops {
        qi_v4i b0, b1;
        int32_t kt, rs, pr[3];
    };
    auto load_ops = [&](int rb, Ops& o) {
        auto ld2 = [&](int ks, int ty) {
            return *reinterpret_cast<const qi_v2i*>(mf + ((rb * KS + ks) * 3 + ty) * 128 + l * 2);
        };
        const qi_v2i x0 = ld2(0, 0), x1 = ld2(1, 0), y0 = ld2(2, 1), y1 = ld2(3, 1);
        o.b0 = qi_v4i{x0.x, x0.y, x1.x, x1.y};
        o.b1 = qi_v4i{y0.x, y0.y, y1.x, y1.y};
        // unconditional loads of a clamped row, selected after (an
        // exec-masked load leaves the vmcnt count unknown to the compiler)
        const int t = 16 * rb + tl, tc = t < L.R ? t : L.R - 1;
        const int32_t k0 = kmf[tc], r0 = rscale[tc];
        o.kt = t < L.R ? k0 : 0;
        o.rs = t < L.R ? r0 : 1;
        o.pr[0] = rowmap[tc];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int ot = 16 * rb + 8 * h + (l >> 3);
            o.pr[1 + h] = rowmap[ot < L.R ? ot : L.R - 1];
        }
    };
    const int rlast = RB - 1;
    Ops oA, oB;
    load_ops(min(wv, rlast), oA);

    // stage the tile: this thread's CPL columns of every RG-th data row (rows
    // past kin: a clamped row, their operand bytes are 0), all loads first
    uint32_t w[KH / RG][CPL / 2];
    {
        const uint32_t rsb = static_cast<uint32_t>(a.src.rs0 * 2);
#pragma unroll
        for (int r = 0; r < KH / RG; r++) {
            const int i = r * RG + rg;
            ld_dw<CPL / 2, true, kAuxLd>(g0, static_cast<uint32_t>(i < kin ? i : kin - 1) * rsb,
                                         voff, w[r]);
        }
    }
    const uint32_t lpos = 64 * (cl / 64) + 16 * ((cl % 16) / 4) + 4 * ((cl % 64) / 16) + cl % 4;
#pragma unroll
    for (int r = 0; r < KH / RG; r++) {
        const int i = r * RG + rg;
        if constexpr (CPL == 4) {
            const uint32_t hi =
                __builtin_amdgcn_perm(w[r][1], w[r][0], 0x07050301u) ^ 0x80808080u;
            const uint32_t lo =
                __builtin_amdgcn_perm(w[r][1], w[r][0], 0x06040200u) ^ 0x80808080u;
            *reinterpret_cast<uint32_t*>(img + i * RSB + lpos) = hi;
            *reinterpret_cast<uint32_t*>(img + (KH + i) * RSB + lpos) = lo;
        } else {
            const uint32_t hi = __builtin_amdgcn_perm(0u, w[r][0], 0x0c0c0301u) ^ 0x8080u;
            const uint32_t lo = __builtin_amdgcn_perm(0u, w[r][0], 0x0c0c0200u) ^ 0x8080u;
            *reinterpret_cast<uint16_t*>(img + i * RSB + lpos) = static_cast<uint16_t>(hi);
            *reinterpret_cast<uint16_t*>(img + (KH + i) * RSB + lpos) = static_cast<uint16_t>(lo);
        }
    }
    if (threadIdx.x == 0)
        *s_cnt = 0;
    __syncthreads();

    const uint32_t ors = static_cast<uint32_t>(a.dst.rs * 2);
    auto* lds = (__attribute__((address_space(3))) uint8_t*)img;
    const uint32_t abase = static_cast<uint32_t>((8 * g + q) * RSB + 8 * p);
    uint8_t* stg = qi_lds + G::kLds + wv * G::kStage;

    auto rb_body = [&](int rb, const Ops& o) {
        const int t = 16 * rb + tl;
        const bool trow = t < L.R;
        const qi_v4i ktv{o.kt, o.kt, o.kt, o.kt};
#pragma unroll 1
        for (int st = 0; st < NST; st++) {
            qi_v4i acc[4][3];
#pragma unroll
            for (int T = 0; T < 4; T++) {
                auto rd = [&](int ks) {
                    auto* pa = (__attribute__((address_space(3))) qi_v2i*)(
                        lds + abase + 32 * ks * RSB + (4 * st + T) * 16);
                    return __builtin_amdgcn_ds_read_tr8_b64_v2i32(pa);
                };
                const qi_v2i h0 = rd(0), h1 = rd(1), l0 = rd(2), l1 = rd(3);
                const qi_v4i ah{h0.x, h0.y, h1.x, h1.y}, al{l0.x, l0.y, l1.x, l1.y};
                acc[T][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, o.b0, qi_v4i{0, 0, 0, 0},
                                                                  0, 0, 0);
                acc[T][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, o.b1, ktv, 0, 0, 0);
                acc[T][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, o.b1, qi_v4i{0, 0, 0, 0},
                                                                  0, 0, 0);
                acc[T][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, o.b0, acc[T][2], 0, 0, 0);
            }
            // lane (g, t) holds row t, columns cb .. cb + 15 (the image's
            // column order): y = 256 D2 + D1 - D0, kt in D1
            const long long cb = col0 + 64 * st + 16 * g;
            int32_t y[16];
#pragma unroll
            for (int T = 0; T < 4; T++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    y[4 * T + j] = fold(fold((acc[T][2][j] << 8) + acc[T][1][j] - acc[T][0][j]));
            if (__builtin_amdgcn_ballot_w64(o.rs != 1)) {
#pragma unroll
                for (int c = 0; c < 16; c++)
                    y[c] = fold(fold(mul_rs(y[c], o.rs)));
            }
            uint32_t bad = 0;
#pragma unroll
            for (int c = 0; c < 16; c++)
                bad |= static_cast<uint32_t>(y[c]);
            if (__builtin_expect(__builtin_amdgcn_ballot_w64((bad >> 16) != 0) != 0, 0)) {
#pragma unroll
                for (int c = 0; c < 16; c++) {
                    if (static_cast<uint32_t>(y[c]) > 65535u) {
                        if (rec && trow) {
                            // LDS atomic: no wait on the stores in flight
                            const int e = atomicAdd(s_cnt, 1);
                            if (e < kMaxTileOor) {
                                s_i[e] = o.pr[0];
                                s_col[e] = static_cast<uint32_t>(cb + c);
                            } else {
                                record_oor(out_oor, s, o.pr[0], cb + c);
                            }
                        }
                        y[c] = 0;  // 65536 (or its alias -1) is stored as 0
                    }
                }
            }
            qi_v4u o0, o1;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                o0[c] = pack_lo(static_cast<uint32_t>(y[2 * c]), static_cast<uint32_t>(y[2 * c + 1]));
                o1[c] = pack_lo(static_cast<uint32_t>(y[8 + 2 * c]),
                                static_cast<uint32_t>(y[8 + 2 * c + 1]));
            }
            *reinterpret_cast<qi_v4u*>(stg + tl * G::kStagePitch + 32 * g) = o0;
            *reinterpret_cast<qi_v4u*>(stg + tl * G::kStagePitch + 32 * g + 16) = o1;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int orow = 8 * h + (l >> 3), c = l & 7;
                const qi_v4u v =
                    *reinterpret_cast<const qi_v4u*>(stg + orow * G::kStagePitch + 16 * c);
                // rows >= R: an offset past the extent (< 2^31), dropped
                const int ot = 16 * rb + orow;
                const uint32_t vo =
                    ot < L.R ? static_cast<uint32_t>(o.pr[1 + h]) * ors +
                                   static_cast<uint32_t>((col0 + 64 * st + 8 * c) * 2)
                             : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b128(v, go.r, static_cast<int>(vo), 0, kAuxStMf);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
    };
    // row blocks in ping-pong over two operand sets, each prefetched one row
    // block ahead and unconditional (a clamped row block past the end)
    for (int rb = wv; rb < RB; rb += 2 * NW) {
        load_ops(min(rb + NW, rlast), oB);
        rb_body(rb, oA);
        if (rb + NW >= RB)
            break;
        load_ops(min(rb + 2 * NW, rlast), oA);
        rb_body(rb + NW, oB);
    }
    // the block's OOR outputs into their buckets
    __syncthreads();
    const int n = min(*s_cnt, kMaxTileOor);
    for (int e = threadIdx.x; e < n; e += 64 * NW)
        record_oor(out_oor, s, s_i[e], s_col[e]);
}

// ---------------------------------------------------------------------------
// Operand-stationary matrix-core kernel (KS = 4, 8, 16: 32 < kin <= 256; the
// decodes of k = 33 .. 256 and the generators of those codes).
//
// matrix_mfma_kernel stages one column block, computes it and exits: every
// block re-fetches the operand tiles of every row block it covers from L2
// (16 KB of non-zero i8 tiles per 16 output rows at KS = 16, ~8x the HBM
// data stream at k = 200), and its load and compute phases run one after
// the other (two blocks per CU in lock step).  Here a block of 8 waves
// stays on one stripe for a range of column tiles:
//   - wave w owns RPW row blocks (slot w % WR) for the block's whole life:
//     their operand tiles stay in registers (KS / 2 + KS / 2 v4i each: 64
//     VGPRs at KS = 16), with kmf / rscale / rowmap;
//   - a tile is 64 NSTT columns, NSTT = 8 / WR super tiles of 64 columns
//     (wave w takes super tile w / WR), staged as the byte-plane image of
//     matrix_mfma_kernel in one of two LDS buffers: the next tile's rows are
//     loaded into registers while this one is on the matrix cores;
//   - a matrix with more than WR RPW row blocks runs G blocks per column
//     range (group gq takes rb = gq WR RPW + slot + WR j); they read the same
//     input tiles, and the XCD-aware map puts them on one XCD (shared L2).
// The arithmetic, operand tiles, epilogue and OOR handling are
// matrix_mfma_kernel's (byte split, 2^16 = -1, D2 folded first at KS = 16).
// ---------------------------------------------------------------------------
// Coefficient M[t][pos] of this lane's output row t (lane (g, t & 15) of a
// 16-row block) from the block's [b | a] operand tile held in registers:
// pick(2 ks + dw) returns this lane's dword dw of K-step ks (lane 16 g + t:
// bytes K = 32 ks + 8 g + 4 dw + 0..3; b at K = pos, a at K = 16 KS + pos,
// pack_mf_dword's layout).  Returns the row-scaled entry as 256 a + b
// (balanced), the value of mf_entry / the `plain` section; pos is
// wave-uniform, and each byte comes from the lane holding it by ds_bpermute
// -- no memory load (waiting for one drains the stores and prefetches).
template <int KS, class Pick>
__device__ __forceinline__ int32_t coef_from_tiles(const Pick& pick, int pos, int lane)
{
    constexpr int KH = 16 * KS;
    auto byte_at = [&](int K) {
        const int ks = K >> 5, g = (K & 31) >> 3, dw = (K >> 2) & 1, sh = 8 * (K & 3);
        const int32_t x = __shfl(pick(2 * ks + dw), 16 * g + (lane & 15));
        return (x << (24 - sh)) >> 24;
    };
    return 256 * byte_at(KH + pos) + byte_at(pos);
}

// uniform-index selection among a wave's operand dwords (a v_cndmask chain)
template <int NP>
__device__ __forceinline__ int32_t pick_v4(const qi_v4i (&v)[NP], int idx)
{
    int32_t r = 0;
#pragma unroll
    for (int i = 0; i < NP; i++)
#pragma unroll
        for (int e = 0; e < 4; e++)
            r = idx == 4 * i + e ? v[i][e] : r;
    return r;
}

// K chunks of the operand-stationary kernel: KS = 40 (384 < k <= 640) stages
// its image in two chunks of 20 K-steps (the received rows [0, 320) and
// [320, 640)), double-buffered over (tile, chunk) items, the accumulators
// held across the chunks of a tile: a whole KS = 40 image (2 x 640 rows of
// 80 bytes, 102 KB) could not be double-buffered in LDS
template <int KS>
struct OsK {
    static constexpr int NCH = KS > 24 ? 2 : 1;  // K chunks per tile
    static constexpr int KC = KS / NCH;          // K-steps per chunk
};

template <int KS, int WR>
struct OsTile {
    static constexpr int kWaves = 8;
    static constexpr int kThreads = 64 * kWaves;
    static constexpr int kNst = kWaves / WR;   // super tiles per tile
    static constexpr int kCols = 64 * kNst;    // columns per tile
    static constexpr int kRows = 16 * KS;      // rows per byte plane (KH)
    static constexpr int kPitch = kCols + 16;  // LDS row pitch: +4 banks/row
    static constexpr size_t kImg = static_cast<size_t>(2 * kRows) * kPitch;
    static constexpr int kStagePitch = 144;
    static constexpr size_t kStage = 16 * kStagePitch;
    static constexpr size_t kStageOff = 2 * kImg;
    static constexpr size_t kMarkOff = kStageOff + kWaves * kStage;
    // two mark lists (s_i, s_col) + two counts
    static constexpr size_t kLds = kMarkOff + 2 * 2 * 4 * kMaxTileOor + 16;
    // staging: 4 columns (b64) per lane, kTpr lanes per image row
    static constexpr int kTpr = kCols / 4;
    static constexpr int kRpp = kThreads / kTpr;  // rows per pass
    static constexpr int kRpt = kRows / kRpp;     // rows per thread
    static_assert(kRpt >= 1 && kRows % kRpp == 0, "staging");
};

template <int KS, int WR, int RPW, bool TWO>
__global__ __launch_bounds__(512) void matrix_os_kernel(MatArgs a, int G, int C, int TS)
{
    constexpr int NCH = OsK<KS>::NCH, KC = OsK<KS>::KC;
    using O = OsTile<KC, WR>;  // one chunk's image (the whole K when NCH = 1)
    constexpr int KH = O::kRows, RSB = O::kPitch, RPT = O::kRpt, NCOL = O::kCols;
    static_assert(KS % 4 == 0 && KC % 4 == 0, "x64 pairs with zero halves");
    static_assert(NCH == 1 || RPW == 1, "K chunks: one row block per wave");
    extern __shared__ __attribute__((aligned(16))) uint8_t qi_lds[];
    const MatLayout L = a.L;
    const RowSrc src = a.src;
    const RowDst dst = a.dst;
    const MatExt ext = a.ext;
    const Oor in_oor = a.in_oor;
    const Oor out_oor = a.out_oor;
    const int kin = L.kin;
    const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
    const int g = l >> 4, q = (l & 15) >> 1, p = l & 1, tl = l & 15;

    // block -> (stripe, row-block group, column range); every block of one
    // stripe on the same XCD (block b runs on XCD b % 8), consecutive in its
    // dispatch order, when the stripes tile the 8 XCDs: the stripe's context
    // tiles (256 KB per stripe at k = 256, 4 KiB packets: a quarter of its
    // data bytes) and the input tiles its G groups share are read from HBM
    // once and hit that XCD's L2 after (round 6: the C column ranges had
    // landed on different XCDs, k256 decode reads 1.23x algorithmic);
    // otherwise the G groups of one (stripe, range) on one XCD
    int s, gq, cr;
    {
        const int L0 = blockIdx.x;
        int unit;
        const int S = static_cast<int>(gridDim.x) / (G * C);
        if ((S & 7) == 0) {
            const int x = L0 & 7, j = L0 >> 3, per = G * C;
            const int sg = j / per, rem = j - sg * per;
            s = sg * 8 + x;
            cr = rem / G;
            gq = rem - cr * G;
            unit = s * C + cr;
        } else if (((S * C) & 7) == 0) {
            const int x = L0 & 7, j = L0 >> 3;
            gq = j % G;
            unit = (j / G) * 8 + x;
        } else {
            gq = L0 % G;
            unit = L0 / G;
        }
        s = unit / C;
        cr = unit - s * C;
    }
    const int t0 = static_cast<int>(static_cast<long long>(cr) * TS / C);
    const int t1 = static_cast<int>(static_cast<long long>(cr + 1) * TS / C);
    // one bit per tile of the block (<= kOsMaxTiles, os_launch), behind the
    // other LDS sections; cleared before the first mark scan's barrier
    uint32_t* slow_bits = reinterpret_cast<uint32_t*>(qi_lds + O::kLds);
    for (int wd = tid; wd <= (t1 - t0 - 1) >> 5; wd += 512)
        slow_bits[wd] = 0u;

    const int RB = L.RB();
    const int slot = wv % WR, st = wv / WR;  // row-block slot, super tile
    const int32_t* M = a.mat + s * a.ms;
    const int32_t* mf = M + L.mf();
    const int32_t* kmf = M + L.kmf();
    const int32_t* rscale = M + L.rscale_mf();
    const int32_t* __restrict__ rowmap = a.rowmap;
    const int32_t* sid = a.ids ? a.ids + s * a.is : nullptr;

    // this wave's row blocks and their operand tiles, for the block's whole
    // life: [a|0] over the h' K-steps, [0|b] over the l' K-steps (x64
    // pairs); [b|a] over the h' half is b1 and over the l' half b0, lane for
    // lane (see matrix_mfma_kernel's load_ops), so it is neither stored in
    // the context nor held twice
    int rbj[RPW];
    bool act[RPW];
    qi_v4i b0[RPW][KS / 4], b1[RPW][KS / 4];
    int32_t kt[RPW], rs[RPW], pr[RPW][3];
#pragma unroll
    for (int j = 0; j < RPW; j++) {
        // row blocks dealt round-robin over the G groups (their counts
        // differ by at most one): a group with fewer busy waves ran ahead of
        // the others, and the input tiles it had fetched were evicted from
        // L2 before they came by (k300: 1.88x the input bytes read)
        const int rb = gq + G * (slot + WR * j);
        act[j] = rb < RB;  // wave-uniform
        const int rbc = act[j] ? rb : RB - 1;
        rbj[j] = rbc;
        auto ld2 = [&](int ks, int ty) {
            return *reinterpret_cast<const qi_v2i*>(mf + ((rbc * KS + ks) * 3 + ty) * 128 + l * 2);
        };
#pragma unroll
        for (int i = 0; i < KS / 4; i++) {
            const qi_v2i x0 = ld2(2 * i, 0), x1 = ld2(2 * i + 1, 0);
            b0[j][i] = qi_v4i{x0.x, x0.y, x1.x, x1.y};
            const qi_v2i y0 = ld2(KS / 2 + 2 * i, 1), y1 = ld2(KS / 2 + 2 * i + 1, 1);
            b1[j][i] = qi_v4i{y0.x, y0.y, y1.x, y1.y};
        }
        const int t = 16 * rbc + tl;
        const int tcl = t < L.R ? t : L.R - 1;
        const int32_t k0 = kmf[tcl], r0 = rscale[tcl];
        kt[j] = t < L.R ? k0 : 0;
        rs[j] = t < L.R ? r0 : 1;
        pr[j][0] = rowmap[tcl];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int ot = 16 * rbc + 8 * h + (l >> 3);
            pr[j][1 + h] = rowmap[ot < L.R ? ot : L.R - 1];
        }
    }

    // staging: lane (rowgrp, cl) loads 4 columns (b64) of rows kRpp r +
    // rowgrp; per-lane row offsets fixed for the block (rows past kin
    // clamped: their operand bytes are 0); chunk c stages the received rows
    // KH c .. KH c + KH - 1.
    //   TWO (two source regions, the systematic decodes): one offset per
    // row, in its own region.  The context lists the received rows region by
    // region (order_ids, ctx.hip), so a wave's load of pass (c, r) reads one
    // region, through that region's descriptor (bit c RPT + r of sel), but
    // for at most one pass (xcr) that straddles the boundary: its region-1
    // lanes take an extra load (wx, one per item, past the extent in every
    // other item: zeros), ORed into that row when it is written to LDS.
    // (Each row loaded through both descriptors, past the extent in the
    // other region, took the k600 systematic decode 1.11 -> 1.92 ms:
    // twice the load instructions, gpurun_out/r6l.)
    const Region<true> g0(src.base0 + s * src.ss0, ext.e0);
    const Region<true> g1(src.base1 ? src.base1 + s * src.ss1 : src.base0, ext.e1);
    const Region<true> go(dst.base + s * dst.ss, ext.eo);
    const int rowgrp = tid / O::kTpr, cl = (tid % O::kTpr) * 4;
    constexpr uint32_t kOob = 0x80000000u;  // past any extent (< 2^31)
    static_assert(NCH * RPT <= 32, "pass bits");
    uint32_t off0[NCH][RPT];
    uint32_t sel = 0, offx = kOob;  // sel: wave-uniform
    int xcr = -1;                   // wave-uniform: c RPT + r of the straddling pass
#pragma unroll
    for (int c = 0; c < NCH; c++)
#pragma unroll
        for (int r = 0; r < RPT; r++) {
            const int i = KH * c + O::kRpp * r + rowgrp;
            const int ii = i < kin ? i : kin - 1;
            const int id = src.by_pos ? ii : (sid ? sid[ii] : ii);
            const uint32_t lane = static_cast<uint32_t>(cl * 2);
            if constexpr (TWO) {
                const bool lo = id < src.split;
                off0[c][r] = (lo ? static_cast<uint32_t>(id * src.rs0 * 2)
                                 : static_cast<uint32_t>((id - src.split) * src.rs1 * 2)) +
                             lane;
                const uint64_t b1 = __ballot(!lo);
                if (b1 == ~0ull) {
                    sel |= 1u << (c * RPT + r);
                } else if (b1 != 0ull) {
                    if (xcr >= 0 && a.err && l == 0)
                        atomicOr(a.err, kErrBadIds);  // rows not in region order
                    xcr = c * RPT + r;
                    offx = lo ? kOob : off0[c][r];
                }
            } else {
                off0[c][r] = static_cast<uint32_t>(id * src.rs0 * 2) + lane;
            }
        }
    sel = __builtin_amdgcn_readfirstlane(sel);
    xcr = __builtin_amdgcn_readfirstlane(xcr);
    const int xc = xcr >= 0 ? xcr / RPT : -1, xr = xcr >= 0 ? xcr % RPT : -1;
    // DEEP (KS = 4, the short decodes): ND tiles of rows in flight per
    // block (a ring of ND register sets, 8 VGPRs each) -- with one, a CU
    // kept ~32 KB of loads in flight and the cfg3 decode was bound by the
    // load latency; three measured the same as two, four slower (125 / 133
    // VGPRs: cfg3 decode 0.143 / 0.168 ms, profiles/r5_ab_notes.txt)
    constexpr int ND = KS == 4 ? 2 : 1;
    constexpr bool DEEP = ND >= 2;
    uint32_t w[RPT][2], wring[DEEP ? ND : 1][DEEP ? RPT : 1][2];
    uint32_t wx[2], wxring[DEEP ? ND : 1][2];  // TWO: the straddling pass's region-1 lanes
    // rows of `tile` into wr; an invalid tile (past the block's range) loads
    // from past the buffer's extent (no memory access, zeros), so the number
    // of loads in flight is the same on every path
    auto issue_rows_to = [&](int tile, bool valid, auto& wr, auto& wxr, auto cc) {
        constexpr int c = decltype(cc)::value;  // K chunk
        const int so = valid ? tile * NCOL * 2 : 0;  // byte offset of the tile's first column
        const uint32_t oob = valid ? 0u : kOob;
#pragma unroll
        for (int r = 0; r < RPT; r++) {
            uint32_t o = off0[c][r] | oob;
            auto rsrc = g0.r;
            if constexpr (TWO) {
                // (the straddling pass: its region-1 lanes through wx)
                o = c * RPT + r == xcr && offx != kOob ? kOob : o;
                rsrc = (sel >> (c * RPT + r)) & 1u ? g1.r : g0.r;
            }
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, static_cast<int>(o), so,
                                                                kAuxLdOs);
            wr[r][0] = v[0];
            wr[r][1] = v[1];
        }
        if constexpr (TWO) {
            const auto u = __builtin_amdgcn_raw_buffer_load_b64(
                g1.r, static_cast<int>(c == xc ? offx | oob : kOob), so, kAuxLdOs);
            wxr[0] = u[0];
            wxr[1] = u[1];
        }
    };
    using C0 = std::integral_constant<int, 0>;
    auto issue_rows = [&](int tile, auto cc) { issue_rows_to(tile, true, w, wx, cc); };
    const uint32_t lpos = 64 * (cl / 64) + 16 * ((cl % 16) / 4) + 4 * ((cl % 64) / 16);
    auto write_rows_from = [&](uint8_t* img, const auto& w, const auto& wxr) {
#pragma unroll
        for (int r = 0; r < RPT; r++) {
            const int i = O::kRpp * r + rowgrp;
            uint32_t w0 = w[r][0], w1 = w[r][1];
            if constexpr (TWO) {
                // (zeros unless this item's chunk holds the straddling pass)
                w0 |= r == xr ? wxr[0] : 0u;
                w1 |= r == xr ? wxr[1] : 0u;
            }
            const uint32_t hi = __builtin_amdgcn_perm(w1, w0, 0x07050301u) ^ 0x80808080u;
            const uint32_t lo = __builtin_amdgcn_perm(w1, w0, 0x06040200u) ^ 0x80808080u;
            *reinterpret_cast<uint32_t*>(img + i * RSB + lpos) = hi;
            *reinterpret_cast<uint32_t*>(img + (KH + i) * RSB + lpos) = lo;
        }
    };
    auto write_rows = [&](uint8_t* img) { write_rows_from(img, w, wx); };

    // OOR marks of the received rows in a tile (route table or bucket
    // scan) into mark list mb; returns the count (all threads)
    auto s_i = [&](int mb) {
        return reinterpret_cast<int*>(qi_lds + O::kMarkOff) + mb * 2 * kMaxTileOor;
    };
    auto s_col = [&](int mb) { return reinterpret_cast<uint32_t*>(s_i(mb) + kMaxTileOor); };
    auto s_cnt = [&](int mb) {
        return reinterpret_cast<int*>(qi_lds + O::kMarkOff + 2 * 2 * 4 * kMaxTileOor) + mb;
    };
    const bool marks_in = in_oor.counts != nullptr;
    // the route-table list each mark buffer holds (block-uniform): the tiles
    // of one kRouteTile-column route tile share its list (the epilogue keeps
    // the marks in its own columns), so a buffer that already holds it is not
    // staged again.  (Staging it every tile cost the cfg3 decode ~8 us: the
    // wait for the scalar load also drained the LDS accesses in flight,
    // tools/ab/probe_os_nomarks.patch)
    // (not at KS = 8, whose kernel measured faster staging every tile from
    // scalar loads: k128 decode 1.5 %)
    constexpr bool kOnce = KS != 8;
    int srt0 = -1, srt1 = -1, scnt0 = 0, scnt1 = 0;
    auto stage_marks = [&](int tile, int mb) -> int {
        if (!marks_in)
            return 0;
        const long long col0 = static_cast<long long>(tile) * NCOL;
        if (a.route) {
            const int rti = static_cast<int>(col0 / kRouteTile);
            if (kOnce && (mb ? srt1 : srt0) == rti)
                return mb ? scnt1 : scnt0;
            const int rc = stage_route_marks_s<kOnce>(
                a.route + s * a.rstride + static_cast<long long>(rti) * kRouteStride, col0,
                s_i(mb), s_col(mb));
            if (rc >= 0) {
                if constexpr (kOnce) {
                    if (mb) {
                        srt1 = rti;
                        scnt1 = rc;
                    } else {
                        srt0 = rti;
                        scnt0 = rc;
                    }
                }
                return rc;
            }
        }
        if constexpr (kOnce) {
            if (mb)  // this buffer now holds a bucket scan of one tile
                srt1 = -1;
            else
                srt0 = -1;
        }
        OorScan sc{in_oor, sid, src.by_pos, a.slot_base, kin, s, false};
        const int cnt = scan_tile_marks(sc, col0, col0 + NCOL, a.words, s_cnt(mb), s_i(mb),
                                        s_col(mb), a.err);
        if (cnt > kMaxTileOor && tid == 0)  // rare: redone at the block's end
            atomicOr(&slow_bits[(tile - t0) >> 5], 1u << ((tile - t0) & 31));
        return min(cnt, kMaxTileOor);
    };
    // the block's slow tiles (bits over [t0, t1)), redone by the block once
    // its stores are done, with the images as scratch
    auto finish = [&]() {
        if (!marks_in)
            return;
        bool any = false;
        for (int wd = 0; wd <= (t1 - t0 - 1) >> 5; wd++)
            any |= slow_bits[wd] != 0u;
        if (!any)
            return;  // block-uniform
        drain_block_stores();
        for (int wd = 0; wd <= (t1 - t0 - 1) >> 5; wd++) {
            uint32_t bits = slow_bits[wd];
            while (bits) {
                const int tile = t0 + 32 * wd + __builtin_ctz(bits);
                bits &= bits - 1;
                const long long c0 = static_cast<long long>(tile) * NCOL;
                // this group's row blocks only: the G blocks of a column
                // range each redo (and earlier stored) disjoint rows
                redo_columns<512>(a, s, c0, c0 + NCOL, reinterpret_cast<uint16_t*>(qi_lds),
                                  reinterpret_cast<uint32_t*>(qi_lds + kin * 2 * kRedoCols),
                                  reinterpret_cast<uint32_t*>(qi_lds + kin * (2 * kRedoCols + 8)),
                                  gq, G);
            }
        }
    };

    const bool rec = out_oor.counts != nullptr;
    const uint32_t ors = static_cast<uint32_t>(dst.rs * 2);
    const uint32_t abase = static_cast<uint32_t>((8 * g + q) * RSB + 8 * p + 64 * st);
    uint8_t* stg = qi_lds + O::kStageOff + wv * O::kStage;

    // row block j of this wave over its super tile (columns col0 ..
    // col0 + 63) from image img
    // row block j's accumulators: D0 = 0, D1 = kmf (the byte offsets'
    // correction), D2 = 0
    auto init_acc = [&](qi_v4i (&acc)[4][3], auto jc) {
        constexpr int j = decltype(jc)::value;
#pragma unroll
        for (int T = 0; T < 4; T++) {
            acc[T][0] = qi_v4i{0, 0, 0, 0};
            acc[T][1] = qi_v4i{kt[j], kt[j], kt[j], kt[j]};
            acc[T][2] = qi_v4i{0, 0, 0, 0};
        }
    };
    // K chunk cc of row block j over this wave's super tile of image img,
    // accumulated into acc: the chunk's h' half of K (its pairs: [a|0] and
    // [b|a]), then its l' half ([0|b] and [b|a]), KC / 4 A pairs live at a
    // time; operand pair c KC / 4 + i of the row block's registers
    auto mma = [&](const uint8_t* img, qi_v4i (&acc)[4][3], auto jc, auto cc) {
        constexpr int j = decltype(jc)::value, c = decltype(cc)::value;
        auto* lds = (__attribute__((address_space(3))) const uint8_t*)img;
#pragma unroll
        for (int T = 0; T < 4; T++) {
#pragma unroll
            for (int hf = 0; hf < 2; hf++) {
                qi_v4i av[KC / 4];
#pragma unroll
                for (int i = 0; i < KC / 4; i++) {
                    auto rd = [&](int ks) {
                        auto* pa = (__attribute__((address_space(3))) qi_v2i*)(
                            lds + abase + 32 * ks * RSB + T * 16);
                        return __builtin_amdgcn_ds_read_tr8_b64_v2i32(pa);
                    };
                    const int pi = hf * (KC / 4) + i;
                    const qi_v2i x0 = rd(2 * pi), x1 = rd(2 * pi + 1);
                    av[i] = qi_v4i{x0.x, x0.y, x1.x, x1.y};
                }
#pragma unroll
                for (int i = 0; i < KC / 4; i++) {
                    constexpr int o = c * (KC / 4);
                    if (hf == 0)
                        acc[T][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[i], b0[j][o + i],
                                                                          acc[T][0], 0, 0, 0);
                    else
                        acc[T][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av[i], b1[j][o + i],
                                                                          acc[T][1], 0, 0, 0);
                    acc[T][2] = __builtin_amdgcn_mfma_i32_16x16x64_i8(
                        av[i], hf == 0 ? b1[j][o + i] : b0[j][o + i], acc[T][2], 0, 0, 0);
                }
            }
        }
    };
    auto epilogue = [&](const qi_v4i (&acc)[4][3], long long col0, int n_lm, const int* mi,
                        const uint32_t* mc, auto jc, auto&& before_stores) {
        constexpr int j = decltype(jc)::value;
        const int t = 16 * rbj[j] + tl;
        const bool trow = act[j] && t < L.R;
        // epilogue: lane (g, t) holds row t, columns cb .. cb + 15
        const long long cb = col0 + 16 * g;
        int32_t y[16];
#pragma unroll
        for (int T = 0; T < 4; T++)
#pragma unroll
            for (int jj = 0; jj < 4; jj++)
                y[4 * T + jj] =
                    fold(fold(((KS >= 16 ? fold(acc[T][2][jj]) : acc[T][2][jj]) << 8) +
                              acc[T][1][jj] - acc[T][0][jj]));
        // restored OOR symbols of the received rows (decode_prepare,
        // src/fec_base.h:1361-1404): 65536 == -1 where the stored word is 0
        const uint32_t st0 = static_cast<uint32_t>(col0);
        for (int e = 0; e < n_lm; e++) {
            const uint32_t wcu = __builtin_amdgcn_readfirstlane(mc[e]);
            if (wcu - st0 >= 64u)
                continue;
            const int pos = __builtin_amdgcn_readfirstlane(mi[e]);
            const long long d = static_cast<long long>(wcu) - cb;
            // the coefficient from the wave's own operand tiles (no memory
            // load: waiting for one drained the stores and the prefetch)
            const int32_t corr = coef_from_tiles<KS>(
                [&](int idx) {
                    // [b | a]'s dword idx: b1 over the h' pairs, b0 over the l'
                    return idx < KS ? pick_v4(b1[j], idx) : pick_v4(b0[j], idx - KS);
                },
                pos, l);
#pragma unroll
            for (int c = 0; c < 16; c++) {
                const int32_t yc = fold(fold(y[c] - corr));
                y[c] = (trow && d == c) ? yc : y[c];
            }
        }
        if (__builtin_amdgcn_ballot_w64(rs[j] != 1)) {
#pragma unroll
            for (int c = 0; c < 16; c++)
                y[c] = fold(fold(mul_rs(y[c], rs[j])));
        }
        uint32_t bad = 0;
#pragma unroll
        for (int c = 0; c < 16; c++)
            bad |= static_cast<uint32_t>(y[c]);
        if (__builtin_expect(__builtin_amdgcn_ballot_w64((bad >> 16) != 0) != 0, 0)) {
#pragma unroll
            for (int c = 0; c < 16; c++) {
                if (static_cast<uint32_t>(y[c]) > 65535u) {
                    if (rec && trow)
                        record_oor(out_oor, s, pr[j][0], cb + c);
                    y[c] = 0;  // 65536 (or its alias -1) is stored as 0
                }
            }
        }
        qi_v4u o0, o1;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            o0[c] = pack_lo(static_cast<uint32_t>(y[2 * c]), static_cast<uint32_t>(y[2 * c + 1]));
            o1[c] = pack_lo(static_cast<uint32_t>(y[8 + 2 * c]),
                            static_cast<uint32_t>(y[8 + 2 * c + 1]));
        }
        // transposed through the wave's staging tile into whole-line stores
        *reinterpret_cast<qi_v4u*>(stg + tl * O::kStagePitch + 32 * g) = o0;
        *reinterpret_cast<qi_v4u*>(stg + tl * O::kStagePitch + 32 * g + 16) = o1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        qi_v4u v2[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int orow = 8 * h + (l >> 3), c = l & 7;
            v2[h] = *reinterpret_cast<const qi_v4u*>(stg + orow * O::kStagePitch + 16 * c);
        }
        if constexpr (j == RPW - 1)
            before_stores();
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int orow = 8 * h + (l >> 3), c = l & 7;
            const qi_v4u v = v2[h];
            const int ot = 16 * rbj[j] + orow;
            const uint32_t vo = (act[j] && ot < L.R)
                                    ? static_cast<uint32_t>(pr[j][1 + h]) * ors +
                                          static_cast<uint32_t>((col0 + 8 * c) * 2)
                                    : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b128(v, go.r, static_cast<int>(vo), 0, kAuxStMf);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    };
    // the whole K in one image (NCH = 1)
    auto compute = [&](const uint8_t* img, long long col0, int n_lm, const int* mi,
                       const uint32_t* mc, auto jc, auto&& before_stores) {
        qi_v4i acc[4][3];
        init_acc(acc, jc);
        mma(img, acc, jc, C0{});
        epilogue(acc, col0, n_lm, mi, mc, jc, before_stores);
    };

    auto idle_stores = [&]() {
#pragma unroll
        for (int h = 0; h < 2; h++)
            __builtin_amdgcn_raw_buffer_store_b128(qi_v4u{0u, 0u, 0u, 0u}, go.r,
                                                   static_cast<int>(0x80000000u + 16 * h), 0,
                                                   kAuxStMf);
    };

    if (t0 >= t1)
        return;
    auto img = [&](int b) { return qi_lds + b * O::kImg; };
    if constexpr (DEEP) {
        // tiles t0 .. t0 + ND - 1 in flight, the first one into image 0
#pragma unroll
        for (int d = 0; d < ND; d++)
            issue_rows_to(t0 + d, t0 + d < t1, wring[d], wxring[d], C0{});
        write_rows_from(img(0), wring[0], wxring[0]);
        int nl[2];
        nl[0] = stage_marks(t0, 0);
        nl[1] = 0;
        __syncthreads();
        // tile's rows are in image b; set J (tile's, already written) takes
        // tile + ND's, set J + 1 holds tile + 1's (in flight)
        auto body = [&](int tile, auto jc) {
            constexpr int J = decltype(jc)::value;
            const int b = (tile - t0) & 1;
            const bool more = tile + 1 < t1;  // block-uniform
            issue_rows_to(tile + ND, tile + ND < t1, wring[J], wxring[J], C0{});
            const long long col0 = static_cast<long long>(tile) * NCOL + 64 * st;
            auto none = [] {};
            [&]<int... R>(std::integer_sequence<int, R...>) {
                ((act[R] ? compute(img(b), col0, nl[b], s_i(b), s_col(b),
                                   std::integral_constant<int, R>{}, none)
                         : idle_stores()),
                 ...);
            }(std::make_integer_sequence<int, RPW>{});
            // unconditional, so every path waits for the next set's loads
            // here (a skipped write left them pending on one path, and the
            // compiler then drained vmcnt(0) before reusing the registers);
            // past the last tile it writes the invalid tile's zeros into an
            // image no wave reads again
            write_rows_from(img(b ^ 1), wring[(J + 1) % ND], wxring[(J + 1) % ND]);
            if (more)
                nl[b ^ 1] = stage_marks(tile + 1, b ^ 1);
            __syncthreads();
        };
#pragma unroll 1
        for (int tile = t0; tile < t1; tile += ND) {
            bool done = false;
            [&]<int... J>(std::integer_sequence<int, J...>) {
                ((done = done || tile + J >= t1, done ? void() : body(tile + J,
                                                                     std::integral_constant<int, J>{})),
                 ...);
            }(std::make_integer_sequence<int, ND>{});
            if (done)
                break;
        }
        finish();
        return;
    }
    issue_rows(t0, C0{});
    write_rows(img(0));
    int nl[2];
    nl[0] = stage_marks(t0, 0);
    nl[1] = 0;
    __syncthreads();
    if constexpr (NCH > 1) {
        // (tile, chunk) items, double-buffered: item q's rows in image q & 1
        // while item q + 1's are in flight; a tile's accumulators live over
        // its chunks, its epilogue (marks, stores) after the last one
        static_assert(NCH == 2, "two K chunks");
        constexpr bool rows_first = true;
        int ib = 0;
#pragma unroll 1
        for (int tile = t0; tile < t1; tile++) {
            const int mb = (tile - t0) & 1;
            const bool more = tile + 1 < t1;  // block-uniform
            const long long col0 = static_cast<long long>(tile) * NCOL + 64 * st;
            qi_v4i acc[4][3];
            using J0 = std::integral_constant<int, 0>;
            // chunk 0; chunk 1's rows in flight, staged right after
            issue_rows(tile, std::integral_constant<int, 1>{});
            init_acc(acc, J0{});
            if (act[0])
                mma(img(ib), acc, J0{}, C0{});
            write_rows(img(ib ^ 1));
            __syncthreads();
            ib ^= 1;
            // chunk 1, then the epilogue; the next tile's chunk 0 in flight
            if (more)
                issue_rows(tile + 1, C0{});
            if (act[0])
                mma(img(ib), acc, J0{}, std::integral_constant<int, 1>{});
            auto stage_next = [&]() {
                if (rows_first && more)
                    write_rows(img(ib ^ 1));
            };
            if (act[0])
                epilogue(acc, col0, nl[mb], s_i(mb), s_col(mb), J0{}, stage_next);
            else {
                stage_next();
                idle_stores();
            }
            if (more)
                nl[mb ^ 1] = stage_marks(tile + 1, mb ^ 1);
            __syncthreads();
            ib ^= 1;
        }
        finish();
        return;
    }
#pragma unroll 1
    for (int tile = t0; tile < t1; tile++) {
        const int b = (tile - t0) & 1;
        const bool more = tile + 1 < t1;  // block-uniform
        if (more)
            issue_rows(tile + 1, C0{});
        const long long col0 = static_cast<long long>(tile) * NCOL + 64 * st;
        // an idle wave (row block past RB) issues the same two stores, past
        // the buffer's extent (dropped): with the store count equal on both
        // sides of the branch, the compiler's vmcnt wait for the next tile's
        // rows stays behind them instead of draining this tile's stores
        // (vmcnt(0) on the merged path)
        // the next tile's rows go to LDS before this tile's stores issue: on
        // gfx9 loads and stores share vmcnt, so waiting for the rows after
        // the stores drained the stores too (the whole store latency per
        // tile); here the wait covers the rows (issued at the top of the
        // iteration) and the previous tile's stores
        // (KS >= 8: k128 encode 0.985 -> 0.917 ms, k200 0.70 -> 0.67 ms; the
        // short KS = 4 decodes keep the rows after the stores: cfg3 decode
        // 0.186 vs 0.192 ms, gpurun_out ab_ws)
        constexpr bool rows_first = KS >= 8;
        auto stage_next = [&]() {
            if (rows_first && more)
                write_rows(img(b ^ 1));
        };
        [&]<int... J>(std::integer_sequence<int, J...>) {
            ((act[J] ? compute(img(b), col0, nl[b], s_i(b), s_col(b),
                               std::integral_constant<int, J>{}, stage_next)
                     : (J == RPW - 1 ? (stage_next(), idle_stores()) : idle_stores())),
             ...);
        }(std::make_integer_sequence<int, RPW>{});
        if (!rows_first && more)
            write_rows(img(b ^ 1));
        if (more)
            nl[b ^ 1] = stage_marks(tile + 1, b ^ 1);
        __syncthreads();
    }
    finish();
}


// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static int grid_for(long long words, int cols, int n_stripes, int* tiles)
{
    const long long per = static_cast<long long>(kBlock) * cols;
    const long long t = (words + per - 1) / per;
    if (t <= 0 || t * n_stripes > 0x7fffffffLL)
        return -1;
    *tiles = static_cast<int>(t);
    return 0;
}

// byte extent of `rows` rows of `words` u16 at row stride rs (elements);
// 0 when it does not fit a 32-bit buffer range
static uint32_t extent(long long rows, long long rs, long long words)
{
    if (rows <= 0)
        return 0;
    const long long e = ((rows - 1) * rs + words) * 2;
    return e > 0 && e < 0x7fffffffLL ? static_cast<uint32_t>(e) : 0;
}

template <int K, int COLS, bool KEQ, bool BUF>
static int enc_launch(int k, int n, int n_out, const int32_t* tw,
                      const uint16_t* data, long long dss, long long drs,
                      uint32_t iext, RowDst out, uint32_t oext, long long words,
                      int S, Oor oor, hipStream_t st)
{
    int tiles;
    if (grid_for(words, COLS, S, &tiles))
        return -1;
    hipLaunchKernelGGL((encode_fnt_kernel<K, COLS, KEQ, BUF>), dim3(tiles * S),
                       dim3(kBlock), 0, st, k, n, n_out, tw, data, dss,
                       static_cast<uint32_t>(drs * 2), iext, out.base, out.ss,
                       static_cast<uint32_t>(out.rs * 2), oext, words, tiles,
                       oor);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

static bool aligned_for(int cols, const void* p, long long a, long long b,
                        long long c, long long d)
{
    const long long m = cols;
    return (reinterpret_cast<uintptr_t>(p) % (2 * cols)) == 0 && a % m == 0 &&
           b % m == 0 && c % m == 0 && d % m == 0;
}

int launch_encode_fnt(int k, int n, int n_out, const int32_t* d_twist,
                      const uint16_t* data, long long dss, long long drs,
                      RowDst out, long long words, int S, Oor oor,
                      uint32_t* /*d_err*/, hipStream_t st)
{
    const int K = static_cast<int>(ceil2(static_cast<uint32_t>(k)));
    const bool a2 = aligned_for(2, data, dss, drs, out.ss, out.rs) &&
                    (reinterpret_cast<uintptr_t>(out.base) % 4) == 0;
    const uint32_t ie = extent(k, drs, words), oe = extent(n_out, out.rs, words);
    if (!ie || !oe) {
        // stripes wider than a 31-bit buffer range: flat addressing
        switch (K) {
#define QI_ENC_FLAT(KK)                                                        \
    case KK:                                                                   \
        return enc_launch<KK, 1, false, false>(k, n, n_out, d_twist, data, dss, \
                                               drs, 0, out, 0, words, S, oor,  \
                                               st);
            QI_ENC_FLAT(1)
            QI_ENC_FLAT(2)
            QI_ENC_FLAT(4)
            QI_ENC_FLAT(8)
            QI_ENC_FLAT(16)
            QI_ENC_FLAT(32)
            QI_ENC_FLAT(64)
#undef QI_ENC_FLAT
        default:
            return -3;
        }
    }
#define QI_ENC(KK, C2)                                                         \
    if (K == KK) {                                                             \
        if (a2 && k == KK)                                                     \
            return enc_launch<KK, C2, true, true>(k, n, n_out, d_twist, data,  \
                                                  dss, drs, ie, out, oe,       \
                                                  words, S, oor, st);          \
        if (a2)                                                                \
            return enc_launch<KK, C2, false, true>(k, n, n_out, d_twist, data, \
                                                   dss, drs, ie, out, oe,      \
                                                   words, S, oor, st);         \
        return enc_launch<KK, 1, false, true>(k, n, n_out, d_twist, data, dss, \
                                              drs, ie, out, oe, words, S, oor, \
                                              st);                             \
    }
    QI_ENC(1, 2)
    QI_ENC(2, 2)
    QI_ENC(4, 2)
    QI_ENC(8, 2)
    QI_ENC(16, 2)
    QI_ENC(32, 1)
    QI_ENC(64, 1)
#undef QI_ENC
    return -3;  // K > 64: caller uses the matrix path
}

int matrix_kp(int kin)
{
    const int pairs = (kin + 1) / 2;
    if (pairs <= 2)
        return 2;
    if (pairs <= 4)
        return 4;
    if (pairs <= 8)
        return 8;
    if (pairs <= 16)
        return 16;
    if (pairs <= 32)
        return 32;
    if (pairs <= 64)
        return 64;
    if (pairs <= 128)
        return 128;
    if (2 * pairs <= kMatGenMaxKin + 1)
        return 256;  // 256 < k <= 384: matrix cores only (no dot2 tails)
    if (2 * pairs <= kMatMaxKin + 1)
        return 320;  // 384 < k <= 640: (the context layout's unused section)
    return -1;  // larger k runs the NTT path (ntt.hip)
}

template <int KP, int COLS, bool BUF>
static int mat_launch(MatArgs a, int S, hipStream_t st)
{
    if (grid_for(a.words - a.ext.c0, COLS, S, &a.tiles))
        return -1;
    hipLaunchKernelGGL((matrix_kernel<KP, COLS, BUF>), dim3(a.tiles * S), dim3(kBlock), 0,
                       st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// columns per lane: 4 (b64 row loads) while the packed rows fit in
// registers, 2 up to KP 16, else 1; cols 1 is also the flat (BUF=false) path
template <int KP>
static int mat_dispatch(int cols, const MatArgs& a, int S, hipStream_t st)
{
    const bool buf = a.ext.e0 && a.ext.eo && (!a.src.base1 || a.ext.e1);
    if (!buf)
        return mat_launch<KP, 1, false>(a, S, st);
    if constexpr (KP <= 8)
        if (cols == 4)
            return mat_launch<KP, 4, true>(a, S, st);
    if constexpr (KP <= 16)
        if (cols >= 2)
            return mat_launch<KP, 2, true>(a, S, st);
    return mat_launch<KP, 1, true>(a, S, st);
}

template <int KS, int NST, int NW, bool RSPLIT>
static int mfma_launch(MatArgs a, long long wfull, int S, hipStream_t st)
{
    using G = MfmaTile<KS, NST, NW>;
    const long long t = wfull / G::kCols;
    if (t <= 0 || t * S > 0x7fffffffLL)
        return -1;
    a.tiles = static_cast<int>(t);
    const size_t lds = a.L.RB() > 1 ? G::kLdsStaged : G::kLds;
    // dynamic LDS above 64 KiB needs opting in, once per device (a bit per
    // device; a race only repeats the idempotent call)
    static std::atomic<uint64_t> attr_done{0};
    if (G::kLdsStaged > 65536) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess)
            return -2;
        const uint64_t bit = dev < 64 ? 1ull << dev : 0;
        if (!bit || !(attr_done.load(std::memory_order_acquire) & bit)) {
            if (hipFuncSetAttribute(
                    reinterpret_cast<const void*>(&matrix_mfma_kernel<KS, NST, NW, RSPLIT>),
                    hipFuncAttributeMaxDynamicSharedMemorySize,
                    static_cast<int>(G::kLdsStaged)) != hipSuccess)
                return -2;
            attr_done.fetch_or(bit, std::memory_order_release);
        }
    }
    hipLaunchKernelGGL((matrix_mfma_kernel<KS, NST, NW, RSPLIT>), dim3(t * S),
                       dim3(G::kThreads), lds, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}


static int gen_launch(MatArgs a, long long wfull, int S, hipStream_t st)
{
    constexpr int NST = 8, NW = 4;
    using G = MfmaTile<4, NST, NW>;
    const long long t = wfull / G::kCols;
    if (t <= 0 || t * S > 0x7fffffffLL)
        return -1;
    a.tiles = static_cast<int>(t);
    static std::atomic<uint64_t> attr_done{0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        return -2;
    const uint64_t bit = dev < 64 ? 1ull << dev : 0;
    if (!bit || !(attr_done.load(std::memory_order_acquire) & bit)) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&gen_mfma_kernel<NST, NW>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                static_cast<int>(G::kLdsStaged)) != hipSuccess)
            return -2;
        attr_done.fetch_or(bit, std::memory_order_release);
    }
    hipLaunchKernelGGL((gen_mfma_kernel<NST, NW>), dim3(t * S), dim3(G::kThreads),
                       G::kLdsStaged, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Block geometry by matrix shape (kRouteTile = 1024 must be a multiple of
// the block width):
//  - short matrices (RB < 4: decodes, k x k): 4 waves, each on its own super
//    tiles; 1024 columns at KS = 1 (35 KB LDS), 512 at KS = 2, 4 (one u16
//    column per lane at KS = 4 -- 256 columns -- slowed the cfg3 decode,
//    profiles/r1_ab_mfma_cols1.txt);
//  - tall ones (RB >= 4: encode generators): the waves split the row blocks
//    over the whole image.  8 waves over 256 columns (54 KB LDS: 2 blocks =
//    4 waves per SIMD instead of 2) measured slower on the 1024 x 64 cfg3
//    generator (1.37 vs 1.22 ms, gpurun_out r2f), so the block stays at 4
//    waves.

// operand-stationary kernel (KS = 8, 16): G row-block groups of 8 waves, C
// column ranges per stripe; about two blocks per CU over the launch
static constexpr bool kMmOs = true;
constexpr long long kOsMaxTiles = 4096;  // tiles per block (slow-tile bitmask)

template <int KS, int WR, int RPW>
static int os_launch(MatArgs a, long long wfull, int S, hipStream_t st)
{
    using O = OsTile<OsK<KS>::KC, WR>;
    // the systematic decodes' two source regions (not at KS = 24 with two
    // row blocks per wave: 28 bytes of scratch; os_geom)
    constexpr bool kTwo = !(KS >= 24 && RPW == 2);
    const long long TS = wfull / O::kCols;
    if (TS <= 0 || TS > 0x7fffffffLL)
        return -1;
    const int RB = a.L.RB();
    const int G = (RB + WR * RPW - 1) / (WR * RPW);
    constexpr size_t lds = O::kLds + kOsMaxTiles / 8;
    // per device, once: the dynamic-LDS attribute and the number of blocks
    // the device holds at once (CUs x blocks per CU)
    static std::atomic<uint64_t> attr_done{0};
    static std::atomic<int> slots_of[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        return -2;
    const uint64_t bit = dev < 64 ? 1ull << dev : 0;
    if (!bit || !(attr_done.load(std::memory_order_acquire) & bit)) {
        const void* two_fn = nullptr;
        if constexpr (kTwo)
            two_fn = reinterpret_cast<const void*>(&matrix_os_kernel<KS, WR, RPW, true>);
        if (lds > 65536 &&
            ((two_fn && hipFuncSetAttribute(two_fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            static_cast<int>(lds)) != hipSuccess) ||
             hipFuncSetAttribute(
                 reinterpret_cast<const void*>(&matrix_os_kernel<KS, WR, RPW, false>),
                 hipFuncAttributeMaxDynamicSharedMemorySize,
                 static_cast<int>(lds)) != hipSuccess))
            return -2;
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &per_cu, reinterpret_cast<const void*>(&matrix_os_kernel<KS, WR, RPW, false>),
                O::kThreads, lds) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                hipSuccess)
            return -2;
        if (bit) {
            slots_of[dev].store(std::max(1, per_cu) * std::max(1, cus),
                                std::memory_order_relaxed);
            attr_done.fetch_or(bit, std::memory_order_release);
        }
    }
    const long long slots = bit ? slots_of[dev].load(std::memory_order_relaxed) : 256;
    // blocks wanted over the launch: ~2 per CU, or ~8 for the short KS = 4
    // decodes (cfg3: two column ranges per stripe, 0.168 -> 0.158 ms; the
    // KS >= 8 decodes and generators lose at 2048, gpurun_out ab_x4)
    constexpr long long kTarget = KS == 4 ? 2048 : 512;
    const long long SG = static_cast<long long>(S) * G;
    const long long cmax = std::max(1LL, TS / 4);
    long long C = (kTarget + SG - 1) / SG;
    C = std::max(1LL, std::min(C, cmax));
    // the blocks are equal: a launch of B blocks takes ceil(B / slots)
    // rounds, so among C .. 2C - 1 take the column-range count whose last
    // round is fullest (k300 / k384: 576 blocks on 256 one-block CUs ran
    // three rounds, the last a quarter full; 768 fill them), then let the
    // XCD map have S * C a multiple of 8
    {
        long long best = C;
        double best_eff = 0.0;
        for (long long c = C; c < 2 * C && c <= cmax; c++) {
            const long long B = SG * c;
            const double eff = static_cast<double>(B) / (((B + slots - 1) / slots) * slots);
            if (eff > best_eff + 1e-9) {
                best_eff = eff;
                best = c;
            }
        }
        C = best;
    }
    while ((S * C) % 8 != 0 && C < TS / 2)
        C++;
    // at most kOsMaxTiles tiles per block (the LDS bitmask of its slow
    // tiles)
    C = std::max(C, (TS + kOsMaxTiles - 1) / kOsMaxTiles);
    const long long blocks = SG * C;
    if (blocks > 0x7fffffffLL)
        return -1;
    a.tiles = static_cast<int>(TS);
    if (a.src.base1) {
        if constexpr (!kTwo)
            return -1;  // not chosen by os_geom
        else
            hipLaunchKernelGGL((matrix_os_kernel<KS, WR, RPW, true>),
                               dim3(static_cast<unsigned>(blocks)), dim3(O::kThreads), lds, st,
                               a, G, static_cast<int>(C), static_cast<int>(TS));
    } else
        hipLaunchKernelGGL((matrix_os_kernel<KS, WR, RPW, false>),
                           dim3(static_cast<unsigned>(blocks)), dim3(O::kThreads), lds, st,
                           a, G, static_cast<int>(C), static_cast<int>(TS));
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// operand-stationary geometry by shape: (WR row-block slots, RPW row blocks
// per wave); 0 = the per-launch kernel
struct OsGeom {
    int wr, rpw;
};
inline OsGeom os_geom(int KS, int RB, bool two)
{
    if (!kMmOs)
        return {0, 0};
    // KS = 16, 20, 24 with more than one block of 8 row blocks, one source
    // region: two row blocks per wave, so one group (k200, k256) or two
    // (k300, k384) stage each input tile instead of two or three (k200
    // decode 0.757 -> 0.66 ms, k300 0.704 -> 0.653, k256 0.30 -> 0.278,
    // k384 0.88 -> 0.83; encodes ~10 % faster).  The systematic decodes'
    // two regions too since their rows load once (round 6), but not at KS =
    // 24 (28 bytes of scratch); not at KS = 8 (k128 encode 0.725 -> 0.757
    // ms; gpurun_out/ab_r5k, ab_r5l)
    if ((KS == 16 || KS == 20 || (KS == 24 && !two)) && RB > 8)
        return {8, 2};
    // KS = 40 (384 < k <= 640, K chunks): one row block per wave (80
    // operand VGPRs), one or two source regions
    if (KS > 24)
        return {8, 1};
    if (KS >= 8)
        return {8, 1};
    // KS = 4: the short decode matrices (2 super tiles per 128-column tile)
    // and up to 8 row blocks; the tall generators (RB = 64 at cfg3) stay on
    // matrix_mfma_kernel (os at 1 or 4 row blocks per wave: 1.48 / 1.37 vs
    // 1.05 ms, gpurun_out ab_os2 / ab_os3)
    if (KS == 4 && RB <= 8)
        return RB <= 4 ? OsGeom{4, 1} : OsGeom{8, 1};
    return {0, 0};
}

template <int KS>
static int mfma_dispatch(const MatArgs& a, long long wfull, int S, hipStream_t st)
{
    if constexpr (KS == 4) {
        const OsGeom og = os_geom(KS, a.L.RB(), a.src.base1 != nullptr);
        if (og.wr == 4 && og.rpw == 1)
            return os_launch<KS, 4, 1>(a, wfull, S, st);
        if (og.wr == 8 && og.rpw == 1)
            return os_launch<KS, 8, 1>(a, wfull, S, st);
    } else if constexpr (KS == 8) {
        if (os_geom(KS, a.L.RB(), a.src.base1 != nullptr).wr)
            return os_launch<KS, 8, 1>(a, wfull, S, st);
    } else if constexpr (KS == 16 || KS == 20 || KS == 24) {
        const OsGeom og = os_geom(KS, a.L.RB(), a.src.base1 != nullptr);
        if (og.wr && og.rpw == 2)
            return os_launch<KS, 8, 2>(a, wfull, S, st);
        if (og.wr)
            return os_launch<KS, 8, 1>(a, wfull, S, st);
    } else if constexpr (KS == 40) {
        if (os_geom(KS, a.L.RB(), a.src.base1 != nullptr).wr)
            return os_launch<KS, 8, 1>(a, wfull, S, st);
        return -1;
    }
    constexpr int NSTS = KS == 1 ? 16 : 8;
    const int RB = a.L.RB();
    if constexpr (KS > 16) {
        return -1;  // only the operand-stationary kernel takes kin > 256
    } else if constexpr (KS == 16) {
        // 128 < k <= 256: a 512-row byte-plane image of 64 columns (41 KB);
        // 8 waves over 128 columns (94 KB, 1 block per CU) measured the
        // same at k200 / k256 (profiles/r2_ab_round2b.txt)
        (void)RB;
        return mfma_launch<KS, 1, 4, true>(a, wfull, S, st);
    } else if constexpr (KS == 8) {
        // 65 <= k <= 128: a 256-row byte-plane image, the waves always
        // splitting the row blocks (a wave past the last row block idles)
        // (256 columns, 81 KB with the staging tiles: 2 blocks per CU as
        // the VGPRs allow anyway; 128 columns measured 5 % slower at k128)
        (void)RB;
        return mfma_launch<KS, 4, 4, true>(a, wfull, S, st);
    } else {
        if constexpr (KS == 4) {
            // a tall generator over one source region (every encode):
            // the lean generator kernel
            if (RB >= 4 && !a.in_oor.counts && !a.route && !a.ids &&
                !a.src.base1)
                return gen_launch(a, wfull, S, st);
        }
        if (RB >= 4)
            return mfma_launch<KS, NSTS, 4, true>(a, wfull, S, st);
        return mfma_launch<KS, NSTS, 4, false>(a, wfull, S, st);
    }
}


// rows at `cols`-word aligned offsets (source regions and destination)
static bool rows_aligned(int cols, const RowSrc& src, const RowDst& dst)
{
    return aligned_for(cols, src.base0, src.ss0, src.rs0, dst.ss, dst.rs) &&
           (src.base1 == nullptr || aligned_for(cols, src.base1, src.ss1, src.rs1, 0, 0)) &&
           (reinterpret_cast<uintptr_t>(dst.base) % (2 * cols)) == 0;
}

static MatExt mat_ext(const RowSrc& src, int R, const RowDst& dst, long long words)
{
    return MatExt{extent(src.rows0, src.rs0, words), extent(src.rows1, src.rs1, words),
                  extent(R, dst.rs, words), 0};
}

bool matrix_cores_take(const RowSrc& src, const RowDst& dst, int R, long long words)
{
    const MatExt e = mat_ext(src, R, dst, words);
    const bool buf = e.e0 && e.eo && (!src.base1 || e.e1);
    return buf && rows_aligned(2, src, dst) && rows_aligned(4, src, dst) &&
           words >= kRouteTile;
}

static int launch_matrix_kernels(MatArgs a, int S, hipStream_t st, bool* dot2)
{
    *dot2 = false;
    const MatLayout& L = a.L;
    const RowSrc& src = a.src;
    const RowDst& dst = a.dst;
    const long long words = a.words;
    const bool a2 = rows_aligned(2, src, dst);
    const bool buf = a.ext.e0 && a.ext.eo && (!src.base1 || a.ext.e1);
    const bool a4 = a2 && rows_aligned(4, src, dst);
    const int cols = !buf ? 1 : a4 ? 4 : a2 ? 2 : 1;
    // whole kRouteTile column tiles on the matrix cores, the tail (and
    // everything the MFMA kernel does not take) on the dot2 kernel
    const long long wfull = words / kRouteTile * kRouteTile;
    if (L.KS() > 0 && buf && a4 && wfull > 0) {
        int rc;
        if (L.KS() == 1)
            rc = mfma_dispatch<1>(a, wfull, S, st);
        else if (L.KS() == 2)
            rc = mfma_dispatch<2>(a, wfull, S, st);
        else if (L.KS() == 4)
            rc = mfma_dispatch<4>(a, wfull, S, st);
        else if (L.KS() == 8)
            rc = mfma_dispatch<8>(a, wfull, S, st);
        else if (L.KS() == 16)
            rc = mfma_dispatch<16>(a, wfull, S, st);
        else if (L.KS() == 20)
            rc = mfma_dispatch<20>(a, wfull, S, st);
        else if (L.KS() == 24)
            rc = mfma_dispatch<24>(a, wfull, S, st);
        else
            rc = mfma_dispatch<40>(a, wfull, S, st);
        if (rc || wfull == words)
            return rc;
        a.ext.c0 = wfull;
    }
    *dot2 = true;
    switch (L.KP) {
    case 2:
        return mat_dispatch<2>(cols, a, S, st);
    case 4:
        return mat_dispatch<4>(cols, a, S, st);
    case 8:
        return mat_dispatch<8>(cols, a, S, st);
    case 16:
        return mat_dispatch<16>(cols, a, S, st);
    case 32:
        return mat_dispatch<32>(cols, a, S, st);
    case 64:
        return mat_dispatch<64>(cols, a, S, st);
    case 128:
        return mat_dispatch<128>(cols, a, S, st);
    default:
        return -3;
    }
}

std::string matrix_kernel_names(const MatLayout& L, long long words, bool in_oor, bool two)
{
    // mirrors launch_matrix_kernels / mfma_dispatch / mat_dispatch for rows
    // at 8-byte aligned offsets inside 31-bit buffer ranges; the names are
    // spelled as the demangler (and rocprofv3) spells the instantiations
    std::string r;
    const long long wfull = words / kRouteTile * kRouteTile;
    const int KS = L.KS();
    auto tf = [](bool b) { return std::string(b ? "true" : "false"); };
    if (KS > 0 && wfull > 0) {
        const int RB = L.RB();
        int nst = KS == 1 ? 16 : 8, nw = 4;
        bool rsplit = RB >= 4;
        if (KS == 16) {
            nst = 1;
            rsplit = true;
        } else if (KS == 8) {
            nst = 4;
            rsplit = true;
        }
        const OsGeom og = os_geom(KS, RB, two);
        if (og.wr)
            r = "matrix_os_kernel<" + std::to_string(KS) + ", " + std::to_string(og.wr) + ", " +
                std::to_string(og.rpw) + ", " + tf(two) + ">";
        else if (KS == 4 && RB >= 4 && !in_oor && !two)
            r = "gen_mfma_kernel<8, 4>";  // (an encode: no ids, no input marks)
        else
            r = "matrix_mfma_kernel<" + std::to_string(KS) + ", " + std::to_string(nst) + ", " +
                std::to_string(nw) + ", " + tf(rsplit) + ">";
    }
    if (wfull < words) {
        const int cols = L.KP <= 8 ? 4 : L.KP <= 16 ? 2 : 1;
        r += std::string(r.empty() ? "" : " + ") + "matrix_kernel<" + std::to_string(L.KP) +
             ", " + std::to_string(cols) + ", true> (tail)";
        // the dot2 kernel's slow tiles (the matrix cores redo their own)
        if (in_oor)
            r += " + matrix_redo_kernel";
    }
    return r;
}

std::string encode_fnt_kernel_name(int k)
{
    const int K = static_cast<int>(ceil2(static_cast<uint32_t>(k)));
    return "encode_fnt_kernel<" + std::to_string(K) + ", " + std::to_string(K <= 16 ? 2 : 1) +
           ", " + (k == K ? "true" : "false") + ", true>";
}

int launch_matrix(const MatLayout& L, const int32_t* mat, long long ms,
                  const int32_t* ids, long long is, RowSrc src, RowDst dst,
                  long long words, int S, const Oor* in_oor, int slot_base,
                  const Oor* out_oor, const int32_t* rowmap, const uint32_t* route,
                  long long rstride, SlowList slow, uint32_t* err, hipStream_t st)
{
    if (!rowmap)
        return -1;
    if (L.KP != matrix_kp(L.kin))
        return -4;
    if (in_oor && !slow.base)
        return -1;  // input marks need the slow-tile lists
    const Oor none{nullptr, nullptr, 0, 0};
    MatArgs a{L, mat, ms, ids, is, src, dst, mat_ext(src, L.R, dst, words), words, 0, in_oor ? *in_oor : none, slot_base, out_oor ? *out_oor : none,
              rowmap, route, rstride, in_oor ? slow : SlowList{nullptr, 0}, err};
    bool dot2 = false;
    const int rc = launch_matrix_kernels(a, S, st, &dot2);
    if (rc || !in_oor || !dot2)
        return rc;
    // the dot2 kernel's tiles with more marks than its LDS list (the matrix
    // cores redo theirs themselves): see push_slow_tile
    const int grid = (S + kRedoSpan - 1) / kRedoSpan;
    hipLaunchKernelGGL(matrix_redo_kernel, dim3(grid), dim3(kBlock), 0, st, a, S);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace qi
