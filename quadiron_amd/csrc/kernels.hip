// HIP kernels for RS-FNT over GF(65537) on CDNA4 (gfx950).
//
// Layout: every fragment row is a contiguous run of u16 symbols ("words");
// a stripe is the set of rows sharing a column index range.  One lane owns
// COLS adjacent columns of one stripe, so every global access of a wave is a
// contiguous 64*COLS*2-byte segment of one row (coalesced), and every column
// -- an independent RS codeword read "vertically" across the fragments
// (src/fec_base.h:1103-1150) -- is transformed entirely in VGPRs.
#include <hip/hip_runtime.h>

#include "fnt_codelets.h"
#include "gf65537.h"
#include "matrix_pack.h"
#include "qi_internal.h"

namespace qi {

constexpr int kBlock = 256;

__device__ __forceinline__ void record_oor(const Oor& o, int s, int slot,
                                           long long col)
{
    const uint32_t e = atomicAdd(&o.counts[static_cast<long long>(s) * o.slots + slot], 1u);
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

// Loads of COLS adjacent u16 columns.  FULL: one dword / dwordx2 per lane;
// otherwise the lane masks columns past `avail`.
template <int COLS, bool FULL>
__device__ __forceinline__ void load_cols(const uint16_t* p, long long avail,
                                          int32_t* v)
{
    if constexpr (FULL) {
        if constexpr (COLS == 1) {
            v[0] = p[0];
        } else if constexpr (COLS == 2) {
            const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
            v[0] = w & 0xffff;
            v[1] = w >> 16;
        } else {
            const uint2 w = *reinterpret_cast<const uint2*>(p);
            v[0] = w.x & 0xffff;
            v[1] = w.x >> 16;
            v[2] = w.y & 0xffff;
            v[3] = w.y >> 16;
        }
    } else {
#pragma unroll
        for (int c = 0; c < COLS; c++)
            v[c] = c < avail ? p[c] : 0;
    }
}

template <int COLS, bool FULL>
__device__ __forceinline__ void store_cols(uint16_t* p, long long avail,
                                           const uint32_t* v)
{
    if constexpr (FULL) {
        if constexpr (COLS == 1) {
            p[0] = static_cast<uint16_t>(v[0]);
        } else if constexpr (COLS == 2) {
            *reinterpret_cast<uint32_t*>(p) = (v[0] & 0xffff) | (v[1] << 16);
        } else {
            uint2 w;
            w.x = (v[0] & 0xffff) | (v[1] << 16);
            w.y = (v[2] & 0xffff) | (v[3] << 16);
            *reinterpret_cast<uint2*>(p) = w;
        }
    } else {
#pragma unroll
        for (int c = 0; c < COLS; c++)
            if (c < avail)
                p[c] = static_cast<uint16_t>(v[c]);
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
// ---------------------------------------------------------------------------
template <int K, int COLS, bool FULL>
__device__ __forceinline__ void encode_body(
    int k, int n, int n_out, const int32_t* __restrict__ twist,
    const uint16_t* __restrict__ src, long long drs, uint16_t* __restrict__ dst,
    long long ors, long long col, long long avail, int s, const Oor& oor)
{
    const bool rec = oor.counts != nullptr;
    int32_t x[COLS][K];
#pragma unroll
    for (int t = 0; t < K; t++) {
        const int row = t < k ? t : k - 1;  // branch-free: clamp, then mask
        int32_t v[COLS];
        load_cols<COLS, FULL>(src + row * drs, avail, v);
#pragma unroll
        for (int c = 0; c < COLS; c++)
            x[c][t] = t < k ? v[c] : 0;
    }

    const int passes = n / K;
    for (int v = 0; v < passes; v++) {
        int32_t y[COLS][K];
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
                    y[c][t] = t == 0 ? x[c][t] : fold(x[c][t] * cb);
            }
#pragma unroll
            for (int c = 0; c < COLS; c++)
                dft<K, kTwLo, kTwHi>(y[c]);
        }
        // outputs are in V = [-2, 65537]: the fast path stores the low 16
        // bits; any value outside [0, 65535] (the true OOR symbol 65536 or a
        // non-canonical alias) sends the pass through the fix-up below
        uint32_t bad = 0;
#pragma unroll
        for (int u = 0; u < K; u++) {
            const int row = passes * u + v;
            uint32_t o[COLS];
#pragma unroll
            for (int c = 0; c < COLS; c++) {
                o[c] = static_cast<uint32_t>(y[c][u]);
                bad |= o[c];
            }
            if (row < n_out)
                store_cols<COLS, FULL>(dst + row * ors, avail, o);
        }
        if (__builtin_expect((bad >> 16) != 0, 0)) {
#pragma unroll
            for (int u = 0; u < K; u++) {
                const int row = passes * u + v;
                bool any = false;
                uint32_t o[COLS];
#pragma unroll
                for (int c = 0; c < COLS; c++) {
                    const uint32_t cv = canon_v(y[c][u]);
                    o[c] = cv & 0xffffu;
                    if (static_cast<uint32_t>(y[c][u]) > 65535u && row < n_out) {
                        any = true;
                        if (rec && cv == 65536u && c < avail)
                            record_oor(oor, s, row, col + c);
                    }
                }
                if (any)
                    store_cols<COLS, FULL>(dst + row * ors, avail, o);
            }
        }
    }
}

template <int K, int COLS>
__global__ __launch_bounds__(kBlock) void encode_fnt_kernel(
    int k, int n, int n_out, const int32_t* __restrict__ twist,
    const uint16_t* __restrict__ data, long long dss, long long drs,
    uint16_t* __restrict__ out, long long oss, long long ors, long long words,
    int tiles, Oor oor)
{
    const int b = blockIdx.x;
    const int s = b / tiles;
    const int tile = b - s * tiles;
    const long long col0 = static_cast<long long>(tile) * kBlock * COLS;
    const long long col = col0 + static_cast<long long>(threadIdx.x) * COLS;
    const uint16_t* src = data + s * dss + col;
    uint16_t* dst = out + s * oss + col;
    if (col0 + kBlock * COLS <= words) {  // block-uniform
        encode_body<K, COLS, true>(k, n, n_out, twist, src, drs, dst, ors, col,
                                   COLS, s, oor);
    } else {
        if (col >= words)
            return;
        encode_body<K, COLS, false>(k, n, n_out, twist, src, drs, dst, ors,
                                    col, words - col, s, oor);
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

template <int KP, int COLS, bool FULL>
__device__ __forceinline__ void matrix_load(int kin, const uint16_t* sid,
                                            const RowSrc& src, long long col,
                                            long long avail, int s,
                                            int32_t (&xp)[COLS][KP])
{
    // every received row, branch-free (rows past kin are masked to 0), then
    // offset to signed 16 bit (x - 32768) and pack row pairs for dot2
#pragma unroll
    for (int j = 0; j < KP; j++) {
        int32_t vv[2][COLS];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int i = 2 * j + h;
            const int ii = i < kin ? i : kin - 1;
            const int id = src.by_pos ? ii : (sid ? sid[ii] : ii);
            const uint16_t* p =
                id < src.split ? src.base0 + s * src.ss0 + id * src.rs0
                               : src.base1 + s * src.ss1 + (id - src.split) * src.rs1;
            load_cols<COLS, FULL>(p + col, avail, vv[h]);
#pragma unroll
            for (int c = 0; c < COLS; c++)
                vv[h][c] = i < kin ? vv[h][c] : 0;
        }
#pragma unroll
        for (int c = 0; c < COLS; c++)
            xp[c][j] = static_cast<int32_t>(
                (static_cast<uint32_t>(vv[0][c]) |
                 (static_cast<uint32_t>(vv[1][c]) << 16)) ^
                0x80008000u);
    }
}

template <int KP, int COLS, bool FULL>
__device__ __forceinline__ void matrix_compute(
    const MatLayout& L, const int32_t* sm, const int32_t* __restrict__ plain,
    const int32_t (&xp)[COLS][KP], uint16_t* __restrict__ obase, long long ors,
    long long col, long long avail, int s, int n_marks, const int* s_i,
    const uint32_t* s_col, const Oor& out_oor)
{
    // sm: the packed matrix, kcorr and rscale staged in LDS
    const int kin = L.kin;
    const int32_t* kcorr = sm + L.kcorr();
    const int32_t* rscale = sm + L.rscale();
    const bool rec = out_oor.counts != nullptr;
    for (int t = 0; t < L.R; t++) {
        const int32_t* mrow = sm + t * KP;
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
        for (int e = 0; e < n_marks; e++) {
            // restored symbol is 65536 == -1 where the stored word is 0
            const long long d = static_cast<long long>(s_col[e]) - col;
            if (d >= 0 && d < COLS) {
                const int32_t corr = plain[t * kin + s_i[e]];
#pragma unroll
                for (int c = 0; c < COLS; c++)
                    if (c == d)
                        y[c] = fold(fold(y[c] - corr));
            }
        }
        const int32_t rs = rscale[t];
        if (rs != 1) {
#pragma unroll
            for (int c = 0; c < COLS; c++)
                y[c] = fold(fold(y[c] * rs));
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
                if (static_cast<uint32_t>(y[c]) > 65535u && rec && c < avail)
                    record_oor(out_oor, s, t, col + c);
                o[c] = fix16(y[c]);
            }
        }
        store_cols<COLS, FULL>(obase + t * ors, avail, o);
    }
}

template <int KP, int COLS>
__global__ __launch_bounds__(kBlock) void matrix_kernel(
    MatLayout L, const int32_t* __restrict__ mat, long long mat_stride,
    const uint16_t* __restrict__ ids, RowSrc src, RowDst dst, long long words,
    int tiles, Oor in_oor, int slot_base, Oor out_oor, uint32_t* err)
{
    extern __shared__ int32_t s_mat[];  // packed + kcorr + rscale
    __shared__ int s_cnt;
    __shared__ int s_i[kMaxTileOor];
    __shared__ uint32_t s_col[kMaxTileOor];

    const int b = blockIdx.x;
    const int s = b / tiles;
    const int tile = b - s * tiles;
    const int kin = L.kin;
    const long long col0 = static_cast<long long>(tile) * kBlock * COLS;
    const long long col = col0 + static_cast<long long>(threadIdx.x) * COLS;
    const int32_t* M = mat + s * mat_stride;
    const uint16_t* sid = ids ? ids + static_cast<long long>(s) * kin : nullptr;
    const bool full = col0 + kBlock * COLS <= words;  // block-uniform

    // 1) issue every row load of this lane first
    int32_t xp[COLS][KP];
    if (full) {
        matrix_load<KP, COLS, true>(kin, sid, src, col, COLS, s, xp);
    } else if (col < words) {
        matrix_load<KP, COLS, false>(kin, sid, src, col, words - col, s, xp);
    }
    // 2) meanwhile stage the matrix rows in LDS and gather this tile's OOR
    //    marks of the received rows (decode_prepare, src/fec_base.h:1361-1404)
    const int nm = static_cast<int>(L.plain());
    for (int i = threadIdx.x; i < nm; i += kBlock)
        s_mat[i] = M[i];
    if (threadIdx.x == 0)
        s_cnt = 0;
    __syncthreads();
    int n_marks = 0;
    if (in_oor.counts) {
        const long long col1 = col0 + kBlock * COLS;
        for (int i = threadIdx.x; i < kin; i += kBlock) {
            const int id = sid ? sid[i] : i;
            const int slot = (src.by_pos ? i : id) - slot_base;
            if (slot < 0)
                continue;
            const long long bk = static_cast<long long>(s) * in_oor.slots + slot;
            uint32_t c = in_oor.counts[bk];
            if (c > static_cast<uint32_t>(in_oor.cap))
                c = in_oor.cap;
            for (uint32_t e = 0; e < c; e++) {
                const uint32_t w = in_oor.entries[bk * in_oor.cap + e];
                if (w >= col0 && w < col1 && w < words) {
                    const int p = atomicAdd(&s_cnt, 1);
                    if (p < kMaxTileOor) {
                        s_i[p] = i;
                        s_col[p] = w;
                    } else {
                        atomicOr(err, 1u);
                    }
                }
            }
        }
    }
    __syncthreads();
    n_marks = min(s_cnt, kMaxTileOor);
    uint16_t* obase = dst.base + s * dst.ss + col;
    const int32_t* plain = M + L.plain();
    if (full) {
        matrix_compute<KP, COLS, true>(L, s_mat, plain, xp, obase, dst.rs, col,
                                       COLS, s, n_marks, s_i, s_col, out_oor);
    } else if (col < words) {
        matrix_compute<KP, COLS, false>(L, s_mat, plain, xp, obase, dst.rs, col,
                                        words - col, s, n_marks, s_i, s_col,
                                        out_oor);
    }
}

// ---------------------------------------------------------------------------
// Per-stripe decode context: the Lagrange form of DecodeContext::init
// (src/fec_context.h:232-274).  For received points x_i = r^{id_i}:
//   A(x) = prod_j (x - x_j),  Q_i = A / (x - x_i),  A'(x_i) = Q_i(x_i)
//   mode 0: M[t][i] = coef_t(Q_i) / A'(x_i)       (non-systematic)
//   mode 1: M[t][i] = Q_i(r^t)   / A'(x_i)        (systematic)
// One 64-lane workgroup per stripe; k <= 64.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mulm(uint32_t a, uint32_t b)
{
    return static_cast<uint32_t>((static_cast<uint64_t>(a) * b) % 65537u);
}
__device__ __forceinline__ uint32_t addm(uint32_t a, uint32_t b)
{
    const uint32_t c = a + b;
    return c >= 65537u ? c - 65537u : c;
}
__device__ __forceinline__ uint32_t subm(uint32_t a, uint32_t b)
{
    return a >= b ? a - b : a + 65537u - b;
}

__global__ __launch_bounds__(64) void decode_ctx_kernel(
    int k, uint32_t r, int mode, MatLayout L, const uint16_t* __restrict__ ids,
    int32_t* __restrict__ mat)
{
    __shared__ uint32_t xs[64];
    __shared__ uint32_t A[65];
    __shared__ uint32_t Mt[64 * 64];
    const int s = blockIdx.x;
    const int tid = threadIdx.x;
    const long long mstride = static_cast<long long>(L.words());

    if (tid < k)
        xs[tid] = powmod_c(r, ids[static_cast<long long>(s) * k + tid]);
    __syncthreads();
    if (tid == 0) {
        A[0] = 1;
        for (int i = 0; i < k; i++) {
            const uint32_t neg = subm(0, xs[i]);
            A[i + 1] = A[i];
            for (int d = i; d > 0; d--)
                A[d] = addm(A[d - 1], mulm(A[d], neg));
            A[0] = mulm(A[0], neg);
        }
    }
    __syncthreads();
    if (tid < k) {
        const uint32_t xi = xs[tid];
        uint32_t q[64];
        q[k - 1] = A[k];
        for (int j = k - 1; j >= 1; j--)
            q[j - 1] = addm(A[j], mulm(xi, q[j]));
        uint32_t den = 1;
        for (int j = 0; j < k; j++)
            if (j != tid)
                den = mulm(den, subm(xi, xs[j]));
        const uint32_t inv = powmod_c(den, 65535u);
        if (mode == 0) {
            for (int t = 0; t < k; t++)
                Mt[t * k + tid] = mulm(q[t], inv);
        } else {
            uint32_t e = 1;
            for (int t = 0; t < k; t++) {
                uint32_t acc = 0;
                for (int j = k - 1; j >= 0; j--)
                    acc = addm(mulm(acc, e), q[j]);
                Mt[t * k + tid] = mulm(acc, inv);
                e = mulm(e, r);
            }
        }
    }
    __syncthreads();
    for (int t = tid; t < L.R; t += 64)
        pack_row(Mt + t * k, k, L.KP, L.R, t, mat + s * mstride);
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

template <int K, int COLS>
static int enc_launch(int k, int n, int n_out, const int32_t* tw,
                      const uint16_t* data, long long dss, long long drs,
                      RowDst out, long long words, int S, Oor oor,
                      hipStream_t st)
{
    int tiles;
    if (grid_for(words, COLS, S, &tiles))
        return -1;
    hipLaunchKernelGGL((encode_fnt_kernel<K, COLS>), dim3(tiles * S),
                       dim3(kBlock), 0, st, k, n, n_out, tw, data, dss, drs,
                       out.base, out.ss, out.rs, words, tiles, oor);
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
#define QI_ENC(KK, C2)                                                        \
    if (K == KK)                                                              \
        return a2 ? enc_launch<KK, C2>(k, n, n_out, d_twist, data, dss, drs,  \
                                       out, words, S, oor, st)                \
                  : enc_launch<KK, 1>(k, n, n_out, d_twist, data, dss, drs,   \
                                      out, words, S, oor, st);
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
    return -1;
}

template <int KP, int COLS>
static int mat_launch(const MatLayout& L, const int32_t* mat, long long ms,
                      const uint16_t* ids, RowSrc src, RowDst dst,
                      long long words, int S, Oor in_oor, int slot_base,
                      Oor out_oor, uint32_t* err, hipStream_t st)
{
    int tiles;
    if (grid_for(words, COLS, S, &tiles))
        return -1;
    const size_t lds = L.plain() * sizeof(int32_t);
    if (lds > 64 * 1024)
        return -5;
    hipLaunchKernelGGL((matrix_kernel<KP, COLS>), dim3(tiles * S), dim3(kBlock),
                       lds, st, L, mat, ms, ids, src, dst, words, tiles, in_oor,
                       slot_base, out_oor, err);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_matrix(const MatLayout& L, const int32_t* mat, long long ms,
                  const uint16_t* ids, RowSrc src, RowDst dst, long long words,
                  int S, const Oor* in_oor, int slot_base, const Oor* out_oor,
                  uint32_t* err, hipStream_t st)
{
    Oor none{nullptr, nullptr, 0, 0};
    Oor io = in_oor ? *in_oor : none;
    Oor oo = out_oor ? *out_oor : none;
    const bool a2 = aligned_for(2, src.base0, src.ss0, src.rs0, dst.ss, dst.rs) &&
                    (src.base1 == nullptr ||
                     aligned_for(2, src.base1, src.ss1, src.rs1, 0, 0)) &&
                    (reinterpret_cast<uintptr_t>(dst.base) % 4) == 0;
    if (L.KP != matrix_kp(L.kin))
        return -4;
#define QI_MAT(KK)                                                            \
    if (L.KP == KK)                                                           \
        return a2 ? mat_launch<KK, 2>(L, mat, ms, ids, src, dst, words, S, io, \
                                      slot_base, oo, err, st)                 \
                  : mat_launch<KK, 1>(L, mat, ms, ids, src, dst, words, S, io, \
                                      slot_base, oo, err, st);
    QI_MAT(2)
    QI_MAT(4)
    QI_MAT(8)
    QI_MAT(16)
    QI_MAT(32)
    QI_MAT(64)
#undef QI_MAT
    return -3;
}

int launch_decode_ctx(int k, int /*n*/, uint32_t r, int mode,
                      const MatLayout& L, const uint16_t* d_ids, int S,
                      int32_t* d_mat, hipStream_t st)
{
    if (k > 64 || S <= 0)
        return -3;
    hipLaunchKernelGGL(decode_ctx_kernel, dim3(S), dim3(64), 0, st, k, r, mode,
                       L, d_ids, d_mat);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace qi
