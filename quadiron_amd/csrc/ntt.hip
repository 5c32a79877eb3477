// General-k RS-FNT path (k > 384, and 256 < k <= 384 at column counts that
// are not a multiple of 1024): NTT-structured encode and decode.
//
// These codes do not fit the register codelets of encode_fnt_kernel
// (K = ceil2(k) <= 64) nor the matrix kernels (the operand-stationary
// kernel's LDS image tops out at k = 384, and it has no column tail above
// k = 256: qi_gpu.cpp use_matrix).  They run the reference's own algorithm
// as column-batched NTTs:
//
//   non-systematic encode  NTT_n of the k data rows zero-padded to n
//                          (Radix2::fft, src/fft_2n.h:360-407; outputs
//                          0 .. k+m-1, src/fec_rs_fnt.h:236-251)
//   decode                 FecCode::decode_apply (src/fec_base.h:1418-1448):
//                            y_i = v_i * inv_A_i      (65536 restored at the
//                                                      OOR marks first,
//                                                      decode_prepare :1361-1404)
//                            INTT_n of the y_i placed at positions z_i = ids
//                            NTT_2k of its first k outputs (zero-extended)
//                            x C[j] = -A_fft_2k[j] / len_2k
//                            INTT_2k; first k outputs = the coefficients
//                          (ifft's 1/N and the final negation are folded into
//                          the per-pattern constants C: linear maps commute)
//   systematic decode      the same, then NTT_n evaluated at r^t, t < k
//                          (src/fec_base.h:1348-1353)
//   systematic encode      the interpolation through the data at r^0..r^{k-1}
//                          (the plan's constant context), then NTT_n, outputs
//                          k .. k+m-1 (src/fec_rs_fnt.h:236-251)
//
// Transforms.  X[u] = sum_t x[t] w^(+-ut) down the rows of every column,
// N = 2^b <= 65536, as in-place decimation-in-time passes of radix R <= 32
// over an int32 HBM scratch: pass p (stride S = prod_{q<p} R_q) takes the R
// positions b + s + j S of a group, multiplies element j by w_{SR}^{s j}
// (a wave-uniform table entry) and applies an R-point register codelet
// (fnt_codelets.h, interval-planned lazy reduction).  Pass 0 gathers its
// input in digit-reversed order straight from the source rows (zero past the
// source's rows: the pruned input of Radix2::fft's replicated shortcut,
// src/fft_2n.h:360-407); the last pass writes canonical u16 rows (and OOR
// marks) or leaves the result in the scratch.  Lanes are columns: every load
// and store is a coalesced row run.  The inverse transform uses the same
// codelets with the output index reversed (DFT(x)[-u] = IDFT(x)[u]) and the
// inverse twiddle table.
//
// The per-pattern context (DecodeContext::init, src/fec_context.h:232-274:
// A(x) = prod (x - x_i), 1/(x_i A'(x_i)), FFT_2k(A)) is built on the GPU as
// independent products over the received points (ntt_ctx_kernel), inside
// the caller's stream (no host round trip).
//
// For max(n, len_2k) <= 2048 the whole pipeline of a column tile runs in LDS
// (ntt_lds_kernel); there NTT_2k / INTT_2k run as two len_2k / 2 point
// transforms each (the input's zero half and the output's unused half are
// never transformed).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "fnt_codelets.h"
#include "gf65537.h"
#include "qi_internal.h"
#include "qi_plan.h"

namespace qi {

namespace {

constexpr int kNttBlock = 256;
constexpr int kMaxPasses = 16;

// x * c mod q for |x| < 2^23 and a balanced twiddle |c| <= 32768: the full
// 48-bit product as v_mul_i32_i24 + v_mul_hi_i32_i24, reduced with
// 2^32 = 1 and 2^16 = -1 (p = hi 2^32 + lo: lo16 - hi16 + hi).  Result in
// [-65536, 65535].
__device__ __forceinline__ int32_t mul_rt(int32_t x, int32_t c)
{
    // the two halves written out: the operands are known to fit 24 bits,
    // which the compiler cannot see through the lazily reduced values (it
    // sign-extended both first)
    uint32_t lo;
    int32_t hi;
    asm("v_mul_i32_i24 %0, %1, %2" : "=v"(lo) : "v"(x), "v"(c));
    asm("v_mul_hi_i32_i24 %0, %1, %2" : "=v"(hi) : "v"(x), "v"(c));
    return static_cast<int32_t>(lo & 0xffffu) - static_cast<int32_t>(lo >> 16) + hi;
}

// canonical residue of a V-range value [-2, 65537]
__device__ __forceinline__ uint32_t canon_vr(int32_t y)
{
    const int32_t c = y < 0 ? y + 65537 : y;
    return static_cast<uint32_t>(c >= 65537 ? c - 65537 : c);
}

// codelet input range: gathered u16 (or restored 65536), scratch values
// (V range) and twiddled values [-65536, 65535]
constexpr long long kInLo = -65540, kInHi = 65540;

}  // namespace

// One pass of a transform (all parameters uniform).  Every per-stripe
// pointer is already offset to the first stripe of the launch and to the
// first column of the slice.
struct NttPassArgs {
    int N, S, R, twstep;  // length, stride, radix of this pass; table step
    int first, last, inverse, npass;
    int radix[kMaxPasses];  // the whole radix list (pass 0's digit reversal)
    const int32_t* tw;      // balanced w_nmax^e (inverse table: w_nmax^-e)
    int32_t* scr;           // position P of stripe s at scr + s*sss + P*cols
    long long sss, cols;
    // pass 0 source: sequence element t is source row row(t) = posmap[t]
    // (or t) at in + s*iss + row*irs, u16 or int32; rows outside
    // [0, in_rows) read as zero; optional multiplier scale[s*scs + t]
    const void* in;
    long long iss, irs;
    int in_u16, in_rows;
    const int32_t* posmap;
    const int32_t* scale;
    long long pms, scs;
    // last pass: positions row0 .. row0+out_rows-1 -> u16 rows of out (or
    // stay in the scratch when out is null); OOR marks with absolute column
    // col0 + c into buckets slot = row
    uint16_t* out;
    long long oss, ors;
    int row0, out_rows;
    long long col0;
    Oor oor;
    int tiles;  // column tiles of kNttBlock
};

template <int R>
__global__ __launch_bounds__(kNttBlock) void ntt_pass_kernel(NttPassArgs a)
{
    const int tiles = a.tiles;
    const int s = blockIdx.x / tiles;
    const int tile = blockIdx.x - s * tiles;
    const long long c = static_cast<long long>(tile) * kNttBlock + threadIdx.x;
    if (c >= a.cols)
        return;
    const int grp = blockIdx.y;
    const int S = a.S, N = a.N;
    const int ss = grp % S;             // offset inside the group, [0, S)
    const int b = (grp / S) * (S * R);  // group start
    int32_t* scr = a.scr + s * a.sss;
    int32_t v[R];
    if (a.first) {
        // digit-reversed gather: position b + j holds x[t_rest(b) + j N/R0]
        int trest = 0, Sp = R;
        for (int p = 1; p < a.npass; p++) {
            const int Rp = a.radix[p];
            trest += ((b / Sp) % Rp) * (N / (Sp * Rp));
            Sp *= Rp;
        }
        const int step = N / R;
#pragma unroll
        for (int j = 0; j < R; j++) {
            const int t = trest + j * step;
            const int row = a.posmap ? a.posmap[s * a.pms + t] : t;
            int32_t x = 0;
            if (row >= 0 && row < a.in_rows) {  // uniform
                if (a.in_u16)
                    x = static_cast<const uint16_t*>(a.in)[s * a.iss + row * a.irs + c];
                else
                    x = static_cast<const int32_t*>(a.in)[s * a.iss + row * a.irs + c];
                if (a.scale)
                    x = mul_rt(x, a.scale[s * a.scs + t]);
            }
            v[j] = x;
        }
    } else {
        const int tstep = N / (S * R);
#pragma unroll
        for (int j = 0; j < R; j++) {
            int32_t x = scr[static_cast<long long>(b + ss + j * S) * a.cols + c];
            if (j > 0 && ss > 0)  // w_{SR}^{ss j} = w_N^{ss j N/(SR)}
                x = mul_rt(x, a.tw[ss * j * tstep * a.twstep]);
            v[j] = x;
        }
    }
    dft<R, kInLo, kInHi>(v);  // natural order, outputs in V = [-2, 65537]
    if (a.last && a.out) {
#pragma unroll
        for (int u = 0; u < R; u++) {
            const int32_t y = v[a.inverse ? (R - u) % R : u];
            const int row = b + ss + u * S - a.row0;
            if (row >= 0 && row < a.out_rows) {  // uniform
                const uint32_t cv = canon_vr(y);
                a.out[s * a.oss + row * a.ors + c] = static_cast<uint16_t>(cv);
                if (cv == 65536u && a.oor.counts) {
                    const long long bk = static_cast<long long>(s) * a.oor.slots + row;
                    const uint32_t e = atomicAdd(&a.oor.counts[bk], 1u);
                    if (e < static_cast<uint32_t>(a.oor.cap))
                        a.oor.entries[bk * a.oor.cap + e] = static_cast<uint32_t>(a.col0 + c);
                }
            }
        }
    } else {
#pragma unroll
        for (int u = 0; u < R; u++)
            scr[static_cast<long long>(b + ss + u * S) * a.cols + c] =
                v[a.inverse ? (R - u) % R : u];
    }
}

// ---------------------------------------------------------------------------
// per-pattern decode context (DecodeContext::init, src/fec_context.h:232-274)
// ctx per stripe (int32): inv_A_i[k] | C[len_2k] | posmap[n] | ids[k]
// ---------------------------------------------------------------------------
struct NttCtxLayout {
    int k, n, len2k;
    __host__ __device__ long long c_off() const { return k; }
    __host__ __device__ long long pos_off() const { return static_cast<long long>(k) + len2k; }
    __host__ __device__ long long ids_off() const { return pos_off() + n; }
    __host__ __device__ long long words() const { return ids_off() + k; }
};

__device__ __forceinline__ uint32_t mulm_(uint32_t a, uint32_t b)
{
    const uint64_t p = static_cast<uint64_t>(a) * b;
    const int32_t v = static_cast<int32_t>(p & 0xffffu) -
                      static_cast<int32_t>((p >> 16) & 0xffffu) + static_cast<int32_t>(p >> 32);
    return static_cast<uint32_t>(v < 0 ? v + 65537 : v);
}
__device__ __forceinline__ uint32_t addm_(uint32_t a, uint32_t b)
{
    const uint32_t c = a + b;
    return c >= 65537u ? c - 65537u : c;
}
__device__ __forceinline__ uint32_t subm_(uint32_t a, uint32_t b)
{
    return a >= b ? a - b : a + 65537u - b;
}
__device__ __forceinline__ uint32_t powm_(uint32_t b, uint32_t e)
{
    uint32_t r = 1;
    for (; e; e >>= 1) {
        if (e & 1)
            r = mulm_(r, b);
        b = mulm_(b, b);
    }
    return r;
}

struct NttCtxArgs {
    NttCtxLayout L;
    uint32_t r, w2k;      // n-th and len_2k-th roots of unity
    uint32_t inv_len2k;   // len_2k^-1
    const uint16_t* ids;  // S x k fragment ids (nullptr: 0 .. k-1)
    int32_t* ctx;
    long long cs;
    // lazy build (ntt_build_ctx_lazy): ids as dwords at ids32 + s * cs
    // instead of `ids`; stripes whose lazy word (lazy + s * cs) has
    // kLazyNtt set are skipped
    const int32_t* ids32;
    const uint32_t* lazy;
    uint32_t* err;        // kErrBadIds: an id >= n
};

// a * b mod q for a, b in [0, 65536] on the full-rate 24-bit multipliers:
// the 48-bit product is hi 2^32 + lo (hi <= 1), and with 2^32 = 1, 2^16 = -1
// it reduces to hi + lo16 - lo_hi16 in [-65535, 65536]
__device__ __forceinline__ uint32_t mulm24(uint32_t a, uint32_t b)
{
    uint32_t lo, hi;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(lo) : "v"(a), "v"(b));
    asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(hi) : "v"(a), "v"(b));
    const int32_t v = static_cast<int32_t>(hi + (lo & 0xffffu)) - static_cast<int32_t>(lo >> 16);
    return static_cast<uint32_t>(v < 0 ? v + 65537 : v);
}

constexpr int kCtxChains = 4;  // independent product chains per thread
constexpr int kPosChunk = 2048;  // posmap positions staged in LDS per pass

// The per-pattern constants as independent products, one item per thread
// (DecodeContext::init, src/fec_context.h:232-274, restated):
//   item j < len_2k:   C[j] = -A(w2k^j) / len_2k,  A(z) = prod_i (z - x_i)
//   item len_2k + i:   1 / (x_i A'(x_i)),          A'(x_i) = prod_{j != i} (x_i - x_j)
// so no coefficient of A is ever formed: the reference builds A by k
// in-place multiplications by (x - x_i) and evaluates FFT_2k(A); one
// workgroup per stripe doing that here was a chain of k barriers plus
// O(len_2k k / 256) serial Horner steps per thread (k = 1000: 1.13 ms per
// 16 stripes).  Grid (stripes, item blocks); every block stages the stripe's
// x_i = r^id_i in LDS and each thread multiplies kCtxChains interleaved
// partial products (j = c mod kCtxChains) so the multiplies pipeline.
// Block (s, 0) also writes ids[] and posmap[].
__global__ __launch_bounds__(kNttBlock) void ntt_ctx_kernel(NttCtxArgs a)
{
    extern __shared__ uint32_t xs[];  // x_i, padded to kCtxChains with "x = z"
    const int s = blockIdx.x, tid = threadIdx.x, k = a.L.k;
    const int kp = (k + kCtxChains - 1) / kCtxChains * kCtxChains;
    int32_t* ctx = a.ctx + s * a.cs;
    int32_t* invA = ctx;
    int32_t* C = ctx + a.L.c_off();
    int32_t* posmap = ctx + a.L.pos_off();
    int32_t* ids = ctx + a.L.ids_off();
    if (a.lazy && (a.lazy[s * a.cs] & kLazyNtt))
        return;  // built by an earlier decode (block-uniform)
    const uint16_t* sid = a.ids ? a.ids + static_cast<long long>(s) * k : nullptr;
    const int32_t* sid32 = a.ids32 ? a.ids32 + s * a.cs : nullptr;
    auto id_of = [&](int i) -> uint32_t {
        return sid32 ? static_cast<uint32_t>(sid32[i]) : sid ? sid[i] : static_cast<uint32_t>(i);
    };
    for (int i = tid; i < kp; i += kNttBlock)
        xs[i] = i < k ? powm_(a.r, id_of(i)) : 0xffffffffu;
    if (blockIdx.y == 0) {
        // posmap[t] = the received row holding sequence element t, or -1.
        // Every global word is written once with its final value (staged in
        // LDS, kPosChunk positions at a time): a lazy rebuild racing with a
        // decode on another stream that reads the same context
        // only ever rewrites a word with the value it already holds.
        __shared__ int32_t pm[kPosChunk];
        for (int i = tid; i < k; i += kNttBlock) {
            const int id = static_cast<int>(id_of(i));
            ids[i] = id;
            if (id >= a.L.n)
                atomicOr(a.err, kErrBadIds);
        }
        for (int c0 = 0; c0 < a.L.n; c0 += kPosChunk) {
            for (int t = tid; t < kPosChunk; t += kNttBlock)
                pm[t] = -1;
            __syncthreads();
            for (int i = tid; i < k; i += kNttBlock) {
                const int id = static_cast<int>(id_of(i));
                if (id >= c0 && id < c0 + kPosChunk)
                    pm[id - c0] = i;
            }
            __syncthreads();
            for (int t = tid; t < kPosChunk && c0 + t < a.L.n; t += kNttBlock)
                posmap[c0 + t] = pm[t];
            __syncthreads();
        }
    }
    __syncthreads();
    const int u = blockIdx.y * kNttBlock + tid;
    const int len2k = a.L.len2k;
    if (u >= len2k + k)
        return;
    const bool is_c = u < len2k;
    const int self = is_c ? -1 : u - len2k;
    const uint32_t z = is_c ? powm_(a.w2k, static_cast<uint32_t>(u)) : xs[self];
    uint32_t acc[kCtxChains];
#pragma unroll
    for (int c = 0; c < kCtxChains; c++)
        acc[c] = 1;
    // padding entries (0xffffffff) and x_self contribute a factor 1
    for (int j = 0; j < kp; j += kCtxChains) {
        const uint4 xv = *reinterpret_cast<const uint4*>(xs + j);
        const uint32_t xj[kCtxChains] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
        for (int c = 0; c < kCtxChains; c++) {
            const bool one = xj[c] == 0xffffffffu || j + c == self;
            acc[c] = mulm24(acc[c], one ? 1u : subm_(z, xj[c]));
        }
    }
    uint32_t p = mulm24(mulm24(acc[0], acc[1]), mulm24(acc[2], acc[3]));
    if (is_c)
        C[u] = static_cast<int32_t>(subm_(0u, mulm24(p, a.inv_len2k)));
    else {
        invA[self] = static_cast<int32_t>(powm_(mulm24(p, z), 65535u));
        if (p == 0u)  // A'(x_i) = 0: x_i = x_j for some j != i (repeated ids)
            atomicOr(a.err, kErrBadIds);
    }
}

// after a lazy ntt_ctx_kernel launch on the same stream: mark the stripes'
// NTT contexts built
__global__ __launch_bounds__(256) void lazy_mark_kernel(uint32_t* lazy, long long cs, int S,
                                                        uint32_t bit)
{
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s < S)
        lazy[s * cs] |= bit;
}

// decode step 1: received row i of stripe s -> scratch row i, y = v inv_A_i
struct NttExpandArgs {
    RowSrc src;  // offset to the slice's first column and stripe
    const int32_t* ctx;
    long long cs;
    int ids_off, k;
    int32_t* scr;
    long long sss, cols;
    int tiles;
};

__global__ __launch_bounds__(kNttBlock) void ntt_expand_kernel(NttExpandArgs a)
{
    const int tiles = a.tiles;
    const int s = blockIdx.x / tiles;
    const int tile = blockIdx.x - s * tiles;
    const int i = blockIdx.y;
    const long long c = static_cast<long long>(tile) * kNttBlock + threadIdx.x;
    if (c >= a.cols)
        return;
    const int32_t* ctx = a.ctx + s * a.cs;
    const int id = a.src.by_pos ? i : ctx[a.ids_off + i];
    const uint16_t* row = id < a.src.split
                              ? a.src.base0 + s * a.src.ss0 + id * a.src.rs0
                              : a.src.base1 + s * a.src.ss1 + (id - a.src.split) * a.src.rs1;
    const int32_t x = row[c];
    a.scr[s * a.sss + static_cast<long long>(i) * a.cols + c] =
        mul_rt(x, balanced(static_cast<uint32_t>(ctx[i])));
}

// decode step 1b (decode_prepare, src/fec_base.h:1361-1404): a marked symbol
// is 65536 = -1 whatever was stored, so y = -inv_A_i at the marks of the
// slice [c0, c0 + cols).  One workgroup per (stripe, received row).
struct NttFixArgs {
    Oor in;  // offset to the launch's first stripe
    int slot_base, by_pos;
    const int32_t* ctx;
    long long cs;
    int ids_off;
    int32_t* scr;
    long long sss, cols, c0;
    uint32_t* err;
};

__global__ __launch_bounds__(kNttBlock) void ntt_fix_kernel(NttFixArgs a)
{
    const int s = blockIdx.x, i = blockIdx.y;
    const int32_t* ctx = a.ctx + s * a.cs;
    const int slot = a.by_pos ? i : ctx[a.ids_off + i] - a.slot_base;
    if (slot < 0)
        return;  // systematic data row: no marks
    const long long bk = static_cast<long long>(s) * a.in.slots + slot;
    uint32_t cnt = a.in.counts[bk];
    if (cnt > static_cast<uint32_t>(a.in.cap)) {
        if (threadIdx.x == 0)
            atomicOr(a.err, kErrOorTruncated);
        cnt = static_cast<uint32_t>(a.in.cap);
    }
    const int32_t y = 65537 - static_cast<int32_t>(ctx[i]);  // -inv_A_i in [1, 65537]
    for (uint32_t e = threadIdx.x; e < cnt; e += kNttBlock) {
        const long long col = static_cast<long long>(a.in.entries[bk * a.in.cap + e]) - a.c0;
        if (col >= 0 && col < a.cols)
            a.scr[s * a.sss + static_cast<long long>(i) * a.cols + col] = y;
    }
}

// ---------------------------------------------------------------------------
// LDS-resident engine (max(n, len_2k) <= kLdsMaxN): one workgroup runs every
// transform of a tile of T columns of one stripe in LDS, so HBM sees only the
// algorithmic bytes (the k input rows and the output rows).  The tile is an
// nmax x T int32 image (element (position, column) at buf[prow(pos) T +
// col]: an empty row after every 32, see prow);
// radix <= 32 passes, with every lane on one column of one butterfly group:
//   forward transforms: decimation in frequency (natural order in, output
//     X[j] at position pos(j) -- a mixed-radix digit reversal);
//   inverse transforms: decimation in time, the transposed passes in reverse
//     order (input x[t] at pos(t), natural order out).
// So INTT_n can take the received rows scattered to pos(id), NTT_2k's output
// is directly INTT_2k's input (C[j] applied at pos(j)), and no reordering
// pass is needed (src/fec_base.h:1418-1448 in this order).
// ---------------------------------------------------------------------------
constexpr int kLdsThreads = 512;
constexpr int kLdsMaxN = 2048;
constexpr int kLdsMaxPasses = 6;

struct XfPlan {
    int N, np;
    int lgr[kLdsMaxPasses];  // log2 radix of pass q
    int sh[kLdsMaxPasses];   // log2 s_q = log2(N / (R_0 ... R_q))
    int tw[kLdsMaxPasses];   // pass q's twiddles in the LDS table: entry
                             // j R_q + u = w_{L_q}^{+-j u}, j < s_q
};

// x[t] of a transform lives at pos(t) (DIF output / DIT input order)
__device__ __forceinline__ int xf_pos(const XfPlan& P, int t)
{
    int p = 0;
    for (int q = 0; q < P.np; q++) {
        p += (t & ((1 << P.lgr[q]) - 1)) << P.sh[q];
        t >>= P.lgr[q];
    }
    return p;
}
__device__ __forceinline__ int ilog2_dev(int n)
{
    return 31 - __builtin_clz(static_cast<unsigned>(n));
}
__device__ __forceinline__ int xf_index(const XfPlan& P, int p)
{
    int t = 0, b = 0;
    for (int q = 0; q < P.np; q++) {
        t += ((p >> P.sh[q]) & ((1 << P.lgr[q]) - 1)) << b;
        b += P.lgr[q];
    }
    return t;
}

// Image row of transform position p: one empty row after every 32.  A
// wave holds 64 / T tasks of a pass; in the short-stride passes (the unit
// pass: 32 consecutive positions per task) those tasks sat 32 T words
// apart, i.e. on the same banks (k1000 encode: 72 % of the LDS cycles were
// bank conflicts); one row per 32 moves task tt by tt T banks.  A pass
// task's positions b + j + q s (b a multiple of 32 or the task inside one
// aligned 32-block, j < s) never carry into bit 5, so
// prow(b + j + q s) = prow(b + j) + prow(q s): a per-task base plus a
// per-q uniform offset, as before.
__host__ __device__ __forceinline__ int prow(int p)
{
    return p + (p >> 5);
}

enum : int { kLdsEnc = 0, kLdsSysEnc = 1, kLdsDec = 2, kLdsSysDec = 3 };

struct NttLdsArgs {
    int mode;
    int k, n, len2k, nmax;
    int lgT, tiles;
    long long words;
    // NTT_n / INTT_n / NTT_2k / INTT_2k: geometry + pass table offsets
    XfPlan pnf, pni, p2f, p2i;  // p2f / p2i: NTT_h / INTT_h, h = len_2k / 2
    int twist;          // w2k^t, then w2k^-t (t < h), in the table range
    const int32_t* tw;  // the pass twiddle tables (qi_plan::d_ldstw)
    int tw_words;
    RowSrc src;         // enc: data rows by position; dec: received rows
    const int32_t* ctx; // decode context (sys encode: the plan's, cs = 0)
    long long cs;
    int ids_off, c_off, pos_off;
    Oor in_oor;
    int slot_base;
    uint16_t* out;      // output row r of stripe s at out + s*oss + r*ors
    long long oss, ors;
    int out_first, out_rows;  // sequence index of output row 0, row count
    Oor out_oor;
    uint32_t* err;
    int wide;  // 16-byte row pieces: every row base and stride 8-word
               // aligned and words % 8 == 0 (lds_launch checks)
    // erasure decode (ntt_eras_kernel): e erased positions, their list and
    // the e x e solve in the context, n^-1 (balanced)
    int eras_e, eras_eid, eras_b;
    int32_t inv_n;
    const int32_t* rinv;  // w_32^-x, x < 32 (d_ldstw tail): w_R^-x for every radix R
};

// One pass over the image: tasks (group start b, offset j < s) of the R
// positions b + j + q s, lane = column.  DIF: codelet, then output u times
// w_L^{j u}; DIT: input q times w_L^{+-j q}, then codelet.  A task's
// twiddles are contiguous in the pass table (vector LDS reads) and its R
// elements sit at one base plus loop-invariant strides.
// UNIT: the s = 1 pass, whose twiddles w_L^{0 u} are all 1 (no table reads,
// no multiplies).  Optional output scale (the decode's x C, fused into the
// last DIF pass of NTT_2k): element u of task tt sits at position tt R + u,
// i.e. holds X[xf_index(tt R) + (u << cb)], times cm[that] (canonical when
// CANON, else balanced).
template <int R, bool DIF, bool INV, bool UNIT, bool CANON>
__device__ __forceinline__ void lds_pass_body(int32_t* buf, const int32_t* twp, int N, int lgs,
                                              int lgL, int lgT, int col, int g, int G,
                                              const int32_t* cm, int cb, const XfPlan* cp,
                                              int lgnb)
{
    const int lgtasks = ilog2_dev(N) - ilog2_dev(R);
    for (int t2 = g; t2 < (1 << (lgtasks + lgnb)); t2 += G) {
        // transform bi of the batch (at image row bi N), its task tt
        const int bi = t2 >> lgtasks, tt = t2 & ((1 << lgtasks) - 1);
        const int j = UNIT ? 0 : tt & ((1 << lgs) - 1);
        const int lb = (prow(bi * N + ((tt >> lgs) << lgL) + j) << lgT) + col;
        const int32_t* tj = twp + j * R;
        int32_t v[R], w[R];
#pragma unroll
        for (int q = 0; q < R; q++) {
            v[q] = buf[lb + (prow(q << lgs) << lgT)];
            if (!UNIT)
                w[q] = tj[q];
        }
        if (!DIF && !UNIT) {
#pragma unroll
            for (int q = 1; q < R; q++)
                v[q] = mul_rt(v[q], w[q]);
        }
        dft<R, kInLo, kInHi>(v);
        int ci0 = 0;
        if (UNIT && DIF && cm)
            ci0 = xf_index(*cp, tt * R);
#pragma unroll
        for (int u = 0; u < R; u++) {
            int32_t y = v[INV ? (R - u) % R : u];
            if (DIF && !UNIT && u > 0)
                y = mul_rt(y, w[u]);
            if (UNIT && DIF && cm) {
                const int32_t c = cm[((ci0 + (u << cb)) << lgnb) + bi];
                y = mul_rt(y, CANON ? balanced(static_cast<uint32_t>(c)) : c);
            }
            buf[lb + (prow(u << lgs) << lgT)] = y;
        }
    }
}

template <int R, bool DIF, bool INV, bool CANON>
__device__ __forceinline__ void lds_pass(int32_t* buf, const int32_t* twp, int N, int lgs,
                                         int lgL, int lgT, int col, int g, int G,
                                         const int32_t* cm, int cb, const XfPlan* cp, int lgnb)
{
    if (lgs == 0)
        lds_pass_body<R, DIF, INV, true, CANON>(buf, twp, N, lgs, lgL, lgT, col, g, G, cm, cb,
                                                cp, lgnb);
    else
        lds_pass_body<R, DIF, INV, false, CANON>(buf, twp, N, lgs, lgL, lgT, col, g, G,
                                                 nullptr, 0, cp, lgnb);
}

// cm (DIF only): the output scale of the last (s = 1) pass, indexed by the
// natural output index (see lds_pass_body).  2^lgnb transforms of P.N
// points back to back (image rows bi N ..), the same passes over all: the
// scale of output m of transform bi is cm[(m << lgnb) + bi].
template <bool DIF, bool INV, bool CANON = false>
__device__ void lds_transform(int32_t* buf, const int32_t* tw, const XfPlan& P, int lgT,
                              int col, int g, int G, const int32_t* cm = nullptr, int lgnb = 0)
{
    const int cb = P.N == 1 ? 0 : ilog2_dev(P.N) - P.lgr[P.np - 1];
    for (int i = 0; i < P.np; i++) {
        const int q = DIF ? i : P.np - 1 - i;  // DIT: the passes in reverse
        const int lgs = P.sh[q], lgL = lgs + P.lgr[q];
        const int32_t* twp = tw + P.tw[q];
        const int32_t* c = DIF && i == P.np - 1 ? cm : nullptr;
        switch (P.lgr[q]) {
        case 1:
            lds_pass<2, DIF, INV, CANON>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, c, cb, &P,
                                           lgnb);
            break;
        case 2:
            lds_pass<4, DIF, INV, CANON>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, c, cb, &P,
                                           lgnb);
            break;
        case 3:
            lds_pass<8, DIF, INV, CANON>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, c, cb, &P,
                                           lgnb);
            break;
        case 4:
            lds_pass<16, DIF, INV, CANON>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, c, cb, &P,
                                           lgnb);
            break;
        default:
            lds_pass<32, DIF, INV, CANON>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, c, cb, &P,
                                           lgnb);
            break;
        }
        __syncthreads();
    }
}

// LDS side arrays behind the nmax x T image (int32 words)
__host__ __device__ inline int lds_side_words(int tw_words, int k, int len2k, bool twg)
{
    return twg ? 2 * k : tw_words + 2 * k + len2k;
}

constexpr int kLdsBatch = 8;  // row loads in flight per thread

// TWG: the pass twiddle tables and C are read from global memory (L1/L2
// hits) instead of being staged in LDS, so that two workgroups fit a CU
// where the staged tables would leave room for one (lds_geom; k1000 decode:
// 64 KB image + 8 KB of ids / inv_A instead of + 38 KB).  Staging the pass
// tables again with ids / inv_A in the image rows INTT_n leaves free (two
// workgroups per CU, twist and C from global) measured slower: k1000 decode
// 5.21 -> 5.45 ms (gpurun_out ntt6)
template <bool TWG>
__global__ __launch_bounds__(kLdsThreads) void ntt_lds_kernel(NttLdsArgs a)
{
    extern __shared__ int32_t qi_ntt_lds[];
    const int nmax = a.nmax, lgT = a.lgT, T = 1 << lgT, k = a.k;
    int32_t* buf = qi_ntt_lds;
    int32_t* tw_l = qi_ntt_lds + (prow(nmax) << lgT);  // pass twiddle tables
    const int32_t* tw = TWG ? a.tw : tw_l;
    int32_t* s_inv = TWG ? tw_l : tw_l + a.tw_words;  // inv_A_i (balanced)
    int32_t* s_id = s_inv + k;                 // received ids z_i
    int32_t* s_c = s_id + k;                   // C[j] (balanced), natural order
    // XCD-aware map: workgroups go round-robin over the 8 XCDs (b % 8), and
    // a tile is only T = 8..64 columns (16..128 bytes of a row), so in
    // stripe-major order the tiles sharing a 128-byte line ran on different
    // XCDs (each L2 fetching and partially writing the same lines).  XCD x
    // walks the contiguous eighth x of the (stripe, tile) order instead.
    int b = blockIdx.x;
    if ((gridDim.x & 7) == 0)
        b = (b & 7) * static_cast<int>(gridDim.x >> 3) + (b >> 3);
    const int s = b / a.tiles;
    const long long c0 = static_cast<long long>(b - s * a.tiles) << lgT;
    const int tid = threadIdx.x, col = tid & (T - 1), g = tid >> lgT, G = kLdsThreads >> lgT;
    const long long cg = c0 + col;
    const bool valid = cg < a.words;
    const bool dec = a.mode != kLdsEnc;
    // every per-stripe constant into LDS first (one round of independent
    // loads), so the hot loops below wait on nothing but their row loads
    const int32_t* ctx = a.ctx + s * a.cs;
    if (!TWG)
        for (int e = tid; e < a.tw_words; e += kLdsThreads)
            tw_l[e] = a.tw[e];
    if (dec) {
        for (int i = tid; i < k; i += kLdsThreads) {
            s_inv[i] = balanced(static_cast<uint32_t>(ctx[i]));
            s_id[i] = ctx[a.ids_off + i];
        }
        if (!TWG)
            for (int j = tid; j < a.len2k; j += kLdsThreads)
                s_c[j] = balanced(static_cast<uint32_t>(ctx[a.c_off + j]));
    }
    const RowSrc& src = a.src;
    auto row_ptr = [&](int id) {
        return id < src.split ? src.base0 + s * src.ss0 + id * src.rs0
                              : src.base1 + s * src.ss1 + (id - src.split) * src.rs1;
    };
    // wide row pieces: lane (rl, cj) moves columns 8 cj .. 8 cj + 7 of a
    // row as one 16-byte access (a wave covers 64 / LPR rows); otherwise a
    // lane moves one u16 column and a wave 64 / T rows of T columns, i.e.
    // 16..128-byte pieces per wave instruction and few bytes in flight
    const int lgL = lgT - 3, rl = tid >> lgL, cj = tid & ((1 << lgL) - 1);
    const int RPP = kLdsThreads >> lgL;  // rows per sweep
    const long long cw = c0 + 8 * cj;    // first column of the lane's piece
    const bool wvalid = cw < a.words;
    auto ld_piece = [&](int id) {
        const uint16_t* r = row_ptr(id) + cw;
        return *reinterpret_cast<const uint4*>(r);
    };
    // 8 u16 (a uint4) -> int32 words at image row p, columns 8 cj ..
    auto put_piece = [&](int p, uint4 x, int32_t scale, bool sc) {
        int4 lo, hi;
        const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
        int32_t e[8];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            e[2 * q] = static_cast<int32_t>(xs[q] & 0xffffu);
            e[2 * q + 1] = static_cast<int32_t>(xs[q] >> 16);
        }
        if (sc) {
#pragma unroll
            for (int q = 0; q < 8; q++)
                e[q] = mul_rt(e[q], scale);
        }
        lo = int4{e[0], e[1], e[2], e[3]};
        hi = int4{e[4], e[5], e[6], e[7]};
        int4* d = reinterpret_cast<int4*>(buf + (prow(p) << lgT) + 8 * cj);
        d[0] = lo;
        d[1] = hi;
    };
    if (!dec && a.wide) {
        // data rows t < k at natural positions, zero above (DIF input)
        for (int p0 = rl; p0 < a.n; p0 += RPP * kLdsBatch) {
            uint4 x[kLdsBatch];
#pragma unroll
            for (int u = 0; u < kLdsBatch; u++) {
                const int p = p0 + u * RPP;
                x[u] = (p < k && wvalid) ? ld_piece(p) : uint4{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < kLdsBatch; u++) {
                const int p = p0 + u * RPP;
                if (p < a.n)
                    put_piece(p, x[u], 0, false);
            }
        }
        __syncthreads();
        lds_transform<true, false>(buf, tw, a.pnf, lgT, col, g, G);
    } else if (!dec) {
        // data rows t < k at natural positions, zero above (DIF input);
        // kLdsBatch row loads in flight per thread
        for (int p0 = g; p0 < a.n; p0 += G * kLdsBatch) {
            int32_t x[kLdsBatch];
#pragma unroll
            for (int u = 0; u < kLdsBatch; u++) {
                const int p = p0 + u * G;
                x[u] = (p < k && valid) ? row_ptr(p)[cg] : 0;
            }
#pragma unroll
            for (int u = 0; u < kLdsBatch; u++) {
                const int p = p0 + u * G;
                if (p < a.n)
                    buf[(prow(p) << lgT) + col] = x[u];
            }
        }
        __syncthreads();
        lds_transform<true, false>(buf, tw, a.pnf, lgT, col, g, G);
    } else {
        // INTT_n input (DIT order): zero, then y_i = v_i inv_A_i at pos_n(z_i)
        for (int p = g; p < a.n; p += G)
            buf[(prow(p) << lgT) + col] = 0;
        __syncthreads();
        if (a.wide) {
            for (int i0 = rl; i0 < k; i0 += RPP * kLdsBatch) {
                uint4 x[kLdsBatch];
#pragma unroll
                for (int u = 0; u < kLdsBatch; u++) {
                    const int i = i0 + u * RPP;
                    x[u] = (i < k && wvalid) ? ld_piece(src.by_pos ? i : s_id[i])
                                             : uint4{0, 0, 0, 0};
                }
#pragma unroll
                for (int u = 0; u < kLdsBatch; u++) {
                    const int i = i0 + u * RPP;
                    if (i < k)
                        put_piece(xf_pos(a.pnf, s_id[i]), x[u], s_inv[i], true);
                }
            }
        } else
        for (int i0 = g; i0 < k; i0 += G * kLdsBatch) {
            int32_t x[kLdsBatch];
#pragma unroll
            for (int u = 0; u < kLdsBatch; u++) {
                const int i = i0 + u * G;
                x[u] = 0;
                if (i < k && valid)
                    x[u] = row_ptr(src.by_pos ? i : s_id[i])[cg];
            }
#pragma unroll
            for (int u = 0; u < kLdsBatch; u++) {
                const int i = i0 + u * G;
                if (i < k)
                    buf[(prow(xf_pos(a.pnf, s_id[i])) << lgT) + col] = mul_rt(x[u], s_inv[i]);
            }
        }
        __syncthreads();
        if (a.in_oor.counts) {
            // decode_prepare (src/fec_base.h:1361-1404): a marked symbol is
            // 65536 = -1, so y = -inv_A_i at the marks inside this tile
            for (int i = tid; i < k; i += kLdsThreads) {
                const int id = s_id[i];  // sequence index z_i
                const int slot = src.by_pos ? i : id - a.slot_base;
                if (slot < 0)
                    continue;  // systematic data row: no marks
                const long long bk = static_cast<long long>(s) * a.in_oor.slots + slot;
                uint32_t cnt = a.in_oor.counts[bk];
                if (cnt > static_cast<uint32_t>(a.in_oor.cap)) {
                    atomicOr(a.err, kErrOorTruncated);
                    cnt = static_cast<uint32_t>(a.in_oor.cap);
                }
                const int p = xf_pos(a.pnf, id);
                const int32_t y = -s_inv[i];  // -inv_A_i, balanced
                for (uint32_t e = 0; e < cnt; e++) {
                    const long long c = static_cast<long long>(
                                            a.in_oor.entries[bk * a.in_oor.cap + e]) - c0;
                    if (c >= 0 && c < T)
                        buf[(prow(p) << lgT) + static_cast<int>(c)] = y;
                }
            }
            __syncthreads();
        }
        lds_transform<false, true>(buf, tw, a.pni, lgT, col, g, G);
        // NTT_2k of the first k outputs (zero from k, k <= h = len_2k / 2),
        // x C, INTT_2k, split in halves (no pass touches the zero half):
        //   X[2m] = NTT_h(x)[m],  X[2m+1] = NTT_h(x_t w2k^t)[m]
        //   y_t = INTT_h(Y_even)[t] + w2k^-t INTT_h(Y_odd)[t]   (t < k)
        // rows [0, h) hold the even transform, rows [h, 2h) the odd one
        const int h = a.len2k >> 1;
        const int32_t* twist = tw + a.twist;
        for (int t = g; t < h; t += G) {
            const int32_t x = t < k ? buf[(prow(t) << lgT) + col] : 0;
            buf[(prow(t) << lgT) + col] = x;
            buf[(prow(h + t) << lgT) + col] = t < k ? mul_rt(x, twist[t]) : 0;
        }
        __syncthreads();
        // both NTT_h (DIF) at once, times C[2m + bi] in the last pass
        if (TWG)
            lds_transform<true, false, true>(buf, tw, a.p2f, lgT, col, g, G, ctx + a.c_off, 1);
        else
            lds_transform<true, false, false>(buf, tw, a.p2f, lgT, col, g, G, s_c, 1);
        lds_transform<false, true>(buf, tw, a.p2i, lgT, col, g, G, nullptr, 1);
        for (int t = g; t < k; t += G) {
            const int32_t e = buf[(prow(t) << lgT) + col];
            const int32_t o = mul_rt(buf[(prow(h + t) << lgT) + col], twist[h + t]);
            buf[(prow(t) << lgT) + col] = fold(e + o);  // [-65538, 131072] -> V range
        }
        __syncthreads();
        if (a.mode != kLdsDec) {
            // systematic: evaluate the coefficients at r^t (NTT_n, DIF)
            for (int p = k + g; p < a.n; p += G)
                buf[(prow(p) << lgT) + col] = 0;
            __syncthreads();
            lds_transform<true, false>(buf, tw, a.pnf, lgT, col, g, G);
        }
    }
    // output rows: sequence index t = out_first + r, at position t (DIT
    // output: natural order) or pos_n(t) (DIF output)
    const bool natural = a.mode == kLdsDec;
    if (a.wide) {
        if (!wvalid)
            return;
        for (int r = rl; r < a.out_rows; r += RPP) {
            const int t = a.out_first + r;
            const int p = natural ? t : xf_pos(a.pnf, t);
            const int4* sp = reinterpret_cast<const int4*>(buf + (prow(p) << lgT) + 8 * cj);
            const int4 lo = sp[0], hi = sp[1];
            const int32_t e[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
            uint32_t cv[8];
            bool any = false;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                cv[q] = canon_vr(e[q]);
                any |= cv[q] == 65536u;
            }
            uint4 o;
            o.x = (cv[0] & 0xffffu) | (cv[1] << 16);
            o.y = (cv[2] & 0xffffu) | (cv[3] << 16);
            o.z = (cv[4] & 0xffffu) | (cv[5] << 16);
            o.w = (cv[6] & 0xffffu) | (cv[7] << 16);
            *reinterpret_cast<uint4*>(a.out + s * a.oss + r * a.ors + cw) = o;
            if (any && a.out_oor.counts) {
                const long long bk = static_cast<long long>(s) * a.out_oor.slots + r;
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    if (cv[q] == 65536u) {
                        const uint32_t en = atomicAdd(&a.out_oor.counts[bk], 1u);
                        if (en < static_cast<uint32_t>(a.out_oor.cap))
                            a.out_oor.entries[bk * a.out_oor.cap + en] =
                                static_cast<uint32_t>(cw + q);
                    }
                }
            }
        }
        return;
    }
    if (!valid)
        return;
    for (int r = g; r < a.out_rows; r += G) {
        const int t = a.out_first + r;
        const int p = natural ? t : xf_pos(a.pnf, t);
        const uint32_t cv = canon_vr(buf[(prow(p) << lgT) + col]);
        a.out[s * a.oss + r * a.ors + cg] = static_cast<uint16_t>(cv);
        if (cv == 65536u && a.out_oor.counts) {
            const long long bk = static_cast<long long>(s) * a.out_oor.slots + r;
            const uint32_t e = atomicAdd(&a.out_oor.counts[bk], 1u);
            if (e < static_cast<uint32_t>(a.out_oor.cap))
                a.out_oor.entries[bk * a.out_oor.cap + e] = static_cast<uint32_t>(cg);
        }
    }
}

// INTT_n (DIT, as lds_transform<false, true>) computing only the outputs
// t >= k (the erasure decode's syndromes): every pass but the last as usual,
// then the last pass (q = 0: tasks j < s, positions j + u s) evaluates just
// the outputs u >= ceil((k - j) / s) of its R-point inverse DFT directly
// (y_u = sum_q v'_q w_R^-qu with the twiddled inputs v'; a handful per task)
// instead of the whole codelet.  rinv: w_32^-x, x < 32, balanced (w_R^-x =
// w_32^(-x 32 / R) for the pass's radix R = 2^lgr[0]).
// With syn (e x T, row t - k) the outputs go there and the image keeps the
// state after the other passes (the two-pass decode completes the transform
// from it); otherwise into the image rows t.
__device__ void lds_intt_top(int32_t* buf, const int32_t* tw, const XfPlan& P, int lgT, int col,
                             int g, int G, int k, const int32_t* rinv, int32_t* syn)
{
    for (int i = 0; i + 1 < P.np; i++) {
        const int q = P.np - 1 - i;
        const int lgs = P.sh[q], lgL = lgs + P.lgr[q];
        const int32_t* twp = tw + P.tw[q];
        switch (P.lgr[q]) {
        case 1:
            lds_pass<2, false, true, false>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, nullptr, 0,
                                            &P, 0);
            break;
        case 2:
            lds_pass<4, false, true, false>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, nullptr, 0,
                                            &P, 0);
            break;
        case 3:
            lds_pass<8, false, true, false>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, nullptr, 0,
                                            &P, 0);
            break;
        case 4:
            lds_pass<16, false, true, false>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, nullptr,
                                             0, &P, 0);
            break;
        default:
            lds_pass<32, false, true, false>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, nullptr,
                                             0, &P, 0);
            break;
        }
        __syncthreads();
    }
    const int lgR = P.lgr[0], R = 1 << lgR, lgs = P.sh[0], sN = 1 << lgs;
    const int32_t* twp = tw + P.tw[0];
    for (int j = g; j < sN; j += G) {
        const int umin = k > j ? (k - j + sN - 1) >> lgs : 0;
        if (umin >= R)
            continue;
        const int lb = (prow(j) << lgT) + col;
        int32_t v[32];
#pragma unroll
        for (int q = 0; q < 32; q++) {
            if (q < R) {
                v[q] = buf[lb + (prow(q << lgs) << lgT)];
                if (q > 0 && lgs > 0)
                    v[q] = mul_rt(v[q], twp[j * R + q]);
            }
        }
        for (int u = umin; u < R; u++) {
            int32_t acc = v[0];  // |acc| <= 32 * 65540
#pragma unroll
            for (int q = 1; q < 32; q++)
                if (q < R)
                    acc += mul_rt(v[q], rinv[((q * u) << (5 - lgR)) & 31]);
            // output t = j + u s >= k: into syn (row t - k) when given,
            // leaving the image as the passes before the last left it
            if (syn)
                syn[(((j + (u << lgs)) - k) << lgT) + col] = fold(fold(acc));
            else
                buf[lb + (prow(u << lgs) << lgT)] = fold(fold(acc));
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// Erasure decode (plans with few erasures: e = n - k <= kErasMax, n <= 2048,
// eras_plan).  The codeword of both types is c_j = P(r^j), deg P < k, over
// all n positions (those >= k + m are never sent); a stripe receives k of
// them and misses the e positions E.  The unnormalised INTT_n of the
// zero-filled codeword, y', holds e "syndromes" in its top outputs
// (y'_t = -sum_{j in E} c_j r^-jt for t >= k, where the true coefficients
// vanish), and with x_j = r^-E_j the erased symbols solve a transposed
// Vandermonde system:
//     c_E = B y'_[k, n),   B[j][u] = -r^(E_j k) coef_u(L_j),
//     L_j = prod_{l != j} (X - x_l) / (x_j - x_l)          (per pattern)
// Then the systematic outputs ARE codeword symbols (received rows copied,
// erased ones from c_E), and the non-systematic coefficients are one more
// INTT_n of the completed codeword times n^-1.  So a decode is 1 or 2
// n-point transforms + e^2 multiply-adds per column instead of decode_apply's
// INTT_n + NTT_2k + INTT_2k (+ NTT_n) (src/fec_base.h:1418-1448), the same
// outputs (the interpolation is unique), on an n-row image; the systematic
// encode is the same solve with E = [k, n) (the plan's constant context).
// The math is emulated in tests/test_ntt_plan.py::test_erasure_decode_math.
// ---------------------------------------------------------------------------
constexpr int kErasMax = 64;

struct ErasCtxLayout {
    int k, n, e;
    __host__ __device__ long long ids_off() const { return 0; }
    __host__ __device__ long long pos_off() const { return k; }  // id -> i, or -1 - j (erased)
    __host__ __device__ long long eid_off() const { return static_cast<long long>(k) + n; }
    __host__ __device__ long long b_off() const { return eid_off() + e; }
    __host__ __device__ long long words() const { return b_off() + static_cast<long long>(e) * e; }
};

struct ErasCtxArgs {
    ErasCtxLayout L;
    uint32_t r, rinv;     // n-th root of unity and its inverse
    const uint16_t* ids;  // S x k received ids, ascending (nullptr: 0 .. k-1)
    int32_t* ctx;
    long long cs;
    uint32_t* err;        // the plan's sticky error word (kErrBadIds)
};

// One wave per stripe: the received bitmap, the erased list E (ascending),
// x_j = r^-E_j, A(X) = prod (X - x_j) with lane d on coefficient d (the
// monic top coefficient stays implicit), then lane j's synthetic division
// Q_j = A / (X - x_j) into LDS and A'(x_j) = Q_j(x_j) beside it, and row j
// of B.  O(e^2) per stripe, e <= 64.
__global__ __launch_bounds__(64) void eras_ctx_kernel(ErasCtxArgs a)
{
    __shared__ uint32_t bm[kLdsMaxN / 32];
    __shared__ int32_t eid[kErasMax];
    __shared__ uint32_t W[kErasMax * kErasMax];
    const int s = blockIdx.x, lane = threadIdx.x;
    const int k = a.L.k, n = a.L.n, e = a.L.e, nw = n >> 5;
    int32_t* ctx = a.ctx + s * a.cs;
    int32_t* ids = ctx + a.L.ids_off();
    int32_t* pos = ctx + a.L.pos_off();
    const uint16_t* sid = a.ids ? a.ids + static_cast<long long>(s) * k : nullptr;
    for (int w = lane; w < nw; w += 64)
        bm[w] = 0;
    __syncthreads();
    // ids must be distinct and < n: an id past n is dropped and a repeated
    // one leaves more than e positions missing; either way nothing is
    // written outside this stripe's context (the E list keeps its first e
    // entries) and the plan's sticky error is raised
    bool bad = false;
    for (int i = lane; i < k; i += 64) {
        const int id = sid ? sid[i] : i;
        ids[i] = id;
        if (id < n) {
            pos[id] = i;
            atomicOr(&bm[id >> 5], 1u << (id & 31));
        } else {
            bad = true;
        }
    }
    __syncthreads();
    // erased positions in ascending order: lane w takes bitmap word w (at
    // most 64 words), its slot offset from an exclusive scan of the counts
    uint32_t miss = lane < nw ? ~bm[lane] : 0u;
    int cnt = __popc(miss), off = cnt;
    for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(off, d);
        if (lane >= d)
            off += v;
    }
    off -= cnt;
    while (miss) {
        const int b = __ffs(miss) - 1;
        miss &= miss - 1;
        const int t = lane * 32 + b;
        if (off < e) {
            eid[off] = t;
            ctx[a.L.eid_off() + off] = t;
            pos[t] = -1 - off;
        } else {
            bad = true;
        }
        off++;
    }
    if (__builtin_amdgcn_ballot_w64(bad) && lane == 0)
        atomicOr(a.err, kErrBadIds);
    __syncthreads();
    const uint32_t xj = lane < e ? powm_(a.rinv, static_cast<uint32_t>(eid[lane])) : 0u;
    uint32_t ad = lane == 0 ? 1u : 0u;  // A, coefficient `lane`
    for (int j = 0; j < e; j++) {
        const uint32_t x = __builtin_amdgcn_readlane(xj, j);
        uint32_t prev = __shfl_up(ad, 1);
        prev = lane == 0 ? 0u : prev;
        ad = subm_(prev, mulm_(x, ad));
    }
    uint32_t q = 1, h = 1;  // q_{e-1} = 1 (A monic); Horner of Q_j at x_j
    if (lane < e)
        W[lane * kErasMax + e - 1] = 1;
    for (int t = e - 1; t >= 1; t--) {
        const uint32_t at = __builtin_amdgcn_readlane(ad, t);
        q = addm_(at, mulm_(xj, q));
        h = addm_(mulm_(h, xj), q);
        if (lane < e)
            W[lane * kErasMax + t - 1] = q;
    }
    if (lane < e) {
        // f_j = -r^(E_j k) / A'(x_j)
        const uint32_t rk = powm_(a.r, static_cast<uint32_t>(
                                           (static_cast<long long>(eid[lane]) * k) % n));
        const uint32_t f = subm_(0u, mulm_(rk, powm_(h, 65535u)));
        int32_t* B = ctx + a.L.b_off() + static_cast<long long>(lane) * e;
        for (int u = 0; u < e; u++)
            B[u] = balanced(mulm_(f, W[lane * kErasMax + u]));
    }
}

// The erasure decode of a tile of T columns of one stripe (and the
// systematic encode, E = [k, n)), in LDS: image n x T, then the tables
// (unless TWG), ids, the position map, E, B and c_E (e x T).
// C2: the non-systematic decode of a two-pass INTT_n (np = 2), completed
// from the image (see below); otherwise the second load + INTT_n.  Separate
// instantiations: one kernel holding both completions kept more registers
// live (150 VGPRs, 3 waves per SIMD: one 512-thread block per CU).
template <bool TWG, bool C2>
__global__ __launch_bounds__(kLdsThreads) void ntt_eras_kernel(NttLdsArgs a)
{
    extern __shared__ int32_t qi_ntt_lds[];
    const int n = a.n, lgT = a.lgT, T = 1 << lgT, k = a.k, e = a.eras_e;
    int32_t* buf = qi_ntt_lds;
    int32_t* tw_l = buf + (prow(n) << lgT);
    const int32_t* tw = TWG ? a.tw : tw_l;
    int32_t* s_id = TWG ? tw_l : tw_l + a.tw_words;
    int32_t* s_pos = s_id + k;  // C2: e x T words of syndromes instead
    int32_t* s_eid = s_pos + (C2 ? (e << lgT) : n);
    int32_t* s_B = s_eid + e;
    int32_t* s_cE = s_B + e * e;
    int32_t* s_rinv = s_cE + (e << lgT);  // w_32^-x (INTT_n's passes' inverse roots)
    // C2: the syndromes y'_[k, n) (e x T <= n words, eras_launch) in the
    // position map's place (a non-systematic decode reads it no more)
    int32_t* s_syn = C2 ? s_pos : nullptr;
    int b = blockIdx.x;  // XCD-contiguous tiles, as ntt_lds_kernel
    if ((gridDim.x & 7) == 0)
        b = (b & 7) * static_cast<int>(gridDim.x >> 3) + (b >> 3);
    const int s = b / a.tiles;
    const long long c0 = static_cast<long long>(b - s * a.tiles) << lgT;
    const int tid = threadIdx.x, col = tid & (T - 1), g = tid >> lgT, G = kLdsThreads >> lgT;
    const long long cg = c0 + col;
    const bool valid = cg < a.words;
    const int32_t* ctx = a.ctx + s * a.cs;
    if (!TWG)
        for (int i = tid; i < a.tw_words; i += kLdsThreads)
            tw_l[i] = a.tw[i];
    for (int i = tid; i < k; i += kLdsThreads)
        s_id[i] = ctx[a.ids_off + i];
    if (!C2)
        for (int t = tid; t < n; t += kLdsThreads)
            s_pos[t] = ctx[a.pos_off + t];
    for (int j = tid; j < e; j += kLdsThreads)
        s_eid[j] = ctx[a.eras_eid + j];
    for (int i = tid; i < e * e; i += kLdsThreads)
        s_B[i] = ctx[a.eras_b + i];
    if (tid < 32)
        s_rinv[tid] = a.rinv[tid];
    __syncthreads();
    const RowSrc& src = a.src;
    auto row_ptr = [&](int id) {
        return id < src.split ? src.base0 + s * src.ss0 + id * src.rs0
                              : src.base1 + s * src.ss1 + (id - src.split) * src.rs1;
    };
    const int lgL = lgT - 3, rl = tid >> lgL, cj = tid & ((1 << lgL) - 1);
    const int RPP = kLdsThreads >> lgL;
    const long long cw = c0 + 8 * cj;
    const bool wvalid = cw < a.words;
    // the received rows at pos(id) (+ c_E at pos(E_j) when `fill`), the
    // marked symbols as 65536 = -1 (decode_prepare, src/fec_base.h:1361-1404)
    auto load = [&](bool fill) {
        if (a.wide) {
            for (int i0 = rl; i0 < k; i0 += RPP * kLdsBatch) {
                uint4 x[kLdsBatch];
#pragma unroll
                for (int u = 0; u < kLdsBatch; u++) {
                    const int i = i0 + u * RPP;
                    x[u] = (i < k && wvalid) ? *reinterpret_cast<const uint4*>(
                                                   row_ptr(src.by_pos ? i : s_id[i]) + cw)
                                             : uint4{0, 0, 0, 0};
                }
#pragma unroll
                for (int u = 0; u < kLdsBatch; u++) {
                    const int i = i0 + u * RPP;
                    if (i < k) {
                        const uint32_t xs[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
                        int4* d = reinterpret_cast<int4*>(
                            buf + (prow(xf_pos(a.pni, s_id[i])) << lgT) + 8 * cj);
                        d[0] = int4{static_cast<int32_t>(xs[0] & 0xffffu),
                                    static_cast<int32_t>(xs[0] >> 16),
                                    static_cast<int32_t>(xs[1] & 0xffffu),
                                    static_cast<int32_t>(xs[1] >> 16)};
                        d[1] = int4{static_cast<int32_t>(xs[2] & 0xffffu),
                                    static_cast<int32_t>(xs[2] >> 16),
                                    static_cast<int32_t>(xs[3] & 0xffffu),
                                    static_cast<int32_t>(xs[3] >> 16)};
                    }
                }
            }
        } else {
            for (int i0 = g; i0 < k; i0 += G * kLdsBatch) {
                int32_t x[kLdsBatch];
#pragma unroll
                for (int u = 0; u < kLdsBatch; u++) {
                    const int i = i0 + u * G;
                    x[u] = (i < k && valid) ? row_ptr(src.by_pos ? i : s_id[i])[cg] : 0;
                }
#pragma unroll
                for (int u = 0; u < kLdsBatch; u++) {
                    const int i = i0 + u * G;
                    if (i < k)
                        buf[(prow(xf_pos(a.pni, s_id[i])) << lgT) + col] = x[u];
                }
            }
        }
        for (int it = tid; it < (e << lgT); it += kLdsThreads) {
            const int j = it >> lgT, c = it & (T - 1);
            buf[(prow(xf_pos(a.pni, s_eid[j])) << lgT) + c] = fill ? s_cE[it] : 0;
        }
        __syncthreads();
        if (a.in_oor.counts) {
            for (int i = tid; i < k; i += kLdsThreads) {
                const int id = s_id[i];
                const int slot = src.by_pos ? i : id - a.slot_base;
                if (slot < 0)
                    continue;  // systematic data row: no marks
                const long long bk = static_cast<long long>(s) * a.in_oor.slots + slot;
                uint32_t cnt = a.in_oor.counts[bk];
                if (cnt > static_cast<uint32_t>(a.in_oor.cap)) {
                    atomicOr(a.err, kErrOorTruncated);
                    cnt = static_cast<uint32_t>(a.in_oor.cap);
                }
                const int p = xf_pos(a.pni, id);
                for (uint32_t f = 0; f < cnt; f++) {
                    const long long c = static_cast<long long>(
                                            a.in_oor.entries[bk * a.in_oor.cap + f]) - c0;
                    if (c >= 0 && c < T)
                        buf[(prow(p) << lgT) + static_cast<int>(c)] = -1;
                }
            }
            __syncthreads();
        }
    };
    load(false);
    // only the syndromes y'_[k, n) are needed from this transform
    lds_intt_top(buf, tw, a.pni, lgT, col, g, G, k, s_rinv, s_syn);
    // c_E = B y'_[k, n): e lazy products per (erasure, column) item
    for (int it = tid; it < (e << lgT); it += kLdsThreads) {
        const int j = it >> lgT, c = it & (T - 1);
        const int32_t* Bj = s_B + j * e;
        int32_t acc = 0;  // |acc| <= 64 * 65536
        for (int u = 0; u < e; u++)
            acc += mul_rt(C2 ? s_syn[(u << lgT) + c] : buf[(prow(k + u) << lgT) + c], Bj[u]);
        s_cE[it] = fold(fold(acc));  // [-1, 65536]
    }
    __syncthreads();
    auto store8 = [&](uint16_t* o, const uint32_t (&cv)[8]) {
        uint4 v;
        v.x = (cv[0] & 0xffffu) | (cv[1] << 16);
        v.y = (cv[2] & 0xffffu) | (cv[3] << 16);
        v.z = (cv[4] & 0xffffu) | (cv[5] << 16);
        v.w = (cv[6] & 0xffffu) | (cv[7] << 16);
        *reinterpret_cast<uint4*>(o) = v;
    };
    auto record = [&](int r, long long c) {
        const long long bk = static_cast<long long>(s) * a.out_oor.slots + r;
        const uint32_t en = atomicAdd(&a.out_oor.counts[bk], 1u);
        if (en < static_cast<uint32_t>(a.out_oor.cap))
            a.out_oor.entries[bk * a.out_oor.cap + en] = static_cast<uint32_t>(c);
    };
    if (a.mode == kLdsDec) {
        // the completed codeword -> INTT_n -> the k coefficients (x n^-1)
        const XfPlan& P = a.pni;
        if constexpr (C2) {
            // By linearity, INTT_n's first (unit) pass of the completed
            // codeword is the image (that pass of the zero-filled one) plus
            // its response to c_E: erased symbol t sits at element
            // q0 = t >> lgr[0] of group t & (R0 - 1), and that group's
            // output u gains c_E w_R1^(-q0 u).  Then only the last pass
            // runs -- no second load of the received rows, no second unit
            // pass.  Thread (u, c) owns output u of every group in column c,
            // so erasures sharing a group add in turn.
            const int lg0 = P.lgr[0], lg1 = P.lgr[1], m0 = (1 << lg0) - 1;
            for (int it = tid; it < (1 << (lg1 + lgT)); it += kLdsThreads) {
                const int u = it >> lgT, c = it & (T - 1);
                for (int j = 0; j < e; j++) {
                    const int t = s_eid[j], q0 = t >> lg0;
                    int32_t* d = buf + (prow(((t & m0) << lg1) + u) << lgT) + c;
                    // w_R1^-x = w_32^(-x 32 / R1)
                    const int32_t w = s_rinv[((q0 * u) << (5 - lg1)) & 31];
                    *d = fold(fold(*d + mul_rt(s_cE[(j << lgT) + c], w)));
                }
            }
            __syncthreads();
            const int lgs = P.sh[0], lgL = lgs + lg0;
            const int32_t* twp = tw + P.tw[0];
            switch (lg0) {
            case 1:
                lds_pass<2, false, true, false>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, nullptr,
                                                0, &P, 0);
                break;
            case 2:
                lds_pass<4, false, true, false>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, nullptr,
                                                0, &P, 0);
                break;
            case 3:
                lds_pass<8, false, true, false>(buf, twp, P.N, lgs, lgL, lgT, col, g, G, nullptr,
                                                0, &P, 0);
                break;
            case 4:
                lds_pass<16, false, true, false>(buf, twp, P.N, lgs, lgL, lgT, col, g, G,
                                                 nullptr, 0, &P, 0);
                break;
            default:
                lds_pass<32, false, true, false>(buf, twp, P.N, lgs, lgL, lgT, col, g, G,
                                                 nullptr, 0, &P, 0);
                break;
            }
            __syncthreads();
        } else {
            load(true);
            lds_transform<false, true>(buf, tw, P, lgT, col, g, G);
        }
        if (a.wide) {
            if (!wvalid)
                return;
            for (int r = rl; r < a.out_rows; r += RPP) {
                const int4* sp = reinterpret_cast<const int4*>(buf + (prow(r) << lgT) + 8 * cj);
                const int4 lo = sp[0], hi = sp[1];
                const int32_t v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
                uint32_t cv[8];
#pragma unroll
                for (int q = 0; q < 8; q++)
                    cv[q] = canon_vr(fold(mul_rt(v[q], a.inv_n)));
                store8(a.out + s * a.oss + r * a.ors + cw, cv);
            }
            return;
        }
        if (!valid)
            return;
        for (int r = g; r < a.out_rows; r += G)
            a.out[s * a.oss + r * a.ors + cg] = static_cast<uint16_t>(
                canon_vr(fold(mul_rt(buf[(prow(r) << lgT) + col], a.inv_n))));
        return;
    }
    // systematic (decode: the data rows t < k; encode: the parities t >= k):
    // codeword symbols, received ones copied, erased ones from c_E
    if (a.wide) {
        if (!wvalid)
            return;
        for (int r = rl; r < a.out_rows; r += RPP) {
            const int t = a.out_first + r, pm = s_pos[t];
            uint16_t* o = a.out + s * a.oss + r * a.ors + cw;
            if (pm >= 0) {
                *reinterpret_cast<uint4*>(o) =
                    *reinterpret_cast<const uint4*>(row_ptr(src.by_pos ? pm : t) + cw);
                continue;
            }
            const int32_t* ce = s_cE + ((-1 - pm) << lgT) + 8 * cj;
            uint32_t cv[8];
            bool any = false;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                cv[q] = canon_vr(ce[q]);
                any |= cv[q] == 65536u;
            }
            store8(o, cv);
            if (any && a.out_oor.counts)
                for (int q = 0; q < 8; q++)
                    if (cv[q] == 65536u)
                        record(r, cw + q);
        }
        return;
    }
    if (!valid)
        return;
    for (int r = g; r < a.out_rows; r += G) {
        const int t = a.out_first + r, pm = s_pos[t];
        uint32_t cv;
        if (pm >= 0) {
            cv = row_ptr(src.by_pos ? pm : t)[cg];
        } else {
            cv = canon_vr(s_cE[((-1 - pm) << lgT) + col]);
            if (cv == 65536u && a.out_oor.counts)
                record(r, cg);
        }
        a.out[s * a.oss + r * a.ors + cg] = static_cast<uint16_t>(cv);
    }
}

namespace {

int ilog2i(long long v)
{
    int l = 0;
    while ((1LL << l) < v)
        l++;
    return l;
}

// radices <= 32, as even as possible
std::vector<int> radices(int N)
{
    const int bits = ilog2i(N);
    const int m = std::max(1, (bits + 4) / 5);
    std::vector<int> r;
    int left = bits;
    for (int p = 0; p < m; p++) {
        const int bp = (left + (m - p) - 1) / (m - p);
        r.push_back(1 << bp);
        left -= bp;
    }
    return r;
}

int launch_pass(const NttPassArgs& a, int S, hipStream_t st)
{
    const dim3 grid(static_cast<unsigned>(a.tiles) * static_cast<unsigned>(S),
                    static_cast<unsigned>(a.N / a.R));
    switch (a.R) {
#define QI_NTT_R(RR)                                                              \
    case RR:                                                                      \
        hipLaunchKernelGGL(ntt_pass_kernel<RR>, grid, dim3(kNttBlock), 0, st, a); \
        break;
        QI_NTT_R(2)
        QI_NTT_R(4)
        QI_NTT_R(8)
        QI_NTT_R(16)
        QI_NTT_R(32)
#undef QI_NTT_R
    default:
        return -3;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// One transform of length N over S stripes: pass 0 gathers from a.in, the
// last pass writes a.out rows (or leaves the result in a.scr).
int transform(NttPassArgs a, const qi_plan* p, int N, bool inverse, int S, hipStream_t st)
{
    const std::vector<int> rs = radices(N);
    if (N < 2 || N > p->nmax || static_cast<int>(rs.size()) > kMaxPasses)
        return -3;
    a.N = N;
    a.inverse = inverse ? 1 : 0;
    a.tw = p->d_tw[inverse ? 1 : 0];
    a.twstep = p->nmax / N;
    a.npass = static_cast<int>(rs.size());
    for (int q = 0; q < a.npass; q++)
        a.radix[q] = rs[q];
    int Sp = 1;
    uint16_t* out = a.out;
    for (int q = 0; q < a.npass; q++) {
        a.R = rs[q];
        a.S = Sp;
        a.first = q == 0;
        a.last = q == a.npass - 1;
        a.out = a.last ? out : nullptr;
        if (const int rc = launch_pass(a, S, st))
            return rc;
        Sp *= rs[q];
    }
    return 0;
}

// slice geometry: columns per slice and stripes per launch so that one
// scratch buffer (nmax rows x cols int32 per stripe) stays within ~256 MiB
struct Slicing {
    long long W;
    int Sg;
};

Slicing slicing(const qi_plan* p, long long words, int S)
{
    const long long budget = 64LL << 20;  // int32 elements per buffer
    const long long wp = (words + kNttBlock - 1) / kNttBlock * kNttBlock;
    long long W = budget / p->nmax / kNttBlock * kNttBlock;
    W = std::max<long long>(kNttBlock, std::min(W, wp));
    const long long sg = std::max<long long>(1, budget / (p->nmax * W));
    return Slicing{W, static_cast<int>(std::min<long long>(sg, S))};
}

struct Scratch {
    void* p = nullptr;
    hipStream_t st = nullptr;
    ~Scratch()
    {
        if (p)
            (void)hipFreeAsync(p, st);
    }
};

NttCtxLayout ctx_layout_of(const qi_plan* p)
{
    return NttCtxLayout{p->k, p->n, p->len2k};
}

// radices <= 32 for the LDS passes, as even as possible (fewest twiddled
// passes)
XfPlan xf_plan(int N)
{
    // radices <= 32 as even as possible (2048: 16, 16, 8).  Round 6 tried the
    // radix-32 unit pass the image's row padding keeps conflict-free (2048:
    // 8, 8, 32; the k600 encode had 58 % of its LDS cycles in bank
    // conflicts): 2.06-2.09 -> 2.17-2.26 ms, the radix-8 passes cost more
    // than the conflicts (profiles/r6_ab_notes.txt), so the plan stays
    XfPlan P{};
    P.N = N;
    const int bits = ilog2i(N);
    P.np = std::max(1, (bits + 4) / 5);
    int left = bits, sh = bits;
    for (int q = 0; q < P.np; q++) {
        const int b = (left + (P.np - q) - 1) / (P.np - q);
        P.lgr[q] = b;
        sh -= b;
        P.sh[q] = sh;
        left -= b;
    }
    return P;
}

// The four transforms' pass twiddle tables, back to back (offsets kept 4-
// aligned for the vector LDS reads): pass q of a length-N transform holds
// w_{L_q}^{+-j u} at j R_q + u, with w_L = w_nmax^{nmax / L}.  Fills `tab`
// when given; returns the total words.
// Order INTT_n, NTT_2k, INTT_2k, NTT_n: a decode stages the first three, a
// non-systematic encode the last one, systematic codes all four.
enum : int { kTwPni = 0, kTwP2f = 1, kTwP2i = 2, kTwPnf = 3 };

int lds_tables(const qi_plan* p, XfPlan* pl, std::vector<int32_t>* tab, int* twist = nullptr,
               int* rinv_off = nullptr)
{
    const uint32_t w = root_of_unity(static_cast<uint32_t>(p->nmax));
    const int h = p->len2k / 2;
    const int Ns[4] = {p->n, h, h, p->n};
    const bool invs[4] = {true, false, true, false};
    int off = 0;
    for (int t = 0; t < 4; t++) {
        if (t == kTwPnf) {
            if (twist)
                *twist = off;
            // the decode's twist w2k^{+-t}, t < h, between INTT_h and NTT_n
            // (a decode stages [0, NTT_n's offset))
            if (tab) {
                tab->resize(off + 2 * h);
                const uint32_t w2 = powmod_c(w, static_cast<uint32_t>(p->nmax / p->len2k));
                const uint32_t w2i = invmod_c(w2);
                for (int i = 0; i < h; i++) {
                    (*tab)[off + i] = balanced(powmod_c(w2, static_cast<uint32_t>(i)));
                    (*tab)[off + h + i] = balanced(powmod_c(w2i, static_cast<uint32_t>(i)));
                }
            }
            off += (2 * h + 3) & ~3;
        }
        pl[t] = xf_plan(Ns[t]);
        const bool inv = invs[t];
        for (int q = 0; q < pl[t].np; q++) {
            const int R = 1 << pl[t].lgr[q], sq = 1 << pl[t].sh[q], L = R * sq;
            pl[t].tw[q] = off;
            if (tab) {
                tab->resize(off + L);
                const uint32_t wl = powmod_c(w, static_cast<uint32_t>(p->nmax / L));
                const uint32_t wb = inv ? invmod_c(wl) : wl;
                for (int j = 0; j < sq; j++)
                    for (int u = 0; u < R; u++)
                        (*tab)[off + j * R + u] = balanced(
                            powmod_c(wb, static_cast<uint32_t>(j * u % L)));
            }
            off += (L + 3) & ~3;
        }
    }
    // w_32^-x, x < 32: the inverse R-th roots of INTT_n's DIT passes for
    // every radix R | 32 (w_R^-x = w_32^(-x 32 / R)), for the erasure
    // decode's pruned last pass (lds_intt_top) and its two-pass completion
    if (rinv_off)
        *rinv_off = off;
    if (tab) {
        tab->resize(off + 32);
        const uint32_t wi = invmod_c(root_of_unity(32u));
        for (int x = 0; x < 32; x++)
            (*tab)[off + x] = balanced(powmod_c(wi, static_cast<uint32_t>(x)));
    }
    off += 32;
    if (tab)
        tab->resize(off);
    return off;
}

// rows: the image's rows (nmax; n for the non-systematic encode, which
// runs NTT_n alone)
size_t lds_bytes(const qi_plan* p, int lgT, int tw_words, bool twg, int rows)
{
    return ((static_cast<size_t>(prow(rows)) << lgT) +
            lds_side_words(tw_words, p->k, p->len2k, twg)) *
           4;
}

constexpr size_t kLdsCap = 160 * 1024;  // LDS per CU

// the table range [lo, hi) a mode stages (see the table order above)
void lds_table_range(const qi_plan* p, int mode, int* lo, int* hi)
{
    XfPlan pl[4];
    const int end = lds_tables(p, pl, nullptr);
    if (mode == kLdsEnc) {
        *lo = pl[kTwPnf].tw[0];
        *hi = end;
    } else {
        *lo = 0;
        *hi = mode == kLdsDec ? pl[kTwPnf].tw[0] : end;
    }
}

// columns per workgroup: the widest tile (<= 64 columns) that leaves room
// for two workgroups per CU with the tables staged, else with the tables
// read from global memory (*twg), else one workgroup per CU (at least 8
// columns)
int lds_geom(const qi_plan* p, int tw_words, bool* twg, int rows)
{
    for (int g = 0; g < 2; g++)
        for (int lg = 6; lg >= 3; lg--)
            if (lds_bytes(p, lg, tw_words, g == 1, rows) <= kLdsCap / 2) {
                *twg = g == 1;
                return lg;
            }
    *twg = false;
    return lds_bytes(p, 3, tw_words, false, rows) <= kLdsCap ? 3 : -1;
}

bool lds_engine(const qi_plan* p)
{
    if (p->nmax > kLdsMaxN)
        return false;
    int lo, hi;
    lds_table_range(p, kLdsSysDec, &lo, &hi);  // the largest set
    bool twg;
    return lds_geom(p, hi - lo, &twg, p->nmax) >= 0;
}

// ---- erasure decode (ntt_eras_kernel) ----
// the two-pass completion (ntt_eras_kernel<., true>): the non-systematic
// decode of a two-pass INTT_n; it reads no position map, and that region
// holds the e x T syndromes instead
static bool eras_c2(const XfPlan& pni)
{
    return pni.np == 2;
}

bool eras_plan(const qi_plan* p)
{
    return p->ntt && !p->mbig && eras_shape(p->k, p->n);
}

ErasCtxLayout eras_layout(const qi_plan* p)
{
    return ErasCtxLayout{p->k, p->n, p->n - p->k};
}

size_t eras_bytes(const qi_plan* p, int lgT, int tw_words, bool twg, bool c2)
{
    const ErasCtxLayout L = eras_layout(p);
    const size_t posw = c2 ? static_cast<size_t>(L.e) << lgT : static_cast<size_t>(L.n);
    return ((static_cast<size_t>(prow(p->n)) << lgT) + (twg ? 0 : tw_words) + L.k + posw + L.e +
            static_cast<size_t>(L.e) * L.e + (static_cast<size_t>(L.e) << lgT) + 32) *
           4;
}

// INTT_n's tables only: [0, NTT_h's first table)
int eras_tw_words(const qi_plan* p, XfPlan* pl)
{
    lds_tables(p, pl, nullptr);
    return pl[kTwP2f].tw[0];
}

// tile width (log2 T) at two workgroups per CU, tables staged when they
// fit; *c2: the launch takes the two-pass completion (dec: a non-systematic
// decode)
int eras_geom(const qi_plan* p, bool dec, bool* twg, bool* c2)
{
    XfPlan pl[4];
    const int tw_words = eras_tw_words(p, pl);
    for (int g = 0; g < 2; g++)
        for (int lg = 6; lg >= 3; lg--) {
            const bool two = dec && eras_c2(pl[kTwPni]);
            if (eras_bytes(p, lg, tw_words, g == 1, two) <= kLdsCap / 2) {
                *twg = g == 1;
                *c2 = two;
                return lg;
            }
        }
    *twg = false;
    *c2 = dec && eras_c2(pl[kTwPni]);
    return eras_bytes(p, 3, tw_words, false, *c2) <= kLdsCap ? 3 : -1;
}

int eras_launch(const qi_plan* p, NttLdsArgs a, int S, hipStream_t st)
{
    a.k = p->k;
    a.n = p->n;
    a.len2k = p->len2k;
    a.nmax = p->n;
    XfPlan pl[4];
    a.tw_words = eras_tw_words(p, pl);
    a.pni = pl[kTwPni];
    a.tw = p->d_ldstw;
    int rinv_off = 0;
    lds_tables(p, pl, nullptr, nullptr, &rinv_off);
    a.rinv = p->d_ldstw ? p->d_ldstw + rinv_off : nullptr;
    bool twg, c2;
    a.lgT = eras_geom(p, a.mode == kLdsDec, &twg, &c2);
    if (a.lgT < 0 || !a.tw)
        return -3;
    const ErasCtxLayout L = eras_layout(p);
    a.ids_off = static_cast<int>(L.ids_off());
    a.pos_off = static_cast<int>(L.pos_off());
    a.eras_e = L.e;
    a.eras_eid = static_cast<int>(L.eid_off());
    a.eras_b = static_cast<int>(L.b_off());
    a.inv_n = balanced(invmod_c(static_cast<uint32_t>(p->n)));
    const long long tiles = (a.words + (1LL << a.lgT) - 1) >> a.lgT;
    if (tiles * S > 0x7fffffffLL)
        return -3;
    a.tiles = static_cast<int>(tiles);
    {
        auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
        auto a8 = [](long long v) { return (v & 7) == 0; };
        const RowSrc& r = a.src;
        a.wide = (a.words & 7) == 0 && al(r.base0) && a8(r.ss0) && a8(r.rs0) &&
                 (!r.base1 || (al(r.base1) && a8(r.ss1) && a8(r.rs1))) && al(a.out) &&
                 a8(a.oss) && a8(a.ors);
    }
    const size_t lds = eras_bytes(p, a.lgT, a.tw_words, twg, c2);
    const void* fn =
        twg ? (c2 ? reinterpret_cast<const void*>(&ntt_eras_kernel<true, true>)
                  : reinterpret_cast<const void*>(&ntt_eras_kernel<true, false>))
            : (c2 ? reinterpret_cast<const void*>(&ntt_eras_kernel<false, true>)
                  : reinterpret_cast<const void*>(&ntt_eras_kernel<false, false>));
    if (lds > 65536 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           static_cast<int>(lds)) != hipSuccess)
        return -2;
    const dim3 grid(static_cast<unsigned>(tiles * S));
    if (twg && c2)
        hipLaunchKernelGGL((ntt_eras_kernel<true, true>), grid, dim3(kLdsThreads), lds, st, a);
    else if (twg)
        hipLaunchKernelGGL((ntt_eras_kernel<true, false>), grid, dim3(kLdsThreads), lds, st, a);
    else if (c2)
        hipLaunchKernelGGL((ntt_eras_kernel<false, true>), grid, dim3(kLdsThreads), lds, st, a);
    else
        hipLaunchKernelGGL((ntt_eras_kernel<false, false>), grid, dim3(kLdsThreads), lds, st,
                           a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int lds_launch(const qi_plan* p, NttLdsArgs a, int S, hipStream_t st)
{
    a.k = p->k;
    a.n = p->n;
    a.len2k = p->len2k;
    a.nmax = p->nmax;
    XfPlan pl[4];
    int twist = 0;
    lds_tables(p, pl, nullptr, &twist);
    int lo, hi;
    lds_table_range(p, a.mode, &lo, &hi);
    for (XfPlan& x : pl)
        for (int q = 0; q < x.np; q++)
            x.tw[q] -= lo;  // offsets within the staged range
    a.twist = twist - lo;  // (read by decodes only, which stage from 0)
    a.pni = pl[kTwPni];
    a.p2f = pl[kTwP2f];
    a.p2i = pl[kTwP2i];
    a.pnf = pl[kTwPnf];
    a.tw = p->d_ldstw + lo;
    a.tw_words = hi - lo;
    // the non-systematic encode runs NTT_n alone and could take an n-row
    // image (wider tiles where len_2k > n); measured slower at k1000 (T = 16
    // instead of 8: encode 1.27-1.29 -> 1.33 ms, gpurun_out ab_route), so the
    // image stays nmax rows (the n-row variant measured 1.31 vs 1.25 ms
    // after the padded rows, round 4)
    bool twg;
    a.lgT = lds_geom(p, a.tw_words, &twg, a.nmax);
    if (a.lgT < 0)
        return -3;
    const NttCtxLayout L = ctx_layout_of(p);
    a.ids_off = static_cast<int>(L.ids_off());
    a.c_off = static_cast<int>(L.c_off());
    a.pos_off = static_cast<int>(L.pos_off());
    const long long tiles = (a.words + (1LL << a.lgT) - 1) >> a.lgT;
    if (tiles * S > 0x7fffffffLL)
        return -3;
    a.tiles = static_cast<int>(tiles);
    {
        auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
        auto a8 = [](long long v) { return (v & 7) == 0; };
        const RowSrc& r = a.src;
        a.wide = (a.words & 7) == 0 && al(r.base0) && a8(r.ss0) && a8(r.rs0) &&
                 (!r.base1 || (al(r.base1) && a8(r.ss1) && a8(r.rs1))) && al(a.out) &&
                 a8(a.oss) && a8(a.ors);
    }
    const size_t lds = lds_bytes(p, a.lgT, a.tw_words, twg, a.nmax);
    const void* fn = twg ? reinterpret_cast<const void*>(&ntt_lds_kernel<true>)
                         : reinterpret_cast<const void*>(&ntt_lds_kernel<false>);
    if (lds > 65536 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           static_cast<int>(lds)) != hipSuccess)
        return -2;
    if (twg)
        hipLaunchKernelGGL(ntt_lds_kernel<true>, dim3(static_cast<unsigned>(tiles * S)),
                           dim3(kLdsThreads), lds, st, a);
    else
        hipLaunchKernelGGL(ntt_lds_kernel<false>, dim3(static_cast<unsigned>(tiles * S)),
                           dim3(kLdsThreads), lds, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

RowSrc offset_src(RowSrc s, int sg0, long long c0)
{
    s.base0 += sg0 * s.ss0 + c0;
    if (s.base1)
        s.base1 += sg0 * s.ss1 + c0;
    return s;
}

// The interpolation (decode_apply) of Sg stripes over the slice: the k
// received rows -> coefficient rows.  res != null: the k coefficient rows
// are written there as u16; otherwise they stay in scratch B (int32).
int interpolate(const qi_plan* p, const int32_t* ctx, long long cs, const RowSrc& src,
                const Oor* in_oor, int slot_base, long long c0, long long cols, int Sg,
                int32_t* A, int32_t* B, long long sss, const RowDst* res, uint32_t* err,
                hipStream_t st)
{
    const NttCtxLayout L = ctx_layout_of(p);
    const int tiles = static_cast<int>((cols + kNttBlock - 1) / kNttBlock);
    // y_i = v_i inv_A_i -> A rows 0..k-1
    NttExpandArgs e{src, ctx, cs, static_cast<int>(L.ids_off()), p->k, A, sss, cols, tiles};
    hipLaunchKernelGGL(ntt_expand_kernel, dim3(tiles * Sg, p->k), dim3(kNttBlock), 0, st, e);
    if (hipGetLastError() != hipSuccess)
        return -2;
    if (in_oor && in_oor->counts) {
        NttFixArgs f{*in_oor, slot_base, src.by_pos, ctx, cs, static_cast<int>(L.ids_off()),
                     A, sss, cols, c0, err};
        hipLaunchKernelGGL(ntt_fix_kernel, dim3(Sg, p->k), dim3(kNttBlock), 0, st, f);
        if (hipGetLastError() != hipSuccess)
            return -2;
    }
    NttPassArgs a{};
    a.tiles = tiles;
    a.cols = cols;
    a.sss = sss;
    // INTT_n of the y_i placed at positions z_i (buf1_n) -> B
    a.scr = B;
    a.in = A;
    a.iss = sss;
    a.irs = cols;
    a.in_u16 = 0;
    a.in_rows = p->k;
    a.posmap = ctx + L.pos_off();
    a.pms = cs;
    if (int rc = transform(a, p, p->n, true, Sg, st))
        return rc;
    // NTT_2k of its first k outputs (zero-extended) -> A
    a.scr = A;
    a.in = B;
    a.posmap = nullptr;
    if (int rc = transform(a, p, p->len2k, false, Sg, st))
        return rc;
    // x C, INTT_2k -> the k coefficient rows (res, or B)
    a.scr = B;
    a.in = A;
    a.in_rows = p->len2k;
    a.scale = ctx + L.c_off();
    a.scs = cs;
    if (res) {
        a.out = res->base;
        a.oss = res->ss;
        a.ors = res->rs;
        a.row0 = 0;
        a.out_rows = p->k;
    }
    return transform(a, p, p->len2k, true, Sg, st);
}

}  // namespace

static int launch_ntt_ctx(const qi_plan* p, const NttCtxArgs& a, int S, hipStream_t st)
{
    const size_t lds =
        static_cast<size_t>((p->k + kCtxChains - 1) / kCtxChains * kCtxChains) * 4;
    if (lds > 65536 && hipFuncSetAttribute(reinterpret_cast<const void*>(&ntt_ctx_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           static_cast<int>(lds)) != hipSuccess)
        return -2;
    const int items = p->len2k + p->k;
    hipLaunchKernelGGL(ntt_ctx_kernel, dim3(S, (items + kNttBlock - 1) / kNttBlock),
                       dim3(kNttBlock), lds, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

bool eras_shape(int k, int n)
{
    return n <= kLdsMaxN && n - k <= kErasMax;
}

long long ntt_ctx_words(const qi_plan* p)
{
    return eras_plan(p) ? eras_layout(p).words() : ctx_layout_of(p).words();
}

int ntt_build_ctx(const qi_plan* p, const uint16_t* d_ids, int S, int32_t* ctx, long long cs,
                  hipStream_t st)
{
    if (S <= 0)
        return 0;
    if (eras_plan(p)) {
        const uint32_t r = root_of_unity(static_cast<uint32_t>(p->n));
        ErasCtxArgs e{eras_layout(p), r, invmod_c(r), d_ids, ctx, cs, p->d_err};
        hipLaunchKernelGGL(eras_ctx_kernel, dim3(S), dim3(64), 0, st, e);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    NttCtxArgs a{ctx_layout_of(p), p->r, root_of_unity(static_cast<uint32_t>(p->len2k)),
                 invmod_c(static_cast<uint32_t>(p->len2k)), d_ids, ctx, cs, nullptr, nullptr,
                 p->d_err};
    return launch_ntt_ctx(p, a, S, st);
}

int ntt_build_ctx_lazy(const qi_plan* p, const int32_t* ids32, int S, int32_t* ctx,
                       long long cs, uint32_t* lazy, hipStream_t st)
{
    if (S <= 0)
        return 0;
    if (eras_plan(p) || !ids32 || !lazy)
        return -1;  // only the 256 < k <= 384 plans build lazily
    NttCtxArgs a{ctx_layout_of(p), p->r, root_of_unity(static_cast<uint32_t>(p->len2k)),
                 invmod_c(static_cast<uint32_t>(p->len2k)), nullptr, ctx, cs, ids32, lazy,
                 p->d_err};
    if (int rc = launch_ntt_ctx(p, a, S, st))
        return rc;
    hipLaunchKernelGGL(lazy_mark_kernel, dim3((S + 255) / 256), dim3(256), 0, st, lazy, cs, S,
                       kLazyNtt);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int ntt_plan_init(qi_plan* p)
{
    p->len2k = static_cast<int>(ceil2(static_cast<uint32_t>(2 * p->k)));
    p->nmax = std::max(p->n, p->len2k);
    if (p->nmax > 65536)
        return -1;
    const uint32_t w = root_of_unity(static_cast<uint32_t>(p->nmax));
    const uint32_t wi = invmod_c(w);
    std::vector<int32_t> tw(2 * static_cast<size_t>(p->nmax));
    uint32_t f = 1, g = 1;
    for (int e = 0; e < p->nmax; e++) {
        tw[e] = balanced(f);
        tw[p->nmax + e] = balanced(g);
        f = mulmod_c(f, w);
        g = mulmod_c(g, wi);
    }
    int32_t* d = nullptr;
    if (hipMalloc(&d, tw.size() * 4) != hipSuccess)
        return -2;
    p->d_tw[0] = d;
    p->d_tw[1] = d + p->nmax;
    if (hipMemcpy(d, tw.data(), tw.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return -2;
    if (lds_engine(p) || eras_plan(p)) {
        XfPlan pl[4];
        std::vector<int32_t> tab;
        lds_tables(p, pl, &tab);
        if (hipMalloc(&p->d_ldstw, tab.size() * 4) != hipSuccess ||
            hipMemcpy(p->d_ldstw, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) !=
                hipSuccess)
            return -2;
    }
    if (p->sys) {
        // the systematic encode's constant context: points r^0 .. r^{k-1}
        const long long cs = ntt_ctx_words(p);
        if (hipMalloc(&p->d_sysctx, cs * 4) != hipSuccess)
            return -2;
        if (ntt_build_ctx(p, nullptr, 1, p->d_sysctx, cs, nullptr) ||
            hipStreamSynchronize(nullptr) != hipSuccess)
            return -2;
    }
    return 0;
}

std::string ntt_kernel_names(const qi_plan* p, bool decode)
{
    if (eras_plan(p) && (decode || p->sys)) {
        bool twg, c2;
        (void)eras_geom(p, decode && !p->sys, &twg, &c2);
        return std::string(decode ? "eras_ctx_kernel + " : "") + "ntt_eras_kernel<" +
               (twg ? "true" : "false") + ", " + (c2 ? "true" : "false") + ">";
    }
    if (!lds_engine(p))
        return decode ? "ntt_ctx_kernel + ntt_expand_kernel + ntt_fix_kernel + ntt_pass_kernel"
                      : "ntt_pass_kernel";
    const int mode = decode ? (p->sys ? kLdsSysDec : kLdsDec) : (p->sys ? kLdsSysEnc : kLdsEnc);
    int lo, hi;
    lds_table_range(p, mode, &lo, &hi);
    bool twg;
    (void)lds_geom(p, hi - lo, &twg, p->nmax);
    return std::string(decode ? "ntt_ctx_kernel + " : "") +
           (twg ? "ntt_lds_kernel<true>" : "ntt_lds_kernel<false>");
}

void ntt_plan_free(qi_plan* p)
{
    if (p->d_tw[0])
        (void)hipFree(p->d_tw[0]);
    if (p->d_sysctx)
        (void)hipFree(p->d_sysctx);
    if (p->d_ldstw)
        (void)hipFree(p->d_ldstw);
    p->d_ldstw = nullptr;
    p->d_tw[0] = p->d_tw[1] = nullptr;
    p->d_sysctx = nullptr;
}

// non-systematic: outputs 0 .. n_out-1 of NTT_n(data zero-padded);
// systematic: parities k .. k+m-1 of NTT_n(interpolation of the data rows)
int ntt_encode(const qi_plan* p, const uint16_t* data, long long dss, long long drs,
               RowDst out, long long words, int S, const Oor* oor, hipStream_t st)
{
    if (S <= 0 || words <= 0)
        return 0;
    if (p->sys && eras_plan(p)) {
        // the parities as the erased symbols of the data's codeword
        NttLdsArgs a{};
        a.mode = kLdsSysEnc;
        a.words = words;
        a.src = RowSrc{data, dss, drs, 1 << 30, nullptr, 0, 0, 1, p->k, 0};
        a.ctx = p->d_sysctx;
        a.cs = 0;
        a.out = out.base;
        a.oss = out.ss;
        a.ors = out.rs;
        a.out_first = p->k;
        a.out_rows = p->n_outputs;
        if (oor && oor->counts)
            a.out_oor = *oor;
        a.err = p->d_err;
        return eras_launch(p, a, S, st);
    }
    if (lds_engine(p)) {
        NttLdsArgs a{};
        a.mode = p->sys ? kLdsSysEnc : kLdsEnc;
        a.words = words;
        a.src = RowSrc{data, dss, drs, 1 << 30, nullptr, 0, 0, 1, p->k, 0};
        a.ctx = p->sys ? p->d_sysctx : nullptr;
        a.cs = 0;
        a.out = out.base;
        a.oss = out.ss;
        a.ors = out.rs;
        a.out_first = p->sys ? p->k : 0;
        a.out_rows = p->n_outputs;
        if (oor && oor->counts)
            a.out_oor = *oor;
        a.err = p->d_err;
        return lds_launch(p, a, S, st);
    }
    const Slicing sl = slicing(p, words, S);
    const long long sss = static_cast<long long>(p->nmax) * sl.W;
    Scratch sa, sb;
    sa.st = sb.st = st;
    const size_t bytes = static_cast<size_t>(sl.Sg) * sss * 4;
    if (hipMallocAsync(&sa.p, bytes, st) != hipSuccess ||
        (p->sys && hipMallocAsync(&sb.p, bytes, st) != hipSuccess))
        return -2;
    int32_t* A = static_cast<int32_t*>(sa.p);
    int32_t* B = static_cast<int32_t*>(sb.p);
    for (int sg0 = 0; sg0 < S; sg0 += sl.Sg) {
        const int Sg = std::min(sl.Sg, S - sg0);
        for (long long c0 = 0; c0 < words; c0 += sl.W) {
            const long long cols = std::min(sl.W, words - c0);
            NttPassArgs a{};
            a.tiles = static_cast<int>((cols + kNttBlock - 1) / kNttBlock);
            a.cols = cols;
            a.sss = sss;
            a.out = out.base + sg0 * out.ss + c0;
            a.oss = out.ss;
            a.ors = out.rs;
            a.out_rows = p->n_outputs;
            a.col0 = c0;
            if (oor && oor->counts) {
                a.oor = *oor;
                a.oor.counts += static_cast<long long>(sg0) * oor->slots;
                a.oor.entries += static_cast<long long>(sg0) * oor->slots * oor->cap;
            }
            const uint16_t* din = data + sg0 * dss + c0;
            if (!p->sys) {
                a.scr = A;
                a.in = din;
                a.iss = dss;
                a.irs = drs;
                a.in_u16 = 1;
                a.in_rows = p->k;
                a.row0 = 0;
                if (int rc = transform(a, p, p->n, false, Sg, st))
                    return rc;
            } else {
                const RowSrc src{din, dss, drs, 1 << 30, nullptr, 0, 0, 1, p->k, 0};
                if (int rc = interpolate(p, p->d_sysctx, 0, src, nullptr, 0, c0, cols, Sg, A, B,
                                         sss, nullptr, p->d_err, st))
                    return rc;
                // coefficient rows (B) -> NTT_n -> rows k .. k+m-1
                a.scr = A;
                a.in = B;
                a.iss = sss;
                a.irs = cols;
                a.in_u16 = 0;
                a.in_rows = p->k;
                a.row0 = p->k;
                if (int rc = transform(a, p, p->n, false, Sg, st))
                    return rc;
            }
        }
    }
    return 0;
}

// decode of S stripes: ctx from ntt_build_ctx; src as in launch_matrix (by
// id through the context's ids, or by position); in_oor buckets by slot =
// id - slot_base (or position)
int ntt_decode(const qi_plan* p, const int32_t* ctx, long long cs, RowSrc src,
               const Oor* in_oor, int slot_base, RowDst out, long long words, int S,
               hipStream_t st)
{
    if (S <= 0 || words <= 0)
        return 0;
    if (lds_engine(p) || eras_plan(p)) {
        NttLdsArgs a{};
        a.mode = p->sys ? kLdsSysDec : kLdsDec;
        a.words = words;
        a.src = src;
        a.ctx = ctx;
        a.cs = cs;
        if (in_oor && in_oor->counts)
            a.in_oor = *in_oor;
        a.slot_base = slot_base;
        a.out = out.base;
        a.oss = out.ss;
        a.ors = out.rs;
        a.out_first = 0;
        a.out_rows = p->k;
        a.err = p->d_err;
        return eras_plan(p) ? eras_launch(p, a, S, st) : lds_launch(p, a, S, st);
    }
    const Slicing sl = slicing(p, words, S);
    const long long sss = static_cast<long long>(p->nmax) * sl.W;
    Scratch sa, sb;
    sa.st = sb.st = st;
    const size_t bytes = static_cast<size_t>(sl.Sg) * sss * 4;
    if (hipMallocAsync(&sa.p, bytes, st) != hipSuccess ||
        hipMallocAsync(&sb.p, bytes, st) != hipSuccess)
        return -2;
    int32_t* A = static_cast<int32_t*>(sa.p);
    int32_t* B = static_cast<int32_t*>(sb.p);
    for (int sg0 = 0; sg0 < S; sg0 += sl.Sg) {
        const int Sg = std::min(sl.Sg, S - sg0);
        const int32_t* cx = ctx + sg0 * cs;
        Oor io{};
        if (in_oor && in_oor->counts) {
            io = *in_oor;
            io.counts += static_cast<long long>(sg0) * in_oor->slots;
            io.entries += static_cast<long long>(sg0) * in_oor->slots * in_oor->cap;
        }
        for (long long c0 = 0; c0 < words; c0 += sl.W) {
            const long long cols = std::min(sl.W, words - c0);
            const RowSrc s2 = offset_src(src, sg0, c0);
            RowDst o{out.base + sg0 * out.ss + c0, out.ss, out.rs};
            if (!p->sys) {
                if (int rc = interpolate(p, cx, cs, s2, io.counts ? &io : nullptr, slot_base, c0,
                                         cols, Sg, A, B, sss, &o, p->d_err, st))
                    return rc;
                continue;
            }
            if (int rc = interpolate(p, cx, cs, s2, io.counts ? &io : nullptr, slot_base, c0,
                                     cols, Sg, A, B, sss, nullptr, p->d_err, st))
                return rc;
            // the data rows are the evaluations at r^t, t < k
            NttPassArgs a{};
            a.tiles = static_cast<int>((cols + kNttBlock - 1) / kNttBlock);
            a.cols = cols;
            a.sss = sss;
            a.scr = A;
            a.in = B;
            a.iss = sss;
            a.irs = cols;
            a.in_u16 = 0;
            a.in_rows = p->k;
            a.out = o.base;
            a.oss = o.ss;
            a.ors = o.rs;
            a.row0 = 0;
            a.out_rows = p->k;
            if (int rc = transform(a, p, p->n, false, Sg, st))
                return rc;
        }
    }
    return 0;
}

}  // namespace qi
