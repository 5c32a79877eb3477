// Per-stripe decode contexts on the GPU for the matrix paths (k <= 256):
// the Lagrange form of DecodeContext::init (src/fec_context.h:232-274), the
// packed / matrix-core forms of the interpolation matrix (matrix_pack.h)
// and the OOR route tables of decode_prepare (src/fec_base.h:1361-1404).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>

#include "gf65537.h"
#include "matrix_pack.h"
#include "qi_internal.h"

namespace qi {
// ---------------------------------------------------------------------------
// Per-stripe decode context: the Lagrange form of DecodeContext::init
// (src/fec_context.h:232-274).  For received points x_i = r^{id_i}:
//   A(x) = prod_j (x - x_j),  Q_i = A / (x - x_i),  A'(x_i) = Q_i(x_i)
//   mode 0: M[t][i] = coef_t(Q_i) / A'(x_i)       (non-systematic)
//   mode 1: M[t][i] = Q_i(r^t)   / A'(x_i)        (systematic)
// plus the OOR route table of the stripe (decode_prepare's props walk,
// src/fec_base.h:1361-1404, precomputed per tile).
// One workgroup per stripe (64 lanes for k <= 32, else 256); k <= 256.
// ---------------------------------------------------------------------------
// canonical a * b mod 65537 for a, b in [0, 65536]: with 2^16 = -1 and
// 2^32 = 1, p = p0 + p1 2^16 + p2 2^32 reduces to p0 - p1 + p2
__device__ __forceinline__ uint32_t mulm(uint32_t a, uint32_t b)
{
    // balanced operands (|a|, |b| <= 32768): the product fits int32 and one
    // full-rate v_mul_i32_i24 forms it (the 64-bit product took two
    // quarter-rate v_mul_{lo,hi}_u32 on the serial Lagrange chains)
    const int32_t ab = static_cast<int32_t>(a) - (a > 32768u ? 65537 : 0);
    const int32_t bb = static_cast<int32_t>(b) - (b > 32768u ? 65537 : 0);
    const int32_t p = __mul24(ab, bb);                      // |p| <= 2^30
    const int32_t v = (p & 0xffff) - (p >> 16);             // [-16384, 81919]
    const int32_t w = v < 0 ? v + 65537 : v;                // [0, 81919]
    return static_cast<uint32_t>(w >= 65537 ? w - 65537 : w);
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
__device__ __forceinline__ uint32_t powm(uint32_t b, uint32_t e)
{
    uint32_t r = 1;
    for (; e; e >>= 1) {
        if (e & 1)
            r = mulm(r, b);
        b = mulm(b, b);
    }
    return r;
}

// x * y mod q for |x|, |y| < 2^17: the 48-bit product as v_mul_i32_i24 +
// v_mul_hi_i32_i24, reduced with 2^32 = 1 and 2^16 = -1: |result| < 65600
__device__ __forceinline__ int32_t mul_lz(int32_t x, int32_t y)
{
    uint32_t lo;
    int32_t hi;
    asm("v_mul_i32_i24 %0, %1, %2" : "=v"(lo) : "v"(x), "v"(y));
    asm("v_mul_hi_i32_i24 %0, %1, %2" : "=v"(hi) : "v"(x), "v"(y));
    return static_cast<int32_t>(lo & 0xffffu) - static_cast<int32_t>(lo >> 16) + hi;
}

// canonical residue of |y| < 98305 (fold -> [-2, 65537], then +-q)
__device__ __forceinline__ uint32_t canon_lz(int32_t y)
{
    const int32_t f = fold(y);
    const int32_t c = f < 0 ? f + 65537 : f;
    return static_cast<uint32_t>(c >= 65537 ? c - 65537 : c);
}

// x^(2^16 - 1) = x^-1 (x != 0) by the chain x^(2^2-1), x^(2^4-1),
// x^(2^8-1), x^(2^16-1): 15 squarings + 4 multiplies, all lazy
__device__ __forceinline__ uint32_t inv_lz(uint32_t xc)
{
    const int32_t x = balanced(xc);
    const int32_t e2 = mul_lz(mul_lz(x, x), x);        // x^3
    int32_t t = mul_lz(e2, e2);
    t = mul_lz(t, t);                                  // x^12
    const int32_t e4 = mul_lz(t, e2);                  // x^15
    t = e4;
#pragma unroll
    for (int i = 0; i < 4; i++)
        t = mul_lz(t, t);
    const int32_t e8 = mul_lz(t, e4);                  // x^255
    t = e8;
#pragma unroll
    for (int i = 0; i < 8; i++)
        t = mul_lz(t, t);
    return canon_lz(mul_lz(t, e8));                    // x^65535
}

// balanced 1 / s for the small row scales s of the rare rescale (the search
// tries s = 2, 3, ...; a powm per candidate had cost ~1 us of serial
// multiplies each, with the whole block waiting at the next barrier)
struct InvSmall {
    int32_t v[64];
};
constexpr InvSmall make_inv_small()
{
    InvSmall t{};
    for (uint32_t v = 1; v < 64; v++)
        t.v[v] = balanced(powmod_c(v, 65535u));
    return t;
}
__constant__ InvSmall kInvSmall = make_inv_small();
__device__ __forceinline__ int32_t inv_small(uint32_t sc)
{
    return sc < 64 ? kInvSmall.v[sc] : balanced(powm(sc, 65535u));
}

// Synthetic-division steps q <- c[t + 1] + x q for t = t_hi down to t_lo,
// f(t, q) after each (lazy: |c| <= 32768, |q| < 98400): eight coefficients
// loaded ahead per group, so the LDS latency is paid once per eight steps
// instead of on every step of the serial chain
template <class F>
__device__ __forceinline__ int32_t div_steps(const int32_t* c, int32_t x, int32_t q, int t_hi,
                                             int t_lo, F&& f)
{
    int t = t_hi;
    for (; t - 7 >= t_lo; t -= 8) {
        int32_t a[8];
#pragma unroll
        for (int u = 0; u < 8; u++)
            a[u] = c[t + 1 - u];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            q = a[u] + mul_lz(q, x);
            f(t - u, q);
        }
    }
    for (; t >= t_lo; t--) {
        q = c[t + 1] + mul_lz(q, x);
        f(t, q);
    }
    return q;
}

// NT threads: the Lagrange part runs on the first wave (lane = point); the
// row packing and the MFMA operand tiles use every thread (NT = 256 for
// k > 32, where they dominate and there are few stripes per launch).
// pack_row (matrix_pack.h) on a group of LPR adjacent lanes (a power of 2,
// <= 16), lane `sub` taking entries sub, sub + LPR, ...: the column scale
// 1 / A'(x_i) applied, the same row scale search (uniform in the group),
// packed pairs, canonical `plain` entries, kcorr / rscale / kmf, and the
// row-scaled entries written back to the LDS row for the tiles.  Entries
// lane-fastest: a group's global stores are runs of LPR dwords (4 lanes per
// row with 16-byte runs took 17 of the 43 us of a k = 64 context).
__device__ __forceinline__ uint32_t grp_or(uint32_t v, int lpr)
{
    for (int m = 1; m < lpr; m <<= 1)
        v |= __shfl_xor(v, m, lpr);
    return v;
}
__device__ __forceinline__ uint32_t grp_add(uint32_t v, int lpr)
{
    for (int m = 1; m < lpr; m <<= 1)
        v += __shfl_xor(v, m, lpr);
    return v;
}
__device__ __forceinline__ void pack_row_grp(uint32_t* row, const uint32_t* cscale, const MatLayout& L,
                             int t, int32_t* block, int sub, int lpr, bool dot2)
{
    // the lane's entries i = sub + m lpr (m < 16: k <= 256 at lpr = 16) in
    // registers: every row load is issued up front (rows in global memory
    // for k > 128), and the packed pairs take the odd entry from the
    // neighbour lane by shuffle instead of re-reading the row
    constexpr int ME = 16;
    const int kin = L.kin, KP = L.KP;
    uint32_t v[ME];
#pragma unroll
    for (int m = 0; m < ME; m++) {
        const int i = sub + m * lpr;
        v[m] = i < kin ? row[i] : 0u;
    }
    uint32_t bad = 0;
#pragma unroll
    for (int m = 0; m < ME; m++) {
        const int i = sub + m * lpr;
        if (i < kin) {
            v[m] = mulm(v[m], cscale[i]);
            bad |= !coef_ok(balanced(v[m]));
        }
    }
    bad = grp_or(bad, lpr);
    uint32_t s = 1;
    while (bad) {  // rare; s, si and bad are uniform in the group
        s++;
        const int32_t si = inv_small(s);
        if (iabs32(si) > 32766)
            continue;
        bad = 0;
#pragma unroll
        for (int m = 0; m < ME; m++) {
            const int i = sub + m * lpr;
            if (i < kin)
                bad |= !coef_ok(balanced(mulm(v[m], s)));
        }
        bad = grp_or(bad, lpr);
    }
    int32_t* packed = block + static_cast<size_t>(t) * KP;
    int32_t* plain = block + L.plain();
    uint32_t sum = 0;  // <= 256 * 65536 = 2^24
#pragma unroll
    for (int m = 0; m < ME; m++) {
        const int i = sub + m * lpr;
        if (s != 1 && i < kin)
            v[m] = mulm(v[m], s);
        // pair (i, i + 1) for even i: the odd entry sits on lane sub + 1
        const uint32_t odd = __shfl_xor(v[m], 1, lpr);
        if (i < kin) {
            row[i] = v[m];
            plain[static_cast<size_t>(t) * kin + i] = static_cast<int32_t>(v[m]);
            sum += v[m];
            if (dot2 && !(sub & 1)) {
                const int32_t lo = balanced(v[m]);
                const int32_t hi = i + 1 < kin ? balanced(odd) : 0;
                packed[i >> 1] = static_cast<int32_t>((static_cast<uint32_t>(lo) & 0xffffu) |
                                                      (static_cast<uint32_t>(hi) << 16));
            }
        }
    }
    // pairs past kin up to KP stay zero (the dot2 kernel's padding)
    for (int j = (kin + 1) / 2 + sub; dot2 && j < KP; j += lpr)
        packed[j] = 0;
    sum = grp_add(sum, lpr);
    if (sub == 0) {
        // sum mod q by two folds (2^16 = -1), then canonical
        int32_t f = static_cast<int32_t>(sum & 0xffffu) - static_cast<int32_t>(sum >> 16);
        f = f < 0 ? f + 65537 : f;
        const uint32_t sq = static_cast<uint32_t>(f >= 65537 ? f - 65537 : f);
        block[L.kcorr() + t] = static_cast<int32_t>(mulm(sq, 32768u));
        block[L.rscale() + t] = s == 1 ? 1 : inv_small(s);
        if (L.KS()) {
            block[L.kmf() + t] = static_cast<int32_t>(mulm(sq, 32896u));
            block[L.rscale_mf() + t] = block[L.rscale() + t];
        }
    }
}

// The BIG contexts' packing for whole-tile widths (see decode_ctx_kernel):
// rows t of Mt (canonical coef_t(Q_i), pitch kp, global memory) scaled by
// the columns' 1 / A'(x_i), row-scaled when an entry breaks coef_ok (as
// pack_row_grp: the row's scale search on its 32-lane group), summed into
// kcorr / kmf, and written as the [a | 0], [0 | b], [b | a] operand tiles.
// rows per chunk of the non-systematic k > 128 contexts (decode_ctx_kernel):
// (the kernel's static LDS + the largest chunk, ctx_chunk(k) rows x k
// entries, must fit kCtxLdsCap; launch_decode_ctx checks)
// 64 rows = 4 row blocks per packing pass at 16 lanes per row (32 rows at 32
// lanes: twice the passes and barriers for the same work; contexts k256
// 120 -> 114 us, k300 179 -> 161 us, k384 219 -> 206 us); 32 rows above
// k = 384 (a 64 x 640 chunk would not fit LDS)
constexpr int kCtxChunk = 64;

// a canonical entry a row may not hold unscaled (!coef_ok): the dot2
// kernel needs |balanced| <= 32766, the i8 split anything but 32640
__device__ __forceinline__ bool coef_bad(uint32_t e)
{
    return e - 32767u < 4u || e == 32640u;
}

// split_i8 of 4 canonical entries, entry jb's bytes into byte jb of aw / bw:
// v = 256 a + b in [-32896, 32639], b = the signed low byte of v (b's byte =
// v's low byte), a = (v - b) / 256 (a's byte = byte 1 of v - b); three byte
// permutes per word
__device__ __forceinline__ void split_i8_x4(const uint32_t (&e)[4], uint32_t& aw, uint32_t& bw)
{
    uint32_t vb[4], va[4];
#pragma unroll
    for (int jb = 0; jb < 4; jb++) {
        int32_t v = balanced(e[jb]);
        v = v > 32639 ? v - kQ : v;
        const int32_t b = (v << 24) >> 24;
        vb[jb] = static_cast<uint32_t>(v);
        va[jb] = static_cast<uint32_t>(v - b);
    }
    bw = __builtin_amdgcn_perm(__builtin_amdgcn_perm(vb[3], vb[2], 0x0c0c0400u),
                               __builtin_amdgcn_perm(vb[1], vb[0], 0x0c0c0400u), 0x05040100u);
    aw = __builtin_amdgcn_perm(__builtin_amdgcn_perm(va[3], va[2], 0x0c0c0501u),
                               __builtin_amdgcn_perm(va[1], va[0], 0x0c0c0501u), 0x05040100u);
}

__host__ __device__ inline int ctx_chunk(int k)
{
    return k > kMatGenMaxKin ? 32 : kCtxChunk;
}
constexpr int kCtxLdsCap = 160 * 1024;
// the packing stage's rows of (aw, bw) words (pitch 2 nj = 8 KS words, at
// most 64 rows x 192 or 32 rows x 320), aliased with the A(x) product tree's
// two level buffers (the tree is done before any packing)
constexpr int kPackStg = 12288;
constexpr int kTreeBuf = 2 * 512 + 4;
static_assert(2 * kTreeBuf <= kPackStg, "tree buffers inside the packing stage");

// One pass: NT / LPR rows from row block rb0 on (LPR lanes per row); row
// t's canonical entries i0 .. i0 + 3, already column-scaled by 1 / A'(x_i),
// from ent(t, i0, e).  stg: a row per pass row of the (aw, bw) words of each
// group (LDS).
template <int NT, int LPR, class Ent>
__device__ __forceinline__ void pack_tiles_pass(int rb0, const Ent& ent, const MatLayout& L,
                                int32_t* mat, uint32_t* stg_base)
{
    constexpr int ROWS = NT / LPR;
    // 16 lanes per row: the 64-row chunks of k <= 384; 32: k <= 640
    constexpr int MM = ((LPR <= 16 ? kMatGenMaxKin : kMatMaxKin) / 4 + LPR - 1) / LPR;
    static_assert(ROWS % 16 == 0, "whole row blocks per pass");
    const int k = L.kin, KS = L.KS(), KH = 16 * KS, nj = KH / 4, RB = L.RB();
    auto stg = [&](int r, int c) -> uint32_t& { return stg_base[r * 2 * nj + c]; };
    const int tid = threadIdx.x, sub = tid % LPR, rl = tid / LPR;
    int32_t* mf = mat + L.mf();
    {
        const int t = 16 * rb0 + rl;
        if (t < L.R) {
            uint32_t v[MM][4];
            uint32_t bad = 0;
#pragma unroll
            for (int m = 0; m < MM; m++) {
                const int i0 = 4 * (sub + m * LPR);
                uint32_t e[4] = {0u, 0u, 0u, 0u};
                if (i0 < k)
                    ent(t, i0, e);
#pragma unroll
                for (int jb = 0; jb < 4; jb++) {
                    const int i = i0 + jb;
                    v[m][jb] = i < k ? e[jb] : 0u;
                    bad |= coef_bad(v[m][jb]);  // (0 past k: never bad)
                }
            }
            bad = grp_or(bad, LPR);
            uint32_t sc = 1;
            while (bad) {  // rare; uniform in the group
                sc++;
                const int32_t si = inv_small(sc);
                if (iabs32(si) > 32766)
                    continue;
                bad = 0;
#pragma unroll
                for (int m = 0; m < MM; m++)
#pragma unroll
                    for (int jb = 0; jb < 4; jb++) {
                        const int i = 4 * (sub + m * LPR) + jb;
                        bad |= i < k && !coef_ok(balanced(mulm(v[m][jb], sc)));
                    }
                bad = grp_or(bad, LPR);
            }
            uint32_t sum = 0;
#pragma unroll
            for (int m = 0; m < MM; m++) {
                const int jg = sub + m * LPR;
                if (jg >= nj)
                    break;
                // (entries past k are 0: a = b = 0, nothing added)
                uint32_t c[4];
#pragma unroll
                for (int jb = 0; jb < 4; jb++) {
                    c[jb] = sc == 1 ? v[m][jb] : mulm(v[m][jb], sc);
                    sum += c[jb];
                }
                uint32_t aw, bw;
                split_i8_x4(c, aw, bw);
                {
                    stg(rl, 2 * jg) = aw;
                    stg(rl, 2 * jg + 1) = bw;
                }
            }
            sum = grp_add(sum, LPR);
            if (sub == 0) {
                int32_t f = static_cast<int32_t>(sum & 0xffffu) - static_cast<int32_t>(sum >> 16);
                f = f < 0 ? f + 65537 : f;
                const uint32_t sq = static_cast<uint32_t>(f >= 65537 ? f - 65537 : f);
                mat[L.kcorr() + t] = static_cast<int32_t>(mulm(sq, 32768u));
                const int32_t rs = sc == 1 ? 1 : inv_small(sc);
                mat[L.rscale() + t] = rs;
                mat[L.kmf() + t] = static_cast<int32_t>(mulm(sq, 32896u));
                mat[L.rscale_mf() + t] = rs;
            }
        } else {
            for (int jg = sub; jg < nj; jg += LPR)
                stg(rl, 2 * jg) = stg(rl, 2 * jg + 1) = 0;
        }
        __syncthreads();
        // the two row blocks' tile dwords, rows fastest (whole 128-byte tile
        // lines per wave store); zero halves of [a | 0] / [0 | b] not written
        // at KS >= 4 (never read)
        const int nrb = min(ROWS / 16, RB - rb0);
        for (int it = tid; it < nrb * nj * 16; it += NT) {
            const int tl = it & 15, jj = it >> 4;
            const int jg = jj % nj, rbl = jj / nj, rb = rb0 + rbl;
            const uint32_t aw = stg(16 * rbl + tl, 2 * jg), bw = stg(16 * rbl + tl, 2 * jg + 1);
#pragma unroll
            for (int half = 0; half < 2; half++) {
                const int K = half * KH + 4 * jg;
                const int ks = K >> 5, g = (K & 31) >> 3, dw = (K & 7) >> 2;
                const size_t base =
                    static_cast<size_t>((rb * KS + ks) * 3) * 128 + (16 * g + tl) * 2 + dw;
                if (KS < 4 || half == 0)
                    mf[base] = static_cast<int32_t>(half ? 0u : aw);        // [a | 0]
                if (KS < 4 || half == 1)
                    mf[base + 128] = static_cast<int32_t>(half ? bw : 0u);  // [0 | b]
                if (KS < 2)  // [b | a]: the kernels rebuild it at KS >= 2
                    mf[base + 256] = static_cast<int32_t>(half ? aw : bw);
            }
        }
        __syncthreads();
    }
}

// LDS row pitch of the context kernel's k x k matrix: 4 x odd, >= k
__host__ __device__ inline int ctx_pitch(int k)
{
    return (k + 3) / 8 * 8 + 4;
}

// The received fragments of stripe s in the context's order: for the
// systematic decodes (part) the data fragments (id < k) first, then the
// parity ones, each in the caller's order (a stable partition from ballot
// counts), so that the matrix kernels' two source regions meet at one
// position (matrix_os_kernel: one load per row).  The matrix columns, the
// route entries and the ids the decode reads (cids) all follow this order;
// identity otherwise.  NT threads, k <= NT; pid and wtot (NT / 64) in LDS.
template <int NT>
__device__ void order_ids(const uint16_t* sids, int k, bool part, uint16_t* pid, int* wtot)
{
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint16_t id = tid < k ? sids[tid] : uint16_t{0};
    if (!part) {  // block-uniform
        if (tid < k)
            pid[tid] = id;
        __syncthreads();
        return;
    }
    const bool lo = tid < k && id < k;
    const uint64_t b = __ballot(lo);
    const int before = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0)
        wtot[w] = __popcll(b);
    __syncthreads();
    int pre = before, P = 0;
#pragma unroll
    for (int v = 0; v < NT / 64; v++) {
        const int c = wtot[v];
        P += c;
        pre += v < w ? c : 0;
    }
    if (tid < k)
        pid[lo ? pre : P + (tid - pre)] = id;
    __syncthreads();
}

template <int NT, bool BIG>
__global__ __launch_bounds__(NT) void decode_ctx_kernel(
    int k, int n, uint32_t r, int mode, MatLayout L, const uint16_t* __restrict__ ids,
    int32_t* __restrict__ ctx, long long ctx_stride, Oor in_oor, int slot_base,
    int by_pos, long long words, int dot2, uint32_t* err, int nb)
{
    __shared__ uint32_t xs[kMatMaxKin];
    __shared__ uint32_t A[kMatMaxKin + 1];
    __shared__ uint32_t cinv[kMatMaxKin];    // 1 / A'(x_i)
    __shared__ uint32_t aprime[kMatMaxKin];  // A'(x_i)
    __shared__ uint16_t pid[kMatMaxKin];     // the ids in the context's order
    __shared__ int wtot[NT / 64];
    // k x k matrix, sized by the launch: 1 KiB at k = 16 instead of a fixed 32 KiB, which had
    // limited the kernel to 4 workgroups per CU
    extern __shared__ __attribute__((aligned(16))) uint32_t qi_ctx_lds[];
    // row pitch = 4 x odd (>= k, a multiple of 4 words): the tile pass
    // reads 16 rows x 16 bytes per wave (ds_read_b128) conflict-free (the
    // odd pitch k | 1 had SQ_LDS_BANK_CONFLICT at 7.4 cycles per LDS
    // instruction at k = 64)
    // nb blocks per stripe (the whole-tile forms only; nb = 1 otherwise):
    // block cb builds the row chunks [c0, c1) of its stripe's
    // matrix, block 0 also the ids and the route table; each computes A(x)
    // and the A'(x_i) itself (few stripes per launch left most CUs idle
    // behind one block per stripe: k300, 32 stripes, 147 us)
    const int s = blockIdx.x / nb, cb = blockIdx.x - s * nb;
    const int tid = threadIdx.x;
    int32_t* mat = ctx + s * ctx_stride;
    // BIG (128 < k <= 256): the k x k matrix (up to 256 KB) does not fit
    // LDS; its rows live in the context's own `plain` section (pitch k),
    // which the packing pass rewrites in place with the row-scaled entries
    const int kp = BIG ? k : ctx_pitch(k);
    uint32_t* Mt = BIG ? reinterpret_cast<uint32_t*>(mat + L.plain()) : qi_ctx_lds;
    int32_t* cids = mat + L.words();
    uint32_t* route = reinterpret_cast<uint32_t*>(cids + 2 * L.KP);
    const bool lead = cb == 0;  // block-uniform
    const long long ntiles = route_tiles(words);
    if (lead) {
        for (int i = k + tid; i < 2 * L.KP; i += NT)
            cids[i] = 0;
        // route table: clear, then (after the barrier below) fill; the
        // slow-tile list behind it starts empty.  A context built without
        // the buckets (ids only: init_context_dec, src/fec_context.h) marks
        // every tile unrouted (count > kRouteCap): a decode given marks then
        // scans the buckets itself
        const uint32_t rt0 = in_oor.counts ? 0u : static_cast<uint32_t>(kRouteCap) + 1u;
        for (long long t = tid; t < ntiles; t += NT)
            route[t * kRouteStride] = rt0;
        if (tid == 0) {
            route[ntiles * kRouteStride] = 0;
            route[lazy_word_off(words)] = 0;  // no lazily filled section yet
        }
    }
    order_ids<NT>(ids + static_cast<long long>(s) * k, k, mode != 0 && !by_pos, pid, wtot);
    if (tid < k) {
        const uint32_t id = pid[tid];
        xs[tid] = powm(r, id);
        if (lead) {
            cids[tid] = static_cast<int32_t>(id);
            if (id >= static_cast<uint32_t>(n))  // not a point of the code
                atomicOr(err, kErrBadIds);
        }
    }
    // the route-table clears (every thread of the lead block, above) must
    // have reached memory before any thread's atomicAdd below: each wave
    // waits for its own stores, then the barrier
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (lead && in_oor.counts && tid < k) {
        const int id = pid[tid];
        const int slot = (by_pos ? tid : id) - slot_base;
        // rows outside the bucket array (systematic data rows below
        // slot_base; bad ids past it) have no marks here
        if (slot >= 0 && slot < in_oor.slots) {
            const long long bk = static_cast<long long>(s) * in_oor.slots + slot;
            uint32_t c = in_oor.counts[bk];
            if (c > static_cast<uint32_t>(in_oor.cap)) {
                atomicOr(err, kErrOorTruncated);
                c = static_cast<uint32_t>(in_oor.cap);
            }
            for (uint32_t e = 0; e < c; e++) {
                const uint32_t w = in_oor.entries[bk * in_oor.cap + e];
                if (w >= words)
                    continue;
                uint32_t* rt = route + (w / kRouteTile) * kRouteStride;
                const uint32_t p = atomicAdd(rt, 1u);
                if (p < static_cast<uint32_t>(kRouteCap))
                    rt[1 + p] = (static_cast<uint32_t>(tid) << 16) | (w % kRouteTile);
            }
        }
    }
    // A(x) = prod_i (x - x_i) on wave 0: slot u of lane d holds coefficient
    // 64 u + d (u < nslot <= 6), lazy (folded once per step, |a| < 2^17):
    // the shift by DPP (wave_shr:1) with the slot carry by readlane, the
    // product as mul_lz, x_i by readlane from the lane-held points (the
    // ds_bpermute shifts and canonical mulm of round 2 took ~620 cycles per
    // step: 62 us of a k = 200 context).  A is monic: A[k] = 1 is set
    // explicitly, so k = 64 u needs no extra slot.  Stored balanced.
    // (BIG: the product tree's levels, then the split Horner chains of the
    // A'(x_i))
    __shared__ __attribute__((aligned(16))) uint32_t big_lds[BIG ? kPackStg : 2 * kTreeBuf];
    int32_t(*pt)[kTreeBuf] = reinterpret_cast<int32_t(*)[kTreeBuf]>(big_lds);
    if constexpr (BIG) {
        // k > 128: A(x) by a product tree instead of k dependent steps on one
        // wave (k = 256: 256 steps x 4 coefficient slots of DPP shifts and
        // products).  Leaves: wave w multiplies out the points [w g, w g +
        // g), g = ceil(k / 16) <= 24, as the k <= 64 kernel does (lane d
        // holds coefficient d; the shift by DPP, x_i by readlane).  Then 4
        // levels of pairwise products (16 -> 1 polynomials of span g 2^l
        // points, slots of g 2^l + 1 balanced coefficients): each pair's
        // outer product in 4 x 4 tiles, one per thread, its 7 anti-diagonal
        // sums added into the level by LDS atomics (|sum| < 2^24), then
        // folded and stored balanced; tiles past the children's true degrees
        // are skipped.  (One thread per coefficient of a 2-leaf tree left the
        // top levels serial: 257 + 129 + ... products, 31 of a k300
        // context's 147 us; the 9-level tiled tree still took 14.)
        constexpr int NWV = NT / 64;
        static_assert(NWV == 16, "16 leaf polynomials");
        const int g = (k + NWV - 1) / NWV;  // <= 24 (k <= 384)
        {
            const int w = tid >> 6, ln = tid & 63;
            const int p0 = w * g, cnt = max(0, min(k, p0 + g) - p0);
            const int32_t xv = ln < cnt ? balanced(xs[p0 + ln]) : 0;
            int32_t a = ln == 0 ? 1 : 0;
            for (int i = 0; i < cnt; i++) {
                const int32_t x = __builtin_amdgcn_readlane(xv, i);
                const int32_t prev = __builtin_amdgcn_update_dpp(0, a, 0x138, 0xf, 0xf, false);
                a = fold(prev - mul_lz(a, x));
            }
            if (ln <= g)
                pt[0][w * (g + 1) + ln] = balanced(canon_lz(a));
        }
        int cur = 0, D = g + 1, span = g;
        for (int m = NWV; m > 1; m >>= 1) {
            const int np = m / 2, D2 = 2 * D - 1;
            const int32_t* in = pt[cur];
            int32_t* out = pt[cur ^ 1];
            for (int it = tid; it < np * D2; it += NT)
                out[it] = 0;
            __syncthreads();
            // the live tiles only: rows u <= degL / 4, columns v <= degR / 4
            // of each pair (np <= 8 pairs, scanned per tile)
            auto deg = [&](int c) { return min(max(k - c * span, 0), span); };
            int total = 0;
            for (int pp = 0; pp < np; pp++)
                total += (deg(2 * pp) / 4 + 1) * (deg(2 * pp + 1) / 4 + 1);
            for (int it = tid; it < total; it += NT) {
                int pp = 0, r0 = it, tv = deg(1) / 4 + 1;
                for (int c = (deg(0) / 4 + 1) * tv; r0 >= c; c = (deg(2 * pp) / 4 + 1) * tv) {
                    r0 -= c;
                    pp++;
                    tv = deg(2 * pp + 1) / 4 + 1;
                }
                const int u = r0 / tv, v = r0 - u * tv;
                const int degL = deg(2 * pp), degR = deg(2 * pp + 1);
                const int32_t* Lp = in + (2 * pp) * D;
                const int32_t* Rp = Lp + D;
                int32_t la[4], rb[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    la[j] = 4 * u + j <= degL ? Lp[4 * u + j] : 0;
                    rb[j] = 4 * v + j <= degR ? Rp[4 * v + j] : 0;
                }
                int32_t acc[7];
#pragma unroll
                for (int d = 0; d < 7; d++)
                    acc[d] = 0;
#pragma unroll
                for (int a = 0; a < 4; a++)
#pragma unroll
                    for (int b = 0; b < 4; b++)
                        acc[a + b] += mul_lz(la[a], rb[b]);
                int32_t* o = out + pp * D2 + 4 * (u + v);
#pragma unroll
                for (int d = 0; d < 7; d++)
                    if (4 * (u + v) + d < D2)
                        atomicAdd(o + d, acc[d]);
            }
            __syncthreads();
            for (int it = tid; it < np * D2; it += NT)
                out[it] = balanced(canon_lz(fold(out[it])));
            __syncthreads();
            cur ^= 1;
            D = D2;
            span *= 2;
        }
        for (int i = tid; i < k; i += NT)
            A[i] = static_cast<uint32_t>(pt[cur][i]);
        if (tid == 0)
            A[k] = 1;
    } else if (tid < 64) {  // wave 0 (wave-uniform)
        constexpr int NS = kMatGenMaxKin / 64;
        const int nslot = (k + 63) / 64;
        int32_t xv[NS], au[NS];
#pragma unroll
        for (int u = 0; u < NS; u++) {
            const int i = 64 * u + tid;
            xv[u] = i < k ? balanced(xs[i]) : 0;
            au[u] = (u == 0 && tid == 0) ? 1 : 0;
        }
#pragma unroll
        for (int u = 0; u < NS; u++) {
            if (u >= nslot)
                break;
            const int cnt = min(64, k - 64 * u);
            for (int i0 = 0; i0 < cnt; i0++) {
                const int32_t x = __builtin_amdgcn_readlane(xv[u], i0);
                int32_t prev[NS];
#pragma unroll
                for (int v = 0; v < NS; v++) {
                    if (v >= nslot)
                        break;
                    prev[v] = __builtin_amdgcn_update_dpp(0, au[v], 0x138, 0xf, 0xf, false);
                    if (v > 0) {
                        const int32_t top = __builtin_amdgcn_readlane(au[v - 1], 63);
                        prev[v] = tid == 0 ? top : prev[v];
                    }
                }
#pragma unroll
                for (int v = 0; v < NS; v++) {
                    if (v >= nslot)
                        break;
                    au[v] = fold(prev[v] - mul_lz(au[v], x));
                }
            }
        }
#pragma unroll
        for (int u = 0; u < NS; u++) {
            const int i = 64 * u + tid;
            if (u < nslot && i < k)
                A[i] = static_cast<uint32_t>(balanced(canon_lz(au[u])));
        }
        if (tid == 0)
            A[k] = 1;
    }
    __syncthreads();
    // (the chunked BIG rows are written by a second division below)
    const bool rows = mode == 0 && !(BIG && !dot2);
    if (BIG && !rows) {
        // only the A'(x_i): the derivative's coefficients d_j = (j + 1)
        // A[j + 1], then PP = NT / k threads per point, each a Horner chain
        // over a k / PP slice of them, combined with powers x^len (the one
        // k-step chain per point took 17 of a k300 context's 147 us)
        int32_t* dA = pt[0];
        int32_t* part = pt[1];
        const int32_t* Ab = reinterpret_cast<const int32_t*>(A);
        for (int j = tid; j < k; j += NT)
            dA[j] = balanced(canon_lz(mul_lz(j + 1, Ab[j + 1])));
        __syncthreads();
        const int PP = NT / k, len = (k + PP - 1) / PP;
        if (tid < PP * k) {
            const int pq = tid / k, i = tid - pq * k;
            const int32_t x = balanced(xs[i]);
            const int lo = pq * len, hi = min(k, lo + len);
            // h <- dA[j] + x h for j = hi - 1 .. lo (|h| < 98400)
            part[pq * k + i] = div_steps(dA - 1, x, 0, hi - 1, lo, [](int, int32_t) {});
        }
        __syncthreads();
        if (tid < k) {
            const int32_t x = balanced(xs[tid]);
            int32_t xl = 1, b = x;
            for (int e = len; e; e >>= 1) {
                if (e & 1)
                    xl = mul_lz(xl, b);
                b = mul_lz(b, b);
            }
            int32_t h = part[(PP - 1) * k + tid];
            for (int pq = PP - 2; pq >= 0; pq--)
                h = fold(part[pq * k + tid] + mul_lz(h, xl));
            const uint32_t ap = canon_lz(fold(h));
            aprime[tid] = ap;
            cinv[tid] = inv_lz(ap);
            if (ap == 0u)  // x_i = x_j for some j != i: repeated ids
                atomicOr(err, kErrBadIds);
        }
    } else if (tid < k) {
        // Q_i = A / (x - x_i) by synthetic division from the top, and
        // A'(x_i) = Q_i(x_i) by Horner beside it (two interleaved chains),
        // lazy as in decode_ctx_lds_kernel (|q| < 98400, |h| < 2^18); the
        // rows get canonical q (off the chain).  The column scale
        // 1 / A'(x_i) is applied by the packing pass.
        const int32_t xi = balanced(xs[tid]);
        const int32_t* Ab = reinterpret_cast<const int32_t*>(A);
        int32_t q = 1, h = 1;  // A[k]; Q_i(x_i) so far
        if (rows)
            Mt[(k - 1) * kp + tid] = 1;
        for (int j = k - 1; j >= 1; j--) {
            q = Ab[j] + mul_lz(q, xi);
            if (rows)
                Mt[(j - 1) * kp + tid] = canon_lz(q);
            h = q + mul_lz(h, xi);
        }
        const uint32_t ap = canon_lz(fold(h));
        aprime[tid] = ap;
        cinv[tid] = inv_lz(ap);
        if (ap == 0u)  // repeated ids
            atomicOr(err, kErrBadIds);
    }
    if (mode != 0 && !(BIG && !dot2)) {
        // systematic: M[t][i] = Q_i(r^t) / A'(x_i), one thread per row t,
        // with Q_i(r^t) = A(r^t) / (r^t - x_i): 0 when r^t is another
        // received point (A(r^t) = 0), A'(x_i) when it is x_i itself.  The
        // k inverses of a row come from one inversion (prefix products, the
        // running inverse walked back), so a row costs ~3k + 24 serial
        // multiplies (Horner of every Q_i at every r^t took k^2 per lane).
        __syncthreads();
        if (tid < k) {
            uint32_t* row = Mt + tid * kp;
            const uint32_t et = powm(r, static_cast<uint32_t>(tid));
            // A(r^t) by a lazy Horner chain over the balanced A (A monic)
            const int32_t* Ab = reinterpret_cast<const int32_t*>(A);
            const int32_t eb = balanced(et);
            int32_t al = 1;
            for (int j = k - 1; j >= 0; j--)
                al = Ab[j] + mul_lz(al, eb);
            const uint32_t av = canon_lz(fold(al));
            uint32_t pre = 1;
            for (int i = 0; i < k; i++) {
                const uint32_t d = subm(et, xs[i]);
                row[i] = pre;
                pre = mulm(pre, d ? d : 1u);
            }
            uint32_t inv = powm(pre, 65535u);
            for (int i = k - 1; i >= 0; i--) {
                const uint32_t d = subm(et, xs[i]);
                const uint32_t inv_i = mulm(inv, row[i]);
                inv = mulm(inv, d ? d : 1u);
                row[i] = d ? mulm(av, inv_i) : aprime[i];
            }
        }
    }
    __syncthreads();
    if constexpr (BIG) {
        uint32_t* stg = big_lds;  // the tree's buffers are dead now
        if (!dot2) {
            // whole-tile widths: the rows in chunks of CH (ctx_chunk), this
            // block's chunks [c0, c1) of the stripe's nb blocks, never in
            // global memory: each chunk's rows written into LDS, then its row
            // blocks packed straight into the operand tiles (LPR lanes per
            // row, 4 entries per lane and group: split, staged, stored
            // rows-fastest as whole tile lines).  The rows are written
            // column-scaled by 1 / A'(x_i) (off the chains, so the packing
            // pass does no multiplies).  No `plain` rows, no dot2 section (the
            // kernels take single coefficients from the tiles).
            //   non-systematic: thread i runs Q_i's synthetic division again
            // (1 / A'(x_i) is known now), from the top down through the rows
            // above the block's chunks without keeping them.
            //   systematic: row t is Q_i(r^t) = A(r^t) / (r^t - x_i), or
            // A'(x_i) where r^t = x_i (scaled: 1).  TPR lanes per row: each evaluates a segment of A's
            // k + 1 coefficients at r^t (the segments summed across the group
            // by shuffles) and inverts a seg-entry slice of the row's r^t - x_i
            // at once (prefix products, one inversion, walked back).  (One
            // thread per row, the rows through `plain`, one block per stripe:
            // k600 systematic context 0.99 ms at 16 stripes.)
            uint32_t* ch = qi_ctx_lds;  // CH x kpc
            const int CH = ctx_chunk(k);
            const int kpc = (k + 3) & ~3;
            const int nch = (k + CH - 1) / CH;
            const int c0 = (cb * nch + nb - 1) / nb, c1 = ((cb + 1) * nch + nb - 1) / nb;
            const int32_t* Ab = reinterpret_cast<const int32_t*>(A);
            const int32_t xi = tid < k ? balanced(xs[tid]) : 0;
            int32_t q = 1;  // coef_{k-1}(Q_i)
            if (mode == 0 && tid < k)
                q = div_steps(Ab, xi, q, k - 2, CH * c1, [](int, int32_t) {});
            const int TPR = NT / CH;  // 16 or 32: a row's lanes share a wave
            for (int c = c1 - 1; c >= c0; c--) {
                const int lo = CH * c, hi = min(k, lo + CH);
                if (mode == 0) {
                    if (tid < k) {
                        const int32_t ci = balanced(cinv[tid]);
                        auto keep = [&](int t, int32_t qt) {
                            ch[(t - lo) * kpc + tid] = canon_lz(mul_lz(qt, ci));
                        };
                        if (hi == k)
                            keep(k - 1, q);
                        q = div_steps(Ab, xi, q, hi == k ? k - 2 : hi - 1, lo, keep);
                    }
                } else if (lo + tid / TPR < k) {  // uniform in the row's lane group
                    const int sub = tid % TPR, rl = tid / TPR, t = lo + rl;
                    const int len = (k + TPR) / TPR;      // ceil((k + 1) / TPR)
                    const int seg = (k + TPR - 1) / TPR;  // ceil(k / TPR)
                    const uint32_t et = powm(r, static_cast<uint32_t>(t));
                    const int j0 = sub * len, j1 = min(k + 1, j0 + len);
                    uint32_t term = 0;
                    if (j0 < j1) {
                        // sum_{j0 <= j < j1} A[j] (r^t)^(j - j0), times (r^t)^j0
                        const int32_t h = div_steps(Ab - 1, balanced(et), 0, j1 - 1, j0,
                                                    [](int, int32_t) {});
                        term = mulm(canon_lz(fold(h)), powm(et, static_cast<uint32_t>(j0)));
                    }
                    const uint32_t av = grp_add(term, TPR) % 65537u;  // A(r^t)
                    uint32_t* row = ch + rl * kpc;
                    const int i0 = sub * seg, i1 = min(k, i0 + seg);
                    uint32_t pre = 1;
                    for (int i = i0; i < i1; i++) {
                        const uint32_t d = subm(et, xs[i]);
                        row[i] = pre;
                        pre = mulm(pre, d ? d : 1u);
                    }
                    uint32_t inv = powm(pre, 65535u);
                    for (int i = i1 - 1; i >= i0; i--) {
                        const uint32_t d = subm(et, xs[i]);
                        const uint32_t inv_i = mulm(inv, row[i]);
                        inv = mulm(inv, d ? d : 1u);
                        row[i] = d ? mulm(mulm(av, inv_i), cinv[i]) : 1u;
                    }
                }
                __syncthreads();
                auto ent = [&](int t, int i0, uint32_t (&e)[4]) {
                    const uint4 v = *reinterpret_cast<const uint4*>(ch + (t - lo) * kpc + i0);
                    e[0] = v.x;
                    e[1] = v.y;
                    e[2] = v.z;
                    e[3] = v.w;
                };
                // (ends with a barrier: the chunk buffer is free again)
                if (CH == kCtxChunk)
                    pack_tiles_pass<NT, NT / kCtxChunk>(lo >> 4, ent, L, mat, stg);
                else
                    pack_tiles_pass<NT, NT / 32>(lo >> 4, ent, L, mat, stg);
            }
            return;
        }
    }
    {
        // LPR lanes per row: 4 entries per lane at k = 64
        // (16 entries per lane: lpr = 32 covers k <= 512)
        const int q4 = (k + 3) / 4;
        const int lpr = q4 <= 4 ? 4 : q4 <= 8 ? 8 : q4 <= 16 ? 16 : 32;
        for (int t = tid / lpr; t < L.R; t += NT / lpr)
            pack_row_grp(Mt + t * kp, cinv, L, t, mat, tid & (lpr - 1), lpr, dot2 != 0);
    }
    if (L.KS()) {
        // the matrix-core operand tiles, from the row-scaled entries in LDS
        __syncthreads();
        // per (row t, 4 consecutive entries): split once, then place the
        // a / b byte words in their tile dwords (pack_mf_dword's layout;
        // rows t >= R are zero).  Items run row-fastest, so 16 lanes read
        // 16 rows' entries i0..i0+3 (one ds_read_b128 each) and a wave's
        // stores cover whole 128-byte tile lines (16 rows x 2 dwords).  At
        // KS >= 4 the zero halves of [a | 0] and [0 | b] are not written:
        // matrix_mfma_kernel skips those K-steps (and never loads them).
        const int KS = L.KS(), KH = 16 * KS, nj = KH / 4, RB = L.RB();
        int32_t* mf = mat + L.mf();
        // BIG: the rows come from global memory; 4 items per thread have
        // their loads in flight together (the stores to the tiles may alias
        // the rows as far as the compiler knows, so it would not overlap
        // the iterations itself)
        constexpr int IB = BIG ? 4 : 1;
        const int items = RB * nj * 16;
        for (int it0 = tid; it0 < items; it0 += IB * NT) {
            uint32_t e[IB][4];
#pragma unroll
            for (int ib = 0; ib < IB; ib++) {
                const int it = it0 + ib * NT;
                const int tl4 = it & 15, jj = it >> 4;
                const int t = 16 * (jj / nj) + tl4, i0 = 4 * (jj % nj);
                const bool live = it < items && t < L.R && i0 < k;
                if constexpr (BIG) {  // global rows, pitch k: no 16-byte alignment
#pragma unroll
                    for (int jb = 0; jb < 4; jb++)
                        e[ib][jb] = live && i0 + jb < k ? Mt[t * kp + i0 + jb] : 0u;
                } else if (live) {
                    const uint4 e4 = *reinterpret_cast<const uint4*>(Mt + t * kp + i0);
                    e[ib][0] = e4.x;
                    e[ib][1] = e4.y;
                    e[ib][2] = e4.z;
                    e[ib][3] = e4.w;
                }
            }
#pragma unroll
            for (int ib = 0; ib < IB; ib++) {
                const int it = it0 + ib * NT;
                if (it >= items)
                    break;
                const int tl4 = it & 15, jj = it >> 4;
                const int j = jj % nj, rb = jj / nj;
                const int t = 16 * rb + tl4, i0 = 4 * j;
                uint32_t aw = 0, bw = 0;
                if (t < L.R && i0 < k) {
#pragma unroll
                    for (int jb = 0; jb < 4; jb++) {
                        if (i0 + jb < k) {
                            int32_t a, b;
                            split_i8(e[ib][jb], a, b);
                            aw |= (static_cast<uint32_t>(a) & 0xffu) << (8 * jb);
                            bw |= (static_cast<uint32_t>(b) & 0xffu) << (8 * jb);
                        }
                    }
                }
#pragma unroll
                for (int half = 0; half < 2; half++) {
                    const int K = half * KH + i0;
                    const int ks = K >> 5, g = (K & 31) >> 3, dw = (K & 7) >> 2;
                    const size_t base =
                        static_cast<size_t>((rb * KS + ks) * 3) * 128 + (16 * g + tl4) * 2 + dw;
                    if (KS < 4 || half == 0)
                        mf[base] = static_cast<int32_t>(half ? 0u : aw);        // [a | 0]
                    if (KS < 4 || half == 1)
                        mf[base + 128] = static_cast<int32_t>(half ? bw : 0u);  // [0 | b]
                    if (KS < 2)  // [b | a]: the kernels rebuild it at KS >= 2
                    mf[base + 256] = static_cast<int32_t>(half ? aw : bw);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// k <= 128: the whole context in LDS, every serial chain short and lazy.
//   - x_i = r^{id_i} from the plan's power table (one load, no powm chain);
//   - A(x) on wave 0, one coefficient (two for k > 64) per lane, the shift
//     by DPP (wave_shr:1) and the product x_i a_j as mul_rt (48-bit product,
//     2^32 = 1 and 2^16 = -1) folded once per step: no canonical reductions
//     on the chain; the route table is filled by the other waves meanwhile;
//   - Q_i and A'(x_i) by the same lazy Horner chains (q, h stay below 2^18);
//     1 / A'(x_i) by a 19-multiply addition chain of x^(2^16 - 1);
//   - the column scale, the row-scale test, the row sums, the operand tiles
//     and the plain / packed rows in item passes (thread = 4 entries of one
//     row, rows fastest), with the rare row rescale done by one lane.
// The round-2 kernel spent 23 of its 47 us (k = 64) in its row packing
// (shuffle reductions per row group) and 14 in the A(x) / Q chains
// (ds_bpermute shifts, canonical mulm at every step).
// ---------------------------------------------------------------------------
// r^(2^b), balanced, b < 16: x = r^id by at most log2(n) multiplies
struct RPow2 {
    int32_t v[16];
};

__device__ __forceinline__ int32_t rpow_lz(const RPow2& rp, uint32_t e, int lgn)
{
    int32_t acc = 1;
    for (int b = 0; b < lgn; b++)
        acc = (e >> b) & 1u ? mul_lz(acc, rp.v[b]) : acc;
    return acc;  // lazy, |acc| < 65600
}

template <int NT>
__global__ __launch_bounds__(NT) void decode_ctx_lds_kernel(
    int k, RPow2 rp, int lgn, int mode, MatLayout L,
    const uint16_t* __restrict__ ids, int32_t* __restrict__ ctx, long long ctx_stride,
    Oor in_oor, int slot_base, int by_pos, long long words, int dot2, uint32_t* err)
{
    __shared__ uint32_t xs[128];
    __shared__ int32_t A[129];        // balanced coefficients of A(x)
    __shared__ __attribute__((aligned(16))) int32_t cinv[128];  // 1 / A'(x_i), balanced
    __shared__ uint32_t aprime[128];  // A'(x_i)
    __shared__ uint16_t pid[128];     // the ids in the context's order
    __shared__ int wtot[NT / 64];
    extern __shared__ __attribute__((aligned(16))) uint32_t qi_ctx_lds[];
    const int s = blockIdx.x;
    const int tid = threadIdx.x;
    int32_t* mat = ctx + s * ctx_stride;
    const int kp = ctx_pitch(k);
    uint32_t* Mt = qi_ctx_lds;
    int32_t* cids = mat + L.words();
    uint32_t* route = reinterpret_cast<uint32_t*>(cids + 2 * L.KP);
    const long long ntiles = route_tiles(words);

    for (int i = k + tid; i < 2 * L.KP; i += NT)
        cids[i] = 0;
    // the route table belongs to the routing waves (1 .. NT / 64 - 1, while
    // wave 0 builds A(x), below): tile t to wave 1 + t % nrw, which clears
    // its count and then adds its marks -- a count cleared by another wave
    // could land after marks were added (no barrier ahead of the chain)
    constexpr int nrw = NT / 64 - 1;
    const int rw = (tid >> 6) - 1, rl = tid & 63;
    if (tid >= 64) {
        // (ids only, no buckets: every tile unrouted, as decode_ctx_kernel)
        const uint32_t rt0 = in_oor.counts ? 0u : static_cast<uint32_t>(kRouteCap) + 1u;
        for (long long t = rw + static_cast<long long>(nrw) * rl; t < ntiles; t += 64 * nrw)
            route[t * kRouteStride] = rt0;
        if (tid == 64) {
            route[ntiles * kRouteStride] = 0;  // the slow-tile list starts empty
            route[lazy_word_off(words)] = 0;   // no lazily filled section yet
        }
        __builtin_amdgcn_s_waitcnt(0);  // this wave's clears before its atomics
    }
    order_ids<NT>(ids + static_cast<long long>(s) * k, k, mode != 0 && !by_pos, pid, wtot);
    // x_i = r^{id_i}: thread tid takes point tid (its Q chain below); wave 0
    // also point 64 + lane (its A(x) chain reads every point by readlane)
    int32_t xt = 0, xt1 = 0;
    if (tid < k) {
        const uint32_t id = pid[tid];
        xt = balanced(canon_lz(rpow_lz(rp, id, lgn)));
        xs[tid] = static_cast<uint32_t>(xt < 0 ? xt + kQ : xt);
        cids[tid] = static_cast<int32_t>(id);
        if (id >= (1u << lgn))  // not a point of the code
            atomicOr(err, kErrBadIds);
    }
    if (tid < 64 && 64 + tid < k)
        xt1 = balanced(canon_lz(rpow_lz(rp, pid[64 + tid], lgn)));
    int32_t ab0 = 0;  // wave 0: balanced A[lane] (k <= 64), for the Q chains
    if (tid < 64) {
        // A(x) = prod_i (x - x_i): lane d holds coefficient d (a0) and
        // 64 + d (a1, k > 64); A is monic, A[k] = 1 set below.  x_i by
        // readlane (no LDS round trip on the chain)
        int32_t a0 = tid == 0 ? 1 : 0, a1 = 0;
        if (k <= 64) {
            for (int i = 0; i < k; i++) {
                const int32_t x = __builtin_amdgcn_readlane(xt, i);
                const int32_t prev = __builtin_amdgcn_update_dpp(0, a0, 0x138, 0xf, 0xf, false);
                a0 = fold(prev - mul_lz(a0, x));
            }
        } else {
            for (int i = 0; i < k; i++) {
                const int32_t x = i < 64 ? __builtin_amdgcn_readlane(xt, i)
                                         : __builtin_amdgcn_readlane(xt1, i - 64);
                const int32_t top = __builtin_amdgcn_readlane(a0, 63);
                const int32_t p0 = __builtin_amdgcn_update_dpp(0, a0, 0x138, 0xf, 0xf, false);
                int32_t p1 = __builtin_amdgcn_update_dpp(0, a1, 0x138, 0xf, 0xf, false);
                p1 = tid == 0 ? top : p1;
                a0 = fold(p0 - mul_lz(a0, x));
                a1 = fold(p1 - mul_lz(a1, x));
            }
            if (64 + tid < k)
                A[64 + tid] = balanced(canon_lz(a1));
        }
        ab0 = balanced(canon_lz(a0));
        if (tid < k)
            A[tid] = ab0;
        if (tid == 0)
            A[k] = 1;
    } else if (in_oor.counts) {
        // route the received rows' OOR marks into per-tile tables (the
        // other waves, while wave 0 builds A(x)): every row's marks, each
        // wave adding those of its own tiles
        for (int i = rl; i < k; i += 64) {
            const int id = pid[i];
            const int slot = (by_pos ? i : id) - slot_base;
            if (slot < 0 || slot >= in_oor.slots)
                continue;
            const long long bk = static_cast<long long>(s) * in_oor.slots + slot;
            uint32_t c = in_oor.counts[bk];
            if (c > static_cast<uint32_t>(in_oor.cap)) {
                atomicOr(err, kErrOorTruncated);
                c = static_cast<uint32_t>(in_oor.cap);
            }
            for (uint32_t e = 0; e < c; e++) {
                const uint32_t w = in_oor.entries[bk * in_oor.cap + e];
                if (w >= words || static_cast<int>((w / kRouteTile) % nrw) != rw)
                    continue;
                uint32_t* rt = route + (w / kRouteTile) * kRouteStride;
                const uint32_t p = atomicAdd(rt, 1u);
                if (p < static_cast<uint32_t>(kRouteCap))
                    rt[1 + p] = (static_cast<uint32_t>(i) << 16) | (w % kRouteTile);
            }
        }
    }
    __syncthreads();
    if (tid < k) {
        // Q_i = A / (x - x_i) by synthetic division from the top, and
        // A'(x_i) = Q_i(x_i) by Horner beside it; lazy: |q| < 98400,
        // |h| < 2^18 (the rows keep the lazy q, scaled and made canonical
        // by the item pass).  k <= 64: A[j] by readlane from wave 0's
        // registers
        const int32_t x = xt;
        int32_t q = 1, h = 1;
        if (mode == 0)
            Mt[(k - 1) * kp + tid] = 1;
        if (k <= 64) {
            // four coefficients per dependent step: from q = q_j,
            //   q_{j-m} = c_m + x^m q_j,  c_1 = A[j], c_m = A[j-m+1] + x c_{m-1}
            // (the c_m off the chain), and Horner's h the same way:
            //   h' = q_{j-4} + x q_{j-3} + x^2 q_{j-2} + x^3 q_{j-1} + x^4 h
            // (33 <= k <= 64; at k <= 32 the short chains measured faster
            // one coefficient per step)
            int j = k - 1;
            if constexpr (NT == 256) {
                const int32_t x2 = balanced(canon_lz(mul_lz(x, x)));
                const int32_t x3 = balanced(canon_lz(mul_lz(x2, x)));
                const int32_t x4 = balanced(canon_lz(mul_lz(x2, x2)));
                for (; j >= 4; j -= 4) {
                    const int32_t A1 = __builtin_amdgcn_readlane(ab0, j);
                    const int32_t A2 = __builtin_amdgcn_readlane(ab0, j - 1);
                    const int32_t A3 = __builtin_amdgcn_readlane(ab0, j - 2);
                    const int32_t A4 = __builtin_amdgcn_readlane(ab0, j - 3);
                    const int32_t c2 = A2 + mul_lz(x, A1);
                    const int32_t c3 = A3 + mul_lz(x, c2);
                    const int32_t c4 = A4 + mul_lz(x, c3);
                    const int32_t q1 = fold(A1 + mul_lz(x, q));
                    const int32_t q2 = fold(c2 + mul_lz(x2, q));
                    const int32_t q3 = fold(c3 + mul_lz(x3, q));
                    const int32_t q4 = fold(c4 + mul_lz(x4, q));
                    if (mode == 0) {
                        Mt[(j - 1) * kp + tid] = static_cast<uint32_t>(q1);
                        Mt[(j - 2) * kp + tid] = static_cast<uint32_t>(q2);
                        Mt[(j - 3) * kp + tid] = static_cast<uint32_t>(q3);
                        Mt[(j - 4) * kp + tid] = static_cast<uint32_t>(q4);
                    }
                    const int32_t hs = q4 + mul_lz(x, q3) + mul_lz(x2, q2) + mul_lz(x3, q1);
                    h = fold(hs + mul_lz(x4, h));
                    q = q4;
                }
            }
            for (; j >= 1; j--) {
                q = __builtin_amdgcn_readlane(ab0, j) + mul_lz(q, x);
                if (mode == 0)
                    Mt[(j - 1) * kp + tid] = static_cast<uint32_t>(q);
                h = q + mul_lz(h, x);
            }
        } else {
            for (int j = k - 1; j >= 1; j--) {
                q = A[j] + mul_lz(q, x);
                if (mode == 0)
                    Mt[(j - 1) * kp + tid] = static_cast<uint32_t>(q);
                h = q + mul_lz(h, x);
            }
        }
        const uint32_t ap = canon_lz(fold(h));
        aprime[tid] = ap;
        cinv[tid] = balanced(inv_lz(ap));
        if (ap == 0u)  // repeated ids
            atomicOr(err, kErrBadIds);
    }
    if (mode != 0) {
        // systematic: M[t][i] = Q_i(r^t) / A'(x_i), Q_i(r^t) = A(r^t) / (r^t -
        // x_i) (0 when r^t is another received point, A'(x_i) when it is
        // x_i).  TPR lanes per row t (2..8: all NT threads busy): each
        // evaluates a segment of A's k + 1 coefficients at r^t (summed over
        // the group by shuffles) and inverts a slice of the row's r^t - x_i
        // at once (prefix products, one inversion, walked back).  (One
        // thread per row ran the k-step chains serially: cfg3 systematic
        // context 52 us against 27 us non-systematic.)
        __syncthreads();
        const int TPR = NT >= 8 * k ? 8 : NT >= 4 * k ? 4 : NT >= 2 * k ? 2 : 1;
        const int t = tid / TPR, sub = tid % TPR;
        if (t < k) {  // uniform in the row's lane group
            uint32_t* row = Mt + t * kp;
            const uint32_t et = canon_lz(rpow_lz(rp, static_cast<uint32_t>(t), lgn));
            const int len = (k + TPR) / TPR;  // ceil((k + 1) / TPR)
            const int j0 = sub * len, j1 = min(k + 1, j0 + len);
            uint32_t part = 0;  // sum_{j0 <= j < j1} A[j] (r^t)^(j - j0); A[k] = 1
            for (int j = j1 - 1; j >= j0; j--)
                part = canon_lz(fold(mul_lz(balanced(part), balanced(et)) + A[j]));
            const uint32_t term = j0 < j1 ? mulm(part, powm(et, static_cast<uint32_t>(j0))) : 0u;
            const uint32_t av = grp_add(term, TPR) % 65537u;  // A(r^t)
            const int seg = (k + TPR - 1) / TPR;
            const int i0 = sub * seg, i1 = min(k, i0 + seg);
            uint32_t pre = 1;
            for (int i = i0; i < i1; i++) {
                const uint32_t d = et >= xs[i] ? et - xs[i] : et + 65537u - xs[i];
                row[i] = pre;
                pre = canon_lz(mul_lz(balanced(pre), balanced(d ? d : 1u)));
            }
            uint32_t inv = inv_lz(pre);
            for (int i = i1 - 1; i >= i0; i--) {
                const uint32_t d = et >= xs[i] ? et - xs[i] : et + 65537u - xs[i];
                const uint32_t inv_i = canon_lz(mul_lz(balanced(inv), balanced(row[i])));
                inv = canon_lz(mul_lz(balanced(inv), balanced(d ? d : 1u)));
                row[i] = d ? canon_lz(mul_lz(balanced(av), balanced(inv_i))) : aprime[i];
            }
        }
    }
    __syncthreads();
    // one pass per row, 4 lanes per row (quad reductions by DPP), lane sub
    // holding the 4-entry groups i0 = 4 sub + 16 m in registers: the column
    // scale 1 / A'(x_i), the row sum and scale test, the rare rescale (a row
    // needs a unit scale with probability ~5 k / 65537, i.e. ~27 % of the
    // stripes at k = 64, so it runs on the quad too: s = 2, 3, ... as
    // pack_row), kcorr / rscale / kmf, and the row's operand tiles.  (Round
    // 5 ran three passes with a barrier between each: column scale by
    // items, rows, tiles by items.)
    const int KS = L.KS(), KH = 16 * KS, RB = L.RB();
    int32_t* mf = mat + L.mf();
    {
        constexpr int MG = 8;  // k <= 128: at most 8 groups per lane
        const int sub = tid & 3;
        for (int t0 = 0; t0 < 16 * RB || t0 < L.R; t0 += NT / 4) {
            const int t = t0 + tid / 4;
            uint32_t* row = Mt + t * kp;
            uint32_t sum = 0, bad = 0;
            uint4 ev[MG];
#pragma unroll
            for (int m = 0; m < MG; m++) {
                const int i0 = 4 * sub + 16 * m;
                ev[m] = uint4{0u, 0u, 0u, 0u};
                if (t < L.R && i0 < k) {
                    const uint4 e4 = *reinterpret_cast<const uint4*>(row + i0);
                    const int4 c4 = *reinterpret_cast<const int4*>(cinv + i0);
                    uint32_t e[4] = {e4.x, e4.y, e4.z, e4.w};
                    const int32_t c[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
                    for (int jb = 0; jb < 4; jb++) {
                        // canonical by one min3: fold(y) is in [-q, 2q)
                        const int32_t f = fold(mul_lz(static_cast<int32_t>(e[jb]), c[jb]));
                        const uint32_t fu = static_cast<uint32_t>(f);
                        e[jb] = i0 + jb < k ? min(min(fu, fu + 65537u), fu - 65537u) : 0u;
                        sum += e[jb];
                        bad |= coef_bad(e[jb]);
                    }
                    ev[m] = uint4{e[0], e[1], e[2], e[3]};
                }
            }
            bad |= __builtin_amdgcn_update_dpp(0u, bad, 0xB1, 0xf, 0xf, false);
            bad |= __builtin_amdgcn_update_dpp(0u, bad, 0x4E, 0xf, 0xf, false);
            // the scaled row back to LDS only where it is read again: the
            // rare rescale below (quad-uniform) and the dot2 sections
            if (bad || dot2) {
#pragma unroll
                for (int m = 0; m < MG; m++) {
                    const int i0 = 4 * sub + 16 * m;
                    if (t < L.R && i0 < k)
                        *reinterpret_cast<uint4*>(row + i0) = ev[m];
                }
            }
            int32_t rs = 1;
            if (bad) {  // quad-uniform, rare; the quad's scaled entries are in
                        // LDS (one wave: its LDS accesses complete in order)
                uint32_t sc = 0;
                for (uint32_t cand = 2; cand < 256 && !sc; cand++) {
                    // |s^-1| <= 32766 (the epilogue's v_mul_i32_i24)
                    const int32_t ci = inv_small(cand);
                    if (iabs32(ci) > 32766)
                        continue;
                    uint32_t fail = 0;
                    for (int i = sub; i < k; i += 4)
                        fail |= coef_bad(canon_lz(static_cast<int32_t>(row[i] * cand)));
                    fail |= __builtin_amdgcn_update_dpp(0u, fail, 0xB1, 0xf, 0xf, false);
                    fail |= __builtin_amdgcn_update_dpp(0u, fail, 0x4E, 0xf, 0xf, false);
                    if (!fail) {
                        sc = cand;
                        rs = ci;
                    }
                }
                if (!sc)  // never seen (p ~ 2^-1000): mark the stripe undecodable
                    atomicOr(err, kErrOorTruncated);
                sum = 0;
                for (int i = sub; i < k; i += 4) {
                    row[i] = canon_lz(static_cast<int32_t>(row[i] * (sc ? sc : 1u)));
                    sum += row[i];
                }
                // the lane's groups back from the rescaled row
#pragma unroll
                for (int m = 0; m < MG; m++) {
                    const int i0 = 4 * sub + 16 * m;
                    if (i0 < k)
                        ev[m] = *reinterpret_cast<const uint4*>(row + i0);
                }
            }
            sum += __builtin_amdgcn_update_dpp(0u, sum, 0xB1, 0xf, 0xf, false);
            sum += __builtin_amdgcn_update_dpp(0u, sum, 0x4E, 0xf, 0xf, false);
            if (t < L.R && sub == 0) {
                // sum < 2^24: two folds, then canonical
                const uint32_t sq = canon_lz(fold(static_cast<int32_t>(sum)));
                mat[L.kcorr() + t] = static_cast<int32_t>(canon_lz(mul_lz(balanced(sq), 32768)));
                mat[L.rscale() + t] = rs;
                if (KS) {
                    mat[L.kmf() + t] = static_cast<int32_t>(canon_lz(mul_lz(balanced(sq), 32896)));
                    mat[L.rscale_mf() + t] = rs;
                }
            }
            // the operand tiles (pack_mf_dword's layout: [a | 0], [0 | b],
            // [b | a]; the zero halves are not written at KS >= 4, the kernel
            // never reads them), zeros past the rows and entries: a wave
            // holds 16 rows of one row block, so each store fills 64
            // consecutive dwords of a tile
            if (!KS || t >= 16 * RB)
                continue;
            const int rb = t >> 4, tl = t & 15;
#pragma unroll
            for (int m = 0; m < MG; m++) {
                const int i0 = 4 * sub + 16 * m;
                if (m >= KS)  // groups j = sub + 4 m < KH / 4
                    break;
                // split_i8 of the 4 entries (0 past k and past R: a = b = 0):
                // v = 256 a + b in [-32896, 32639], b = the signed low byte
                // of v, a = (v - b) / 256; entry jb's bytes into byte jb of
                // aw / bw by three byte permutes each
                const uint32_t e[4] = {ev[m].x, ev[m].y, ev[m].z, ev[m].w};
                uint32_t vb[4], va[4];
#pragma unroll
                for (int jb = 0; jb < 4; jb++) {
                    int32_t v = balanced(e[jb]);
                    v = v > 32639 ? v - kQ : v;
                    const int32_t b = (v << 24) >> 24;
                    vb[jb] = static_cast<uint32_t>(v);      // b's byte: byte 0
                    va[jb] = static_cast<uint32_t>(v - b);  // a's byte: byte 1
                }
                const uint32_t bw = __builtin_amdgcn_perm(
                    __builtin_amdgcn_perm(vb[3], vb[2], 0x0c0c0400u),
                    __builtin_amdgcn_perm(vb[1], vb[0], 0x0c0c0400u), 0x05040100u);
                const uint32_t aw = __builtin_amdgcn_perm(
                    __builtin_amdgcn_perm(va[3], va[2], 0x0c0c0501u),
                    __builtin_amdgcn_perm(va[1], va[0], 0x0c0c0501u), 0x05040100u);
#pragma unroll
                for (int half = 0; half < 2; half++) {
                    const int K = half * KH + i0;
                    const int ks = K >> 5, g = (K & 31) >> 3, dw = (K & 7) >> 2;
                    const size_t base =
                        static_cast<size_t>((rb * KS + ks) * 3) * 128 + (16 * g + tl) * 2 + dw;
                    if (KS < 4 || half == 0)
                        mf[base] = static_cast<int32_t>(half ? 0u : aw);        // [a | 0]
                    if (KS < 4 || half == 1)
                        mf[base + 128] = static_cast<int32_t>(half ? bw : 0u);  // [0 | b]
                    if (KS < 2)  // [b | a]: the kernels rebuild it at KS >= 2
                        mf[base + 256] = static_cast<int32_t>(half ? aw : bw);
                }
            }
        }
    }
    // the canonical `plain` rows and the dot2 kernel's packed pairs, only
    // for widths with a column tail (dot2): the matrix-core kernels read the
    // tiles alone (their OOR restore and the redo kernel take single
    // coefficients back from the tiles), and fill_dot2_sections writes these
    // two from the tiles if a whole-tile decode ever needs the dot2 kernel
    // (rows the matrix cores cannot address).  Items entries-fastest, so a
    // wave's stores are contiguous runs (rows-fastest 16-byte pieces
    // scattered over the rows had made the round-1 context store-bound)
    if (!dot2)
        return;
    __syncthreads();  // every row final (the pass above is row-local)
    int32_t* plain = mat + L.plain();
    const int ng = (k + 3) / 4;
    for (int it = tid; it < L.R * ng; it += NT) {
        const int t = it / ng, i0 = 4 * (it - t * ng);
        const uint4 e4 = *reinterpret_cast<const uint4*>(Mt + t * kp + i0);
        const uint32_t e[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
        for (int jb = 0; jb < 4; jb++)
            if (i0 + jb < k)
                plain[static_cast<size_t>(t) * k + i0 + jb] = static_cast<int32_t>(e[jb]);
        int32_t* packed = mat + static_cast<size_t>(t) * L.KP;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int i = i0 + 2 * h;
            if (i < k) {
                const int32_t lo = balanced(e[2 * h]);
                const int32_t hi = i + 1 < k ? balanced(e[2 * h + 1]) : 0;
                packed[i >> 1] = static_cast<int32_t>((static_cast<uint32_t>(lo) & 0xffffu) |
                                                      (static_cast<uint32_t>(hi) << 16));
            }
        }
    }
    // packed pairs past kin up to KP stay zero (the dot2 kernel's padding)
    const int pz = (k + 1) / 2, npz = L.KP - pz;
    for (int it = tid; it < L.R * npz; it += NT)
        mat[static_cast<size_t>(it / npz) * L.KP + pz + it % npz] = 0;
}

// The dot2 sections (packed pairs, canonical `plain` rows) of contexts built
// without them (whole-tile widths, dot2 = 0), from their operand tiles: for
// a decode whose rows the matrix cores cannot address (launch_matrix then
// runs the dot2 kernel over every column).  Decode contexts hold rows the
// dot2 kernel can take (coef_ok), so the balanced entries fit its pairs.
__global__ __launch_bounds__(256) void fill_dot2_kernel(MatLayout L, int32_t* ctx, long long cs,
                                                        long long lazy_off)
{
    int32_t* mat = ctx + blockIdx.x * cs;
    uint32_t* lazy = reinterpret_cast<uint32_t*>(mat + lazy_off);
    if (*lazy & kLazyDot2)
        return;  // filled by an earlier decode (block-uniform)
    const int32_t* mf = mat + L.mf();
    int32_t* plain = mat + L.plain();
    for (int it = threadIdx.x; it < L.R * L.KP; it += 256) {
        const int t = it / L.KP, j = it - t * L.KP, i = 2 * j;
        int32_t v[2] = {0, 0};
#pragma unroll
        for (int h = 0; h < 2; h++) {
            if (i + h < L.kin) {
                const uint32_t e = mf_entry(L, mf, t, i + h);
                plain[static_cast<size_t>(t) * L.kin + i + h] = static_cast<int32_t>(e);
                v[h] = balanced(e);
            }
        }
        mat[static_cast<size_t>(t) * L.KP + j] = static_cast<int32_t>(
            (static_cast<uint32_t>(v[0]) & 0xffffu) | (static_cast<uint32_t>(v[1]) << 16));
    }
    __syncthreads();
    if (threadIdx.x == 0)
        *lazy |= kLazyDot2;
}

int fill_dot2_sections(const MatLayout& L, int32_t* d_ctx, long long ctx_stride, long long words,
                       int S, hipStream_t st)
{
    if (S <= 0)
        return 0;
    const long long lazy_off = L.words() + 2LL * L.KP + lazy_word_off(words);
    hipLaunchKernelGGL(fill_dot2_kernel, dim3(S), dim3(256), 0, st, L, d_ctx, ctx_stride,
                       lazy_off);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int launch_decode_ctx(int k, int n, uint32_t r, int mode, const MatLayout& L,
                      const uint16_t* d_ids, int S, int32_t* d_ctx,
                      long long ctx_stride, const Oor* in_oor, int slot_base,
                      int by_pos, long long words, int dot2, uint32_t* err, hipStream_t st)
{
    if (k > kMatMaxKin || S <= 0)
        return -3;
    Oor none{nullptr, nullptr, 0, 0};
    if (k > 128) {
        // the matrix rows in the context itself (no LDS image); 1024 threads
        // keep 4x more of the packing and tile passes' row loads in flight
        // (k256 decode 0.81 -> 0.77 ms, k200 2.09 -> 2.05 ms)
        // (the whole-tile contexts stage ctx_chunk(k)-row chunks of the
        // matrix in the dynamic LDS; the dot2 forms keep the rows in global
        // memory and reserve none)
        const size_t lds =
            !dot2 ? static_cast<size_t>(ctx_chunk(k)) * ((k + 3) & ~3) * 4 : 0;
        static std::atomic<uint64_t> attr_done{0};
        static std::atomic<int> cus_of[64];
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess)
            return -2;
        const uint64_t bit = dev < 64 ? 1ull << dev : 0;
        if (!bit || !(attr_done.load(std::memory_order_acquire) & bit)) {
            int cus = 0;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                hipSuccess)
                return -2;
            if (bit)
                cus_of[dev].store(std::max(1, cus), std::memory_order_relaxed);
            const void* fn = reinterpret_cast<const void*>(&decode_ctx_kernel<1024, true>);
            constexpr size_t kDynMax =
                std::max(static_cast<size_t>(kCtxChunk) * kMatGenMaxKin, size_t{32} * kMatMaxKin) * 4;
            // the kernel's static LDS (the packing stage, A, x_i, ...) plus
            // the largest chunk must fit a CU (160 KiB): an added __shared__
            // would make every k > 256 context launch fail, so say so here
            hipFuncAttributes fa{};
            if (hipFuncGetAttributes(&fa, fn) != hipSuccess ||
                fa.sharedSizeBytes + kDynMax > static_cast<size_t>(kCtxLdsCap))
                return -2;
            if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    static_cast<int>(kDynMax)) != hipSuccess)
                return -2;
            attr_done.fetch_or(bit, std::memory_order_release);
        }
        // the whole-tile forms split a stripe's row chunks over up to (CUs /
        // stripes) blocks (one block per CU each)
        int nb = 1;
        if (!dot2) {
            const int cus = bit ? cus_of[dev].load(std::memory_order_relaxed) : 256;
            const int nch = (k + ctx_chunk(k) - 1) / ctx_chunk(k);
            nb = std::max(1, std::min(nch, cus / S));
        }
        if (static_cast<long long>(S) * nb > 0x7fffffffLL)
            return -1;
        hipLaunchKernelGGL((decode_ctx_kernel<1024, true>), dim3(S * nb), dim3(1024), lds, st, k,
                           n, r, mode, L, d_ids, d_ctx, ctx_stride, in_oor ? *in_oor : none,
                           slot_base, by_pos, words, dot2, err, nb);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    RPow2 rp{};
    uint32_t e = r;
    for (int b = 0; b < 16; b++, e = mulmod_c(e, e))
        rp.v[b] = balanced(e);
    int lgn = 0;
    while (lgn < 16 && (1u << lgn) < static_cast<uint32_t>(n))
        lgn++;
    const size_t lds = static_cast<size_t>(k) * ctx_pitch(k) * 4;
    // k > 64: up to 68 KB (k = 128) of dynamic LDS, opted in
    // per launch (cheap; the device may differ between calls)
    if (lds > 65536 &&
        hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_ctx_lds_kernel<256>),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(lds)) != hipSuccess)
        return -2;
    // 2 waves at k <= 32: wave 1 routes the marks while wave 0 builds A(x)
    if (k > 32)
        hipLaunchKernelGGL((decode_ctx_lds_kernel<256>), dim3(S), dim3(256), lds, st, k, rp, lgn,
                           mode, L, d_ids, d_ctx, ctx_stride, in_oor ? *in_oor : none,
                           slot_base, by_pos, words, dot2, err);
    else
        hipLaunchKernelGGL((decode_ctx_lds_kernel<128>), dim3(S), dim3(128), lds, st, k, rp, lgn,
                           mode, L, d_ids, d_ctx, ctx_stride, in_oor ? *in_oor : none,
                           slot_base, by_pos, words, dot2, err);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace qi
