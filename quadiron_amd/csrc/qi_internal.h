// Internal (host-side) declarations shared by the plan, the device shim and
// the drop-in C-ABI.  Nothing here crosses the public C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "matrix_pack.h"  // MatLayout: the packed matrix block

namespace qi {

// OOR routing: the decode context keeps, per stripe and per tile of
// kRouteTile columns, the marks of the received rows that fall in the tile
// (count + up to kRouteCap entries packed as position << 16 | column-in-tile).
// A count above kRouteCap makes the decode kernel scan the OOR buckets.
constexpr int kRouteTile = 1024;  // a multiple of every block width (256*COLS)
constexpr int kRouteCap = 15;
constexpr int kRouteStride = kRouteCap + 1;

__host__ __device__ inline long long route_tiles(long long words)
{
    return (words + kRouteTile - 1) / kRouteTile;
}

// Sticky device error bits (qi_gpu_take_error): an OOR bucket held more
// marks than its capacity `cap`, so some marks were lost (encode keeps the
// exact count, decode could not restore every 65536 symbol).
constexpr uint32_t kErrOorTruncated = 1u;
// A decode context was asked for with received ids that are not distinct or
// not below n (the erasure decode's context, which derives the erased set
// from them, checks; the context is then unusable and nothing outside it is
// written).
constexpr uint32_t kErrBadIds = 2u;

// Row source for the matrix kernel: fragment `id` of stripe `s` is at
//   id <  split : base0 + s*ss0 + id*rs0
//   id >= split : base1 + s*ss1 + (id-split)*rs1        (elements of u16)
//   by_pos != 0: row (and OOR slot) of the i-th received fragment is found
//   by its position i instead of its id (compact staging of the block API)
struct RowSrc {
    const uint16_t* base0;
    long long ss0, rs0;
    int split;
    const uint16_t* base1;
    long long ss1, rs1;
    int by_pos;
    int rows0, rows1;  // rows addressable through base0 / base1
};

// Output rows: row t of stripe s at base + s*ss + t*rs
struct RowDst {
    uint16_t* base;
    long long ss, rs;
};

// OOR buckets: counts[s*slots + slot], entries[(s*slots + slot)*cap + e]
struct Oor {
    uint32_t* counts;
    uint32_t* entries;
    int slots;
    int cap;
};

// Per-stripe list of the column tiles whose received-row OOR marks overflowed
// the matrix kernels' LDS list (more than 256 in one tile; adversarial
// data).  Kept in the decode context: word 0 = count, then one word per
// tile (col0 / 64) << 3 | log2(width / 64).  Every kernel tile is a
// power-of-two multiple of kSlowGrain = 64 columns (the narrowest, KS = 16
// matrix-core blocks) starting on a multiple of its width, and each tile is
// pushed at most once per launch, so capacity slow_words(words) - 1 =
// ceil(words / 64) covers every tile of a stripe.  launch_matrix runs
// matrix_redo_kernel over it right after the matrix kernels.
struct SlowList {
    uint32_t* base;  // stripe s at base + s * stride (nullptr: no input marks)
    long long stride;
};

constexpr int kSlowGrain = 64;

__host__ __device__ inline long long slow_words(long long words)
{
    return 1 + (words + kSlowGrain - 1) / kSlowGrain;
}

// A matrix context's lazy-section word (behind its slow-tile list, per
// stripe, cleared by the context builder): the sections a decode fills on
// first use, when the batch's rows keep it off the matrix cores -- bit 0
// the dot2 sections (fill_dot2_sections), bit 1 the NTT engine's context of
// a 256 < k <= 384 plan (ntt_build_ctx_lazy).  Offset from the route table.
constexpr uint32_t kLazyDot2 = 1u, kLazyNtt = 2u;
__host__ __device__ inline long long lazy_word_off(long long words)
{
    return route_tiles(words) * kRouteStride + slow_words(words);
}
// words reserved for it (keeps the following section's alignment)
constexpr int kLazyWords = 4;

// ---- launchers (kernels.hip) ----
// non-systematic encode by twisted register-resident sub-NTTs
int launch_encode_fnt(int k, int n, int n_out, const int32_t* d_twist,
                      const uint16_t* data, long long dss, long long drs,
                      RowDst out, long long words, int n_stripes, Oor oor,
                      uint32_t* d_err, hipStream_t stream);

// out[t] = sum_i M[t][i] * in[ids[i]]  for t < R
//   mat: per-stripe blocks (mat_stride words apart; 0 = shared)
//   ids: per-stripe kin int32 fragment ids, ids_stride apart (nullptr =
//   identity 0..kin-1)
//   in_oor: restore buckets by slot (nullptr = none); slot_of_id = id -
//     slot_base (ids < slot_base have no bucket)
//   out_oor: record OOR outputs (nullptr = no recording; values stored as 0)
//   rowmap: output row (and OOR slot) of matrix row t (R entries, required;
//   identity for decode matrices)
//   route: per-stripe OOR routing tables (route_stride u32 apart), or null
//   slow: per-stripe slow-tile lists (required when in_oor is given)
int launch_matrix(const MatLayout& L, const int32_t* mat, long long mat_stride,
                  const int32_t* ids, long long ids_stride, RowSrc src,
                  RowDst dst, long long words,
                  int n_stripes, const Oor* in_oor, int slot_base,
                  const Oor* out_oor, const int32_t* rowmap, const uint32_t* route,
                  long long route_stride, SlowList slow, uint32_t* d_err,
                  hipStream_t stream);

// per-stripe decode matrices from fragment ids (S x k).
//   mode 0: coefficient extraction (non-systematic: data = poly coefs)
//   mode 1: evaluation at r^t, t < k (systematic: data = P(r^t))
//   d_ctx: per stripe ctx_stride words: the MatLayout block, the k ids as
//   int32 (padded to 2 KP), the OOR route table (route_tiles(words) x
//   kRouteStride u32) built from in_oor, then the slow-tile list
//   (slow_words(words) u32, count cleared), then the lazy-section word
//   (cleared; lazy_word_off)
//   (slot = by_pos ? position : id - slot_base); in_oor may be null.
//   n: the code length (ids < n), r its root of unity
//   dot2: also write the dot2 kernel's sections (packed pairs, `plain`
//   rows); without them only the matrix cores can apply the context
int launch_decode_ctx(int k, int n, uint32_t r, int mode, const MatLayout& L,
                      const uint16_t* d_ids, int n_stripes, int32_t* d_ctx,
                      long long ctx_stride, const Oor* in_oor, int slot_base,
                      int by_pos, long long words, int dot2, uint32_t* d_err,
                      hipStream_t stream);
// the dot2 sections of n_stripes contexts built with dot2 = 0 for `words`
// columns, from their operand tiles (before a decode that runs the dot2
// kernel over them); a stripe whose lazy word has kLazyDot2 set is skipped,
// and the bit is set after the fill
int fill_dot2_sections(const MatLayout& L, int32_t* d_ctx, long long ctx_stride, long long words,
                       int n_stripes, hipStream_t stream);

// matrix kernel instantiation choice
int matrix_kp(int kin);
// whether launch_matrix runs these rows on the matrix cores (whole
// kRouteTile tiles): 8-byte aligned rows inside 31-bit buffer ranges.  The
// kin > 256 layouts have no other kernel, so their callers check this first.
bool matrix_cores_take(const RowSrc& src, const RowDst& dst, int R, long long words);
// names of the kernels launch_matrix runs for L over `words` columns
// (aligned rows; diagnostics: qi_gpu_kernels); two: rows from two source
// regions (the systematic decode)
std::string matrix_kernel_names(const MatLayout& L, long long words, bool in_oor, bool two);
// the register-codelet encode kernel launch_encode_fnt runs (aligned rows)
std::string encode_fnt_kernel_name(int k);

// ---- host math (plan.cpp) ----
// Lagrange matrix for points x_i = r^{ids[i]}:
//   mode 0: M[t][i] = coef_t(L_i), t < k
//   mode 1: M[t][i] = L_i(eval[t]), t < R
std::vector<uint32_t> lagrange_matrix(int k, uint32_t r, const uint32_t* ids,
                                      int mode, const uint32_t* eval, int R);
// pack a canonical R x kin matrix into a MatLayout block
void pack_matrix(const MatLayout& L, const uint32_t* M, int32_t* block);

}  // namespace qi
