// Device-level C-ABI (include/qi_gpu.h): batch encode / decode on
// device-resident stripes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/qi_gpu.h"
#include "gf65537.h"
#include "qi_internal.h"
#include "qi_plan.h"

using namespace qi;

namespace {

MatLayout ctx_layout(const qi_plan* p)
{
    return MatLayout{p->k, p->k, matrix_kp(p->k)};
}


hipStream_t st(void* s)
{
    return static_cast<hipStream_t>(s);
}

// The decode-context format for this batch width: matrix contexts for
// every k <= 256, and for 256 < k <= 384 (mbig) when the columns tile into
// whole 1024-column blocks (the operand-stationary kernel has no column tail
// there); otherwise the NTT engine's.  A context is valid only for the
// `words` it was built with.
bool use_matrix(const qi_plan* p, long long words)
{
    return !p->ntt || (p->mbig && words % kRouteTile == 0);
}

// the matrix-format part of a context: packed block, ids, route table,
// slow-tile list, lazy-section word
long long mat_ctx_words(const qi_plan* p, long long words)
{
    const MatLayout L = ctx_layout(p);
    return static_cast<long long>(L.words()) + 2 * L.KP + lazy_word_off(words) + kLazyWords;
}

// A context built for a whole-tile width carries only the matrix-core
// form.  Rows the matrix cores cannot address send every column to the dot2
// kernel (k <= 256), whose sections are filled from the tiles by the first
// such decode, or to the NTT engine (256 < k <= 384), whose context is built
// by the first such decode from the ids the matrix context holds; the
// context's lazy word records both, so each is filled once (qi_gpu.h: a
// decode may write its context)
int complete_lazy(const qi_plan* p, const void* d_ctx, long long cs, long long words, int S,
                  hipStream_t s)
{
    if (words % kRouteTile != 0)
        return 0;  // built with them
    int32_t* c = static_cast<int32_t*>(const_cast<void*>(d_ctx));
    const MatLayout L = ctx_layout(p);
    if (p->mbig)
        return ntt_build_ctx_lazy(
            p, c + L.words(), S, c + mat_ctx_words(p, words), cs,
            reinterpret_cast<uint32_t*>(c + L.words() + 2 * L.KP + lazy_word_off(words)), s);
    return fill_dot2_sections(L, c, cs, words, S, s);
}

}  // namespace

namespace qi {

long long ctx_stride(const qi_plan* p, long long words)
{
    if (!use_matrix(p, words))
        return ntt_ctx_words(p);
    // 256 < k <= 384: the NTT engine's context follows the matrix one, for
    // rows the matrix cores cannot address (matrix_cores_take)
    return mat_ctx_words(p, words) + (p->mbig ? ntt_ctx_words(p) : 0);
}

// the slow-tile lists of n contexts (behind each route table)
SlowList ctx_slow(const qi_plan* p, const void* d_ctx, long long words)
{
    const MatLayout L = ctx_layout(p);
    uint32_t* c = static_cast<uint32_t*>(const_cast<void*>(d_ctx));
    return SlowList{c + L.words() + 2 * L.KP + route_tiles(words) * kRouteStride,
                    ctx_stride(p, words)};
}

// Decode contexts for n_stripes stripes, built on the device inside the
// caller's stream: the matrix paths (k <= 256; 256 < k <= 384 at whole-tile
// widths), interpolation matrices + OOR route tables (decode_ctx_kernel);
// otherwise the NTT decode's per-pattern constants (ntt_ctx_kernel or
// eras_ctx_kernel; its decode reads the OOR buckets directly).
int build_ctx(qi_plan* p, const uint16_t* d_ids, int n_stripes, const Oor* in,
              int slot_base, int by_pos, long long words, void* d_ctx, hipStream_t s)
{
    if (n_stripes == 0)
        return 0;
    if (!d_ids)
        return -1;
    const long long cs = ctx_stride(p, words);
    if (!use_matrix(p, words))
        return ntt_build_ctx(p, d_ids, n_stripes, static_cast<int32_t*>(d_ctx), cs, s);
    const MatLayout L = ctx_layout(p);
    // (256 < k <= 384: the NTT engine's half only when a decode needs it,
    // complete_lazy)
    // the dot2 sections only for widths with a column tail (below 256 < k:
    // no dot2 kernel at all); a whole-tile decode that needs them after all
    // fills them from the tiles (qi_gpu_decode)
    const int dot2 = !p->mbig && words % kRouteTile != 0;
    return launch_decode_ctx(p->k, p->n, p->r, p->sys ? 1 : 0, L, d_ids, n_stripes,
                             static_cast<int32_t*>(d_ctx), cs, in, slot_base, by_pos,
                             words, dot2, p->d_err, s);
}

}  // namespace qi

extern "C" {

int qi_gpu_oor_clear(uint32_t* d_counts, size_t n, void* stream)
{
    if (!d_counts || n == 0)
        return 0;
    return hipMemsetAsync(d_counts, 0, n * sizeof(uint32_t), st(stream)) ==
                   hipSuccess
               ? 0
               : -2;
}

int qi_gpu_encode(qi_plan* p, const uint16_t* d_data, long long dss,
                  long long drs, uint16_t* d_out, long long oss, long long ors,
                  long long words, int n_stripes, uint32_t* d_counts,
                  uint32_t* d_entries, int cap, void* stream)
{
    if (!p || !d_data || !d_out || n_stripes < 0 || words < 0)
        return -1;
    if (n_stripes == 0 || words == 0)
        return 0;
    Oor oor{d_counts, d_entries, p->n_outputs, cap};
    RowDst out{d_out, oss, ors};
    RowSrc src{d_data, dss, drs, 1 << 30, nullptr, 0, 0, 0, p->k, 0};
    // k > 256: the NTT engine, unless the matrix cores take the batch (mbig
    // plans with a generator, whole tiles, addressable rows)
    if (p->ntt && !(p->d_gen && use_matrix(p, words) &&
                    matrix_cores_take(src, out, p->gen.R, words)))
        return ntt_encode(p, d_data, dss, drs, out, words, n_stripes,
                          d_counts ? &oor : nullptr, st(stream));
    if (!p->d_gen)
        return launch_encode_fnt(p->k, p->n, p->n_outputs, p->d_twist, d_data,
                                 dss, drs, out, words, n_stripes, oor,
                                 p->d_err, st(stream));
    return launch_matrix(p->gen, p->d_gen, 0, nullptr, 0, src, out, words,
                         n_stripes, nullptr, 0, d_counts ? &oor : nullptr, p->d_rowmap,
                         nullptr, 0, SlowList{nullptr, 0}, p->d_err, st(stream));
}

size_t qi_gpu_decode_ctx_bytes(const qi_plan* p, int n_stripes,
                               long long words)
{
    if (!p || n_stripes < 0 || words < 0)
        return 0;
    // an upper bound for every width up to `words` (the format, and so the
    // stride, of a 256 < k <= 384 context depends on the width: a caller
    // sizing for its widest batch may build narrower ones in the buffer)
    long long w = ctx_stride(p, words);
    if (p->mbig && words >= kRouteTile)
        w = std::max(w, ctx_stride(p, words / kRouteTile * kRouteTile));
    return static_cast<size_t>(w) * sizeof(int32_t) * static_cast<size_t>(n_stripes);
}

int qi_gpu_decode_ctx(qi_plan* p, const uint16_t* d_ids, const uint16_t* h_ids,
                      int n_stripes, const uint32_t* d_counts,
                      const uint32_t* d_entries, int cap, long long words,
                      void* d_ctx, void* stream)
{
    if (!p || !d_ctx || n_stripes < 0 || words < 0)
        return -1;
    Oor in{const_cast<uint32_t*>(d_counts), const_cast<uint32_t*>(d_entries),
           p->n_outputs, cap};
    (void)h_ids;  // contexts are built on the device for every k
    return qi::build_ctx(p, d_ids, n_stripes, d_counts ? &in : nullptr,
                         p->sys ? p->k : 0, 0, words, d_ctx, st(stream));
}

int qi_gpu_decode(qi_plan* p, const void* d_ctx, const uint16_t* d_ids,
                  const uint16_t* d_data, long long dss, long long drs,
                  const uint16_t* d_coded, long long css, long long crs,
                  const uint32_t* d_counts, const uint32_t* d_entries, int cap,
                  uint16_t* d_out, long long oss, long long ors,
                  long long words, int n_stripes, void* stream)
{
    if (!p || !d_ctx || !d_ids || !d_out || !d_coded || n_stripes < 0 || words < 0)
        return -1;
    if (n_stripes == 0 || words == 0)
        return 0;
    const MatLayout L = ctx_layout(p);
    RowSrc src;
    if (p->sys)
        src = RowSrc{d_data ? d_data : d_coded, dss, drs, p->k, d_coded, css, crs, 0,
                     p->k, p->n_outputs};
    else
        src = RowSrc{d_coded, css, crs, 1 << 30, nullptr, 0, 0, 0, p->n_outputs, 0};
    Oor in{const_cast<uint32_t*>(d_counts), const_cast<uint32_t*>(d_entries),
           p->n_outputs, cap};
    RowDst out{d_out, oss, ors};
    const long long cs = ctx_stride(p, words);
    const int32_t* ctx = static_cast<const int32_t*>(d_ctx);
    (void)d_ids;  // the context carries the ids (as dwords)
    if (!use_matrix(p, words))
        return ntt_decode(p, ctx, cs, src, d_counts ? &in : nullptr, p->sys ? p->k : 0, out,
                          words, n_stripes, st(stream));
    if (!matrix_cores_take(src, out, L.R, words)) {
        if (int rc = complete_lazy(p, d_ctx, cs, words, n_stripes, st(stream)))
            return rc;
        if (p->mbig)
            return ntt_decode(p, ctx + mat_ctx_words(p, words), cs, src,
                              d_counts ? &in : nullptr, p->sys ? p->k : 0, out, words,
                              n_stripes, st(stream));
    }
    return launch_matrix(L, ctx, cs, ctx + L.words(), cs, src, out, words,
                         n_stripes, d_counts ? &in : nullptr, p->sys ? p->k : 0,
                         nullptr, p->d_rowid,
                         reinterpret_cast<const uint32_t*>(ctx + L.words() + 2 * L.KP),
                         cs, ctx_slow(p, d_ctx, words), p->d_err, st(stream));
}

int qi_gpu_decode_ctx_packed(qi_plan* p, const uint16_t* d_ids,
                             const uint16_t* h_ids, int n_stripes,
                             const uint32_t* d_counts, const uint32_t* d_entries,
                             int cap, long long words, void* d_ctx, void* stream)
{
    if (!p || !d_ctx || n_stripes < 0 || words < 0)
        return -1;
    Oor in{const_cast<uint32_t*>(d_counts), const_cast<uint32_t*>(d_entries),
           p->k, cap};
    (void)h_ids;
    return qi::build_ctx(p, d_ids, n_stripes, d_counts ? &in : nullptr, 0, 1, words,
                         d_ctx, st(stream));
}

int qi_gpu_decode_packed(qi_plan* p, const void* d_ctx, const uint16_t* d_recv,
                         long long rss, long long rrs, const uint32_t* d_counts,
                         const uint32_t* d_entries, int cap, uint16_t* d_out,
                         long long oss, long long ors, long long words,
                         int n_stripes, void* stream)
{
    if (!p || !d_ctx || !d_recv || !d_out || n_stripes < 0 || words < 0)
        return -1;
    if (n_stripes == 0 || words == 0)
        return 0;
    const MatLayout L = ctx_layout(p);
    RowSrc src{d_recv, rss, rrs, 1 << 30, nullptr, 0, 0, 1, p->k, 0};
    Oor in{const_cast<uint32_t*>(d_counts), const_cast<uint32_t*>(d_entries),
           p->k, cap};
    RowDst out{d_out, oss, ors};
    const long long cs = ctx_stride(p, words);
    const int32_t* ctx = static_cast<const int32_t*>(d_ctx);
    if (!use_matrix(p, words))
        return ntt_decode(p, ctx, cs, src, d_counts ? &in : nullptr, 0, out, words,
                          n_stripes, st(stream));
    if (!matrix_cores_take(src, out, L.R, words)) {
        if (int rc = complete_lazy(p, d_ctx, cs, words, n_stripes, st(stream)))
            return rc;
        if (p->mbig)
            return ntt_decode(p, ctx + mat_ctx_words(p, words), cs, src,
                              d_counts ? &in : nullptr, 0, out, words, n_stripes,
                              st(stream));
    }
    return launch_matrix(L, ctx, cs, ctx + L.words(), cs, src, out, words,
                         n_stripes, d_counts ? &in : nullptr, 0, nullptr, p->d_rowid,
                         reinterpret_cast<const uint32_t*>(ctx + L.words() + 2 * L.KP),
                         cs, ctx_slow(p, d_ctx, words), p->d_err, st(stream));
}

const char* qi_gpu_kernels(const qi_plan* p, long long words)
{
    static thread_local std::string names;
    if (!p || words <= 0)
        return "";
    std::string enc, dec;
    if (!use_matrix(p, words)) {
        enc = ntt_kernel_names(p, false);
        dec = ntt_kernel_names(p, true);
    } else {
        if (p->ntt && !p->d_gen)
            enc = ntt_kernel_names(p, false);
        else if (!p->d_gen)
            enc = encode_fnt_kernel_name(p->k);
        else
            enc = matrix_kernel_names(p->gen, words, false, false);
        const MatLayout L = ctx_layout(p);
        // launch_decode_ctx's choice (ctx.hip)
        dec = std::string(p->k > 128  ? "decode_ctx_kernel<1024, true>"
               : p->k > 32 ? "decode_ctx_lds_kernel<256>"
                           : "decode_ctx_lds_kernel<128>") +
              " + " + matrix_kernel_names(L, words, true, p->sys != 0);
    }
    names = "encode=" + enc + "; decode=" + dec;
    return names.c_str();
}

// git describe of the tree the library was built from + a hash of its
// sources (quadiron_amd/csrc/Makefile writes QI_BUILD_ID), so a run's
// record ties the loaded binary to a commit
const char* qi_build_id(void)
{
#ifdef QI_BUILD_ID
    return QI_BUILD_ID;
#else
    return "unknown";
#endif
}

int qi_gpu_take_error(qi_plan* p)
{
    if (!p)
        return -1;
    uint32_t e = 0;
    if (hipMemcpy(&e, p->d_err, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return -2;
    if (e)
        (void)hipMemset(p->d_err, 0, 4);
    return static_cast<int>(e);
}

}  // extern "C"
