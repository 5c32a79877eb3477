// The opaque qi_plan behind include/qi_gpu.h (host-only definition).
#pragma once

#include <hip/hip_runtime.h>

#include <stddef.h>
#include <stdint.h>

#include <string>

#include "qi_internal.h"

namespace qi {

// grow-only device scratch owned by a plan (block API staging)
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool reserve(size_t n)
    {
        if (n <= bytes)
            return true;
        if (p)
            (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        if (hipMalloc(&p, n) != hipSuccess) {
            p = nullptr;
            return false;
        }
        bytes = n;
        return true;
    }
    void release()
    {
        if (p)
            (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

struct HostState {
    hipStream_t stream = nullptr;
    DevBuf in, out, counts, entries, ids, ctx;
    void release()
    {
        in.release();
        out.release();
        counts.release();
        entries.release();
        ids.release();
        ctx.release();
        if (stream)
            (void)hipStreamDestroy(stream);
        stream = nullptr;
    }
};

}  // namespace qi

struct qi_plan;

namespace qi {
// per-stripe decode context stride (int32 words) and builder (qi_gpu.cpp)
long long ctx_stride(const qi_plan* p, long long words);
SlowList ctx_slow(const qi_plan* p, const void* d_ctx, long long words);
int build_ctx(qi_plan* p, const uint16_t* d_ids, int n_stripes, const Oor* in,
              int slot_base, int by_pos, long long words, void* d_ctx, hipStream_t s);
}  // namespace qi

struct qi_plan {
    int k = 0, m = 0, sys = 0, code_len = 0, n_outputs = 0, n = 0, K = 0;
    uint32_t r = 0;
    int device = 0;
    int32_t* d_twist = nullptr;  // encode twist factors (non-systematic)
    int32_t* d_gen = nullptr;    // generator matrix block (matrix encode)
    qi::MatLayout gen{0, 0, 0};
    // output row of each generator row (rows needing a unit scale grouped
    // at the end, so few 16-row blocks run the scaling epilogue), and the
    // identity map of the k x k decode matrices
    int32_t* d_rowmap = nullptr;
    int32_t* d_rowid = nullptr;
    // general-k path (k > 256, ntt.hip; see mbig): transforms of length <= nmax =
    // max(n, len_2k), balanced twiddle tables w^e / w^-e, and the systematic
    // encode's constant decode context
    int ntt = 0, len2k = 0, nmax = 0;
    // 256 < k <= 384: batches whose columns tile exactly (words a multiple
    // of 1024) run the matrix cores instead (d_gen, k x k contexts); also
    // 384 < k <= 640, n - k > 64: the decodes, and the systematic encodes
    // with a small generator (big_generator_ok; the non-systematic encodes
    // stay on the NTT engine)
    int mbig = 0;
    int32_t* d_tw[2] = {nullptr, nullptr};
    int32_t* d_ldstw = nullptr;  // per-pass twiddle tables of the LDS engine
    int32_t* d_sysctx = nullptr;
    uint32_t* d_err = nullptr;
    qi::HostState host;
};

namespace qi {
// ---- general-k path (ntt.hip) ----
int ntt_plan_init(qi_plan* p);
// the erasure decode's shape (n <= 2048, n - k <= 64; ntt.hip)
bool eras_shape(int k, int n);
// the NTT engine's kernels for an encode or a decode (a decode's list starts
// with its context builder): ntt_eras_kernel<TWG> (few erasures), ntt_lds_kernel<TWG>
// (max(n, len_2k) <= 2048) or the multi-pass engine
std::string ntt_kernel_names(const qi_plan* p, bool decode);
void ntt_plan_free(qi_plan* p);
long long ntt_ctx_words(const qi_plan* p);
int ntt_build_ctx(const qi_plan* p, const uint16_t* d_ids, int n_stripes, int32_t* d_ctx,
                  long long ctx_stride, hipStream_t s);
// the same from ids held as dwords (ids32 + s * ids_stride: a matrix
// context's id section), skipping the stripes whose lazy word (lazy + s *
// ctx_stride) has kLazyNtt set and setting it after: a 256 < k <= 384
// decode builds its NTT context only when the matrix cores cannot take it
int ntt_build_ctx_lazy(const qi_plan* p, const int32_t* ids32, int n_stripes, int32_t* d_ctx,
                       long long ctx_stride, uint32_t* lazy, hipStream_t s);
int ntt_encode(const qi_plan* p, const uint16_t* data, long long dss, long long drs,
               RowDst out, long long words, int n_stripes, const Oor* oor, hipStream_t s);
int ntt_decode(const qi_plan* p, const int32_t* ctx, long long ctx_stride, RowSrc src,
               const Oor* in_oor, int slot_base, RowDst out, long long words,
               int n_stripes, hipStream_t s);
}  // namespace qi
