// Plan construction and host-side matrix math for the RS-FNT engine.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/qi_gpu.h"
#include "gf65537.h"
#include "matrix_pack.h"
#include "qi_internal.h"
#include "qi_plan.h"

namespace qi {

// Non-systematic encodes with K <= 32 run the register FNT codelets; at
// K = 64 the matrix-core kernel over the Vandermonde generator is faster
// (cfg3: 1.04 vs 1.17 ms, profiles/r2_ab_enc_matrix.txt): a 64-point
// codelet pass needs ~15.5 VALU per output, the MFMA epilogue ~6.  At
// K = 16 (cfg2) the codelets win (3.65 vs 3.75 ms).  K = 128, 256 have no
// codelet (registers).  QI_PLAN_ENC_MATRIX / QI_PLAN_ENC_CODELETS
// (qi_plan_create_ex) force either kernel at K <= 64 (parity tests of both).
static bool enc_matrix(int K, int flags)
{
    if (K > 64)
        return true;
    if (flags & QI_PLAN_ENC_MATRIX)
        return true;
    if (flags & QI_PLAN_ENC_CODELETS)
        return false;
    return K >= 64;
}

// 256 < k <= 640: the matrix-core encode's generator (n_outputs x k,
// packed) is built only while it stays small; larger codes encode on the NTT
// engine (a k = 384 generator for m near 65536 would take ~250 MB of device
// memory).  384 < k <= 640: systematic codes only (k600 systematic encode
// on the NTT engine: interpolation + NTT_n, 6.1 ms per 16 stripes, about
// 3x its non-systematic encode, which stays there)
static bool big_generator_ok(int k, int n_outputs, int sys)
{
    if (k > kMatMaxKin || (k > kMatGenMaxKin && !sys))
        return false;
    const long long e = static_cast<long long>(k) * n_outputs;
    return e <= (sys ? (1LL << 20) : (1LL << 21));
}

static uint32_t addm(uint32_t a, uint32_t b)
{
    const uint32_t c = a + b;
    return c >= 65537u ? c - 65537u : c;
}
static uint32_t subm(uint32_t a, uint32_t b)
{
    return a >= b ? a - b : a + 65537u - b;
}

// Lagrange basis for points x_i = r^{ids[i]} (the closed form of the
// interpolation performed by FecCode::decode_apply, src/fec_base.h:682-738).
std::vector<uint32_t> lagrange_matrix(int k, uint32_t r, const uint32_t* ids,
                                      int mode, const uint32_t* eval, int R)
{
    std::vector<uint32_t> x(k), A(k + 1, 0), q(k), M(static_cast<size_t>(R) * k);
    for (int i = 0; i < k; i++)
        x[i] = powmod_c(r, ids[i]);
    A[0] = 1;
    for (int i = 0; i < k; i++) {
        const uint32_t neg = subm(0, x[i]);
        A[i + 1] = A[i];
        for (int d = i; d > 0; d--)
            A[d] = addm(A[d - 1], mulmod_c(A[d], neg));
        A[0] = mulmod_c(A[0], neg);
    }
    std::vector<uint32_t> dinv(k);  // 1 / A'(x_i) = 1 / prod_{j != i} (x_i - x_j)
    for (int i = 0; i < k; i++) {
        uint32_t den = 1;
        for (int j = 0; j < k; j++)
            if (j != i)
                den = mulmod_c(den, subm(x[i], x[j]));
        dinv[i] = invmod_c(den);
    }
    if (mode != 0) {
        // evaluation rows: M[t][i] = Q_i(e_t) / A'(x_i) with Q_i(e_t) = A(e_t) /
        // (e_t - x_i), or delta_ij where e_t = x_j; a row's k inverses from
        // one inversion (prefix products walked back): O(R k) where a Horner
        // of every Q_i at every e_t took O(R k^2) (seconds at k = 600, R =
        // 1400)
        std::vector<uint32_t> pre(k);
        for (int t = 0; t < R; t++) {
            const uint32_t e = eval[t];
            uint32_t ae = 0;  // A(e), A monic of degree k
            for (int j = k; j >= 0; j--)
                ae = addm(mulmod_c(ae, e), A[j]);
            uint32_t acc = 1;
            int hit = -1;
            for (int i = 0; i < k; i++) {
                const uint32_t d = subm(e, x[i]);
                hit = d ? hit : i;
                pre[i] = acc;
                acc = mulmod_c(acc, d ? d : 1u);
            }
            uint32_t inv = invmod_c(acc);
            uint32_t* row = M.data() + static_cast<size_t>(t) * k;
            for (int i = k - 1; i >= 0; i--) {
                const uint32_t d = subm(e, x[i]);
                const uint32_t inv_i = mulmod_c(inv, pre[i]);
                inv = mulmod_c(inv, d ? d : 1u);
                row[i] = hit >= 0 ? (i == hit ? 1u : 0u) : mulmod_c(mulmod_c(ae, inv_i), dinv[i]);
            }
        }
        return M;
    }
    for (int i = 0; i < k; i++) {
        q[k - 1] = A[k];
        for (int j = k - 1; j >= 1; j--)
            q[j - 1] = addm(A[j], mulmod_c(x[i], q[j]));
        for (int t = 0; t < R; t++)
            M[static_cast<size_t>(t) * k + i] = mulmod_c(q[t], dinv[i]);
    }
    return M;
}

// unit scale s for an MFMA row (s = 1 unless some entry is 32640), with
// |s^-1| <= 32766 (the epilogue's y * s^-1 stays below 2^31)
static uint32_t mf_row_scale(const uint32_t* row, int kin)
{
    for (uint32_t s = 1;; s++) {
        const int32_t si = s == 1 ? 1 : balanced(powmod_c(s, 65535u));
        if (iabs32(si) > 32766)
            continue;
        bool ok = true;
        for (int i = 0; i < kin && ok; i++)
            ok = coef_mf_ok(balanced(mulmod_c(row[i], s)));
        if (ok)
            return s;
    }
}

bool mf_row_scaled(const uint32_t* row, int kin)
{
    return mf_row_scale(row, kin) != 1;
}

void pack_matrix(const MatLayout& L, const uint32_t* M, int32_t* block)
{
    std::memset(block, 0, L.words() * sizeof(int32_t));
    for (int t = 0; t < L.R; t++)
        pack_row(M + static_cast<size_t>(t) * L.kin, L, t, block);
    if (!L.KS())
        return;
    // the MFMA section from rows scaled for the i8 split alone
    std::vector<int32_t> rows(static_cast<size_t>(L.R) * L.kin);
    for (int t = 0; t < L.R; t++) {
        const uint32_t* row = M + static_cast<size_t>(t) * L.kin;
        const uint32_t s = mf_row_scale(row, L.kin);
        uint64_t sum = 0;
        for (int i = 0; i < L.kin; i++) {
            const uint32_t c = mulmod_c(row[i], s);
            rows[static_cast<size_t>(t) * L.kin + i] = static_cast<int32_t>(c);
            sum += c;
        }
        block[L.kmf() + t] = static_cast<int32_t>(
            mulmod_c(static_cast<uint32_t>(sum % 65537u), 32896u));
        block[L.rscale_mf() + t] = s == 1 ? 1 : balanced(powmod_c(s, 65535u));
    }
    for (size_t d = 0; d < L.mf_words(); d++)
        block[L.mf() + d] = pack_mf_dword(L, rows.data(), d);
}

}  // namespace qi

using namespace qi;

extern "C" {

int qi_gpu_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}

qi_plan* qi_plan_create(int k, int m, int systematic)
{
    return qi_plan_create_ex(k, m, systematic, 0);
}

qi_plan* qi_plan_create_ex(int k, int m, int systematic, int flags)
{
    if (flags & ~(QI_PLAN_ENC_MATRIX | QI_PLAN_ENC_CODELETS) ||
        (flags & QI_PLAN_ENC_MATRIX && flags & QI_PLAN_ENC_CODELETS))
        return nullptr;
    if (k < 1 || m < 1 || k + m > 65536 || 2 * k >= 65537)
        return nullptr;
    if (qi_gpu_device_count() < 1)
        return nullptr;
    qi_plan* p = new (std::nothrow) qi_plan();
    if (!p)
        return nullptr;
    p->k = k;
    p->m = m;
    p->sys = systematic ? 1 : 0;
    p->code_len = k + m;
    p->n_outputs = p->sys ? m : k + m;
    p->n = static_cast<int>(ceil2(static_cast<uint32_t>(k + m)));
    p->K = static_cast<int>(ceil2(static_cast<uint32_t>(k)));
    p->r = root_of_unity(static_cast<uint32_t>(p->n));
    (void)hipGetDevice(&p->device);

    bool ok = hipMalloc(&p->d_err, 4) == hipSuccess && hipMemset(p->d_err, 0, 4) == hipSuccess;
    if (ok && p->K > 256) {
        // k > 256: NTT-structured encode/decode (ntt.hip), any k + m <= 65536;
        // up to k = 384 the matrix cores also take the whole-tile batches
        // (qi_gpu.cpp use_matrix: words a multiple of 1024), with the
        // generator below and per-stripe k x k contexts
        p->ntt = 1;
        // 384 < k <= 640: the decodes on the matrix cores (KS = 40, two K
        // chunks), unless the code misses few symbols (the erasure decode's
        // O(e^2 + n log n) per column beats O(k^2))
        p->mbig = k <= kMatGenMaxKin || (k <= kMatMaxKin && !eras_shape(k, p->n)) ? 1 : 0;
        ok = ntt_plan_init(p) == 0;
    }
    if (ok && (!p->ntt || p->mbig)) {
        // twist factors w^{v t} for the encode passes (K <= 32; K = 64 to
        // 256 encode on the matrix cores)
        if (!p->ntt && !p->sys && !enc_matrix(p->K, flags)) {
            const int passes = p->n / p->K;
            std::vector<int32_t> tw(static_cast<size_t>(passes) * p->K);
            for (int v = 0; v < passes; v++)
                for (int t = 0; t < p->K; t++)
                    tw[static_cast<size_t>(v) * p->K + t] = balanced(powmod_c(
                        p->r, static_cast<uint32_t>((static_cast<long long>(v) * t) % p->n)));
            ok = hipMalloc(&p->d_twist, tw.size() * 4) == hipSuccess &&
                 hipMemcpy(p->d_twist, tw.data(), tw.size() * 4, hipMemcpyHostToDevice) ==
                     hipSuccess;
        }
        // generator matrix for the systematic encode (and the matrix-core
        // A/B knob of the non-systematic one): outputs x inputs
        const bool gen = p->mbig ? big_generator_ok(k, p->n_outputs, p->sys)
                                 : p->sys || enc_matrix(p->K, flags);
        if (ok && gen) {
            const int kp = matrix_kp(k);
            MatLayout L{p->n_outputs, k, kp};
            std::vector<uint32_t> M;
            if (p->sys) {
                std::vector<uint32_t> ids(k), ev(m);
                for (int i = 0; i < k; i++)
                    ids[i] = static_cast<uint32_t>(i);
                for (int i = 0; i < m; i++)
                    ev[i] = powmod_c(p->r, static_cast<uint32_t>(k + i));
                // parity i = P(r^{k+i}) where P interpolates data at r^0..r^{k-1}
                // (src/fec_rs_fnt.h:204-251 SYSTEMATIC branch)
                M = lagrange_matrix(k, p->r, ids.data(), 1, ev.data(), m);
            } else {
                M.resize(static_cast<size_t>(p->n_outputs) * k);
                for (int i = 0; i < p->n_outputs; i++)
                    for (int t = 0; t < k; t++)
                        M[static_cast<size_t>(i) * k + t] = powmod_c(
                            p->r, static_cast<uint32_t>((static_cast<long long>(i) * t) % p->n));
            }
            // rows whose matrix-core tiles need a unit scale (an entry of
            // 32640, the one residue the i8 split cannot reach) go last:
            // the epilogue multiplies back by the scale for a whole 16-row
            // block when any of its rows needs it.  Vandermonde rows hit
            // 32640 (a root of unity) often: at cfg3, 160 of 1024 rows,
            // spread over 52 of the 64 blocks in natural order, 10 after.
            const int R = p->n_outputs;
            std::vector<int32_t> perm;
            for (int pass = 0; pass < 2; pass++)
                for (int i = 0; i < R; i++)
                    if (mf_row_scaled(M.data() + static_cast<size_t>(i) * k, k) == (pass == 1))
                        perm.push_back(i);
            std::vector<uint32_t> Mp(M.size());
            for (int i = 0; i < R; i++)
                std::copy_n(M.begin() + static_cast<size_t>(perm[i]) * k, k,
                            Mp.begin() + static_cast<size_t>(i) * k);
            std::vector<int32_t> blk(L.words());
            pack_matrix(L, Mp.data(), blk.data());
            p->gen = L;
            ok = hipMalloc(&p->d_gen, blk.size() * 4) == hipSuccess &&
                 hipMemcpy(p->d_gen, blk.data(), blk.size() * 4, hipMemcpyHostToDevice) ==
                     hipSuccess &&
                 hipMalloc(&p->d_rowmap, perm.size() * 4) == hipSuccess &&
                 hipMemcpy(p->d_rowmap, perm.data(), perm.size() * 4, hipMemcpyHostToDevice) ==
                     hipSuccess;
        }
        // identity output rows of the k x k decode matrices
        std::vector<int32_t> id(k);
        for (int i = 0; i < k; i++)
            id[i] = i;
        ok = ok && hipMalloc(&p->d_rowid, id.size() * 4) == hipSuccess &&
             hipMemcpy(p->d_rowid, id.data(), id.size() * 4, hipMemcpyHostToDevice) == hipSuccess;

    }
    if (!ok) {
        qi_plan_destroy(p);
        return nullptr;
    }
    return p;
}

void qi_plan_destroy(qi_plan* p)
{
    if (!p)
        return;
    if (p->d_twist)
        (void)hipFree(p->d_twist);
    if (p->d_gen)
        (void)hipFree(p->d_gen);
    if (p->d_rowmap)
        (void)hipFree(p->d_rowmap);
    if (p->d_rowid)
        (void)hipFree(p->d_rowid);
    if (p->d_err)
        (void)hipFree(p->d_err);
    ntt_plan_free(p);
    p->host.release();
    delete p;
}

int qi_plan_n(const qi_plan* p)
{
    return p ? p->n : -1;
}

int qi_plan_n_outputs(const qi_plan* p)
{
    return p ? p->n_outputs : -1;
}

}  // extern "C"
