/*
 * qi_oracle.c -- TEST INFRASTRUCTURE ONLY (see qi_oracle.h).
 *
 * Plain-C restatement of the reference RS-FNT path.  The algorithm is the
 * reference's, restated column by column (the reference's Buffers code runs
 * the same per-symbol arithmetic on whole packet rows; columns never
 * interact, src/fec_base.h:1103-1150).  Citations are reference file:line.
 */
#include "qi_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* GF(65537): src/gf_ring.h:214-286 (RingModN<uint32_t>, 64-bit product) */

uint32_t qo_add(uint32_t a, uint32_t b)
{
    uint32_t c = a + b; /* src/gf_ring.h:214-224 */
    return c >= QO_Q ? c - QO_Q : c;
}

uint32_t qo_sub(uint32_t a, uint32_t b)
{
    return a >= b ? a - b : QO_Q - (b - a); /* src/gf_ring.h:226-236 */
}

uint32_t qo_mul(uint32_t a, uint32_t b)
{
    return (uint32_t)(((uint64_t)a * b) % QO_Q); /* src/gf_ring.h:238-244 */
}

uint32_t qo_exp(uint32_t a, uint32_t e)
{
    uint32_t r = 1; /* src/gf_ring.h:280-330 (square and multiply) */
    a %= QO_Q;
    while (e) {
        if (e & 1)
            r = qo_mul(r, a);
        a = qo_mul(a, a);
        e >>= 1;
    }
    return r;
}

uint32_t qo_inv(uint32_t a)
{
    return qo_exp(a, QO_Q - 2); /* same value as src/gf_ring.h:259-278 */
}

/* Primitive root of GF(65537) is 3: src/gf_ring.h:624-660 rejects 2 since
 * 2^32768 == 1.  nth root = root^((q-1)/gcd(n,q-1)): src/gf_ring.h:774-781 */
uint32_t qo_nth_root(uint32_t n)
{
    uint32_t a = n, b = QO_Q - 1, t;
    while (b) {
        t = a % b;
        a = b;
        b = t;
    }
    return qo_exp(3, (QO_Q - 1) / a);
}

/* Smallest power of two >= n (all prime factors of q-1 are 2):
 * src/arith.h:692-712 */
uint32_t qo_code_len(uint32_t n)
{
    uint32_t x = 1;
    while (x < n)
        x <<= 1;
    return x;
}

static unsigned bitrev(unsigned i, unsigned log_n)
{
    unsigned r = 0, b;
    for (b = 0; b < log_n; b++)
        r |= ((i >> b) & 1u) << (log_n - 1 - b);
    return r;
}

static unsigned ilog2(unsigned n)
{
    unsigned l = 0;
    while ((1u << l) < n)
        l++;
    return l;
}

/* ------------------------------------------------------------------ */
/* Radix-2 DIT forward with replicated zero padding: src/fft_2n.h:269-318 */
void qo_fft(int n, int data_len, uint32_t w, const uint32_t* in, int in_len,
            uint32_t* out)
{
    unsigned log_n = ilog2((unsigned)n);
    unsigned group_len =
        (unsigned)((in_len > data_len) ? n / in_len : n / data_len);
    unsigned idx, i, m, j;
    uint32_t* W = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);

    /* W[i] = w^i: src/gf_ring.h:494-500 */
    W[0] = 1;
    for (i = 1; i < (unsigned)n; i++)
        W[i] = qo_mul(W[i - 1], w);

    for (idx = 0; idx < (unsigned)in_len; idx++) {
        unsigned s = bitrev(idx, log_n);
        for (i = s; i < s + group_len; i++)
            out[i] = in[idx];
    }
    for (idx = (unsigned)in_len; idx < (unsigned)data_len; idx++) {
        unsigned s = bitrev(idx, log_n);
        for (i = s; i < s + group_len; i++)
            out[i] = 0;
    }
    for (m = group_len; m < (unsigned)n; m *= 2) {
        unsigned dm = 2 * m, ratio = (unsigned)n / dm;
        for (j = 0; j < m; j++) {
            uint32_t r = W[j * ratio];
            for (i = j; i < (unsigned)n; i += dm) {
                uint32_t a = out[i];
                uint32_t b = qo_mul(r, out[i + m]);
                out[i] = qo_add(a, b);
                out[i + m] = qo_sub(a, b);
            }
        }
    }
    free(W);
}

/* DIF inverse (unnormalised), natural-order output: src/fft_2n.h:321-343
 * (the Buffers variant src/fft_2n.h:516-561 computes the same transform of
 * the zero-padded input). */
void qo_fft_inv(int n, uint32_t w, const uint32_t* in, uint32_t* out)
{
    unsigned log_n = ilog2((unsigned)n);
    unsigned i, m, j;
    uint32_t inv_w = qo_inv(w);
    uint32_t* iW = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);

    iW[0] = 1;
    for (i = 1; i < (unsigned)n; i++)
        iW[i] = qo_mul(iW[i - 1], inv_w);

    memcpy(out, in, sizeof(uint32_t) * (size_t)n);
    for (m = (unsigned)n / 2; m >= 1; m /= 2) {
        unsigned dm = 2 * m;
        for (j = 0; j < m; j++) {
            uint32_t r = iW[j * (unsigned)n / dm];
            for (i = j; i < (unsigned)n; i += dm) {
                uint32_t a = out[i], b = out[i + m];
                out[i] = qo_add(a, b);
                out[i + m] = qo_mul(r, qo_sub(a, b));
            }
        }
    }
    /* bit_rev_permute: src/fft_2n.h:232-240 */
    for (i = 0; i < (unsigned)n; i++) {
        unsigned r = bitrev(i, log_n);
        if (r < i) {
            uint32_t t = out[i];
            out[i] = out[r];
            out[r] = t;
        }
    }
    free(iW);
}

/* ------------------------------------------------------------------ */
/* Codec plan: src/fec_rs_fnt.h:69-163 */
int qo_codec_init(qo_codec* c, int k, int m, int sys)
{
    /* oracle limits: k <= QO_KMAX, k + m <= 65536 (fixed-size scratch) */
    if (k < 1 || m < 1 || k > QO_KMAX || k + m > 65536)
        return -1;
    c->sys = sys ? 1 : 0;
    c->k = k;
    c->m = m;
    c->code_len = k + m;
    c->n_outputs = c->sys ? m : k + m;
    c->n = (int)qo_code_len((uint32_t)(k + m));        /* :106 */
    c->r = qo_nth_root((uint32_t)c->n);                 /* :109 */
    c->data_len = (int)qo_code_len((uint32_t)k);        /* :111 */
    c->len_2k = (int)qo_code_len((uint32_t)(2 * k));    /* :119 */
    return 0;
}

/* DecodeContext ctor+init: src/fec_context.h:66-142, :232-274;
 * vx from src/fec_base.h:758-793 (x_i = r^{id_i}, vx_zero = -1). */
int qo_ctx_init(const qo_codec* c, qo_ctx* ctx, const uint32_t* ids)
{
    int k = c->k, n = c->n, i, d;
    uint32_t *A, *Ad, *A_fft, *A2k;

    if (k > QO_KMAX || c->len_2k > 2 * QO_KMAX)
        return -1;
    A = (uint32_t*)calloc((size_t)n + 1, sizeof(uint32_t));
    Ad = (uint32_t*)calloc((size_t)n, sizeof(uint32_t));
    A_fft = (uint32_t*)calloc((size_t)n, sizeof(uint32_t));
    A2k = (uint32_t*)calloc((size_t)c->len_2k, sizeof(uint32_t));

    ctx->k = k;
    for (i = 0; i < k; i++)
        ctx->ids[i] = ids[i];

    /* A(x) = prod (x - x_i): Poly::mul_to_x_plus_coef src/vec_poly.h:218-228 */
    A[0] = 1;
    for (i = 0; i < k; i++) {
        uint32_t coef = qo_sub(0, qo_exp(c->r, ids[i]));
        uint32_t top = A[i];
        for (d = i; d > 0; d--)
            A[d] = qo_add(A[d - 1], qo_mul(A[d], coef));
        A[0] = qo_mul(A[0], coef);
        A[i + 1] = top;
    }
    /* A'(x): Poly::derivative src/vec_poly.h:141-148 */
    for (d = 1; d <= k; d++)
        Ad[d - 1] = qo_mul((uint32_t)d % QO_Q, A[d]);
    /* A'(x_j) for all j via n-point fft of the length-n vector */
    qo_fft(n, c->data_len, c->r, Ad, n, A_fft);
    /* inv_A_i = 1 / (A'(x_i) * x_i): src/fec_context.h:259-267 */
    for (i = 0; i < k; i++)
        ctx->inv_A_i[i] =
            qo_inv(qo_mul(A_fft[ids[i]], qo_exp(c->r, ids[i])));
    /* A_fft_2k = FFT_2k(A zero-extended): src/fec_context.h:270-273 */
    for (d = 0; d <= k && d < c->len_2k; d++)
        A2k[d] = A[d];
    qo_fft(c->len_2k, c->len_2k, qo_nth_root((uint32_t)c->len_2k), A2k,
           c->len_2k, ctx->A_fft_2k);

    free(A);
    free(Ad);
    free(A_fft);
    free(A2k);
    return 0;
}

/* decode_apply: src/fec_base.h:1418-1448 (Buffers) / :740-792 (Vector);
 * SYS tail src/fec_base.h:1349-1354. */
static void decode_apply(const qo_codec* c, const qo_ctx* ctx,
                         const uint32_t* words, uint32_t* coefs)
{
    int k = c->k, n = c->n, L = c->len_2k, i;
    uint32_t* v1n = (uint32_t*)calloc((size_t)n, sizeof(uint32_t));
    uint32_t* v2n = (uint32_t*)calloc((size_t)n, sizeof(uint32_t));
    uint32_t* v1 = (uint32_t*)calloc((size_t)L, sizeof(uint32_t));
    uint32_t* v2 = (uint32_t*)calloc((size_t)L, sizeof(uint32_t));
    uint32_t wL = qo_nth_root((uint32_t)L), invL = qo_inv((uint32_t)L);

    /* N(x) = sum_i (v_i * inv_A_i) x^{z_i} */
    for (i = 0; i < k; i++)
        v1n[ctx->ids[i]] = qo_mul(words[i], ctx->inv_A_i[i]);
    qo_fft_inv(n, c->r, v1n, v2n);
    /* FFT_2k of the first k outputs (zero extended) */
    qo_fft(L, L, wL, v2n, k, v1);
    for (i = 0; i < L; i++)
        v1[i] = qo_mul(v1[i], ctx->A_fft_2k[i]);
    /* ifft = fft_inv * len_2k^-1: src/fft_2n.h:630-639 */
    qo_fft_inv(L, wL, v1, v2);
    for (i = 0; i < k; i++)
        coefs[i] = qo_sub(0, qo_mul(v2[i], invL));
    free(v1n);
    free(v2n);
    free(v1);
    free(v2);
}

void qo_decode_column(const qo_codec* c, const qo_ctx* ctx,
                      const uint32_t* words, uint32_t* data)
{
    decode_apply(c, ctx, words, data);
    if (c->sys) {
        /* fft(dec_inter_codeword, output); keep rows 0..k-1 */
        uint32_t* cw = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)c->n);
        uint32_t tmp[QO_KMAX];
        int i;
        for (i = 0; i < c->k; i++)
            tmp[i] = data[i];
        qo_fft(c->n, c->data_len, c->r, tmp, c->k, cw);
        for (i = 0; i < c->k; i++)
            data[i] = cw[i];
        free(cw);
    }
}

/* RsFnt::encode(Buffers): src/fec_rs_fnt.h:236-251 */
void qo_encode_column(const qo_codec* c, const qo_ctx* enc_ctx,
                      const uint32_t* data, uint32_t* codeword)
{
    if (c->sys) {
        uint32_t inter[QO_KMAX];
        /* decode_data over ids 0..k-1: src/fec_rs_fnt.h:204-234 */
        decode_apply(c, enc_ctx, data, inter);
        qo_fft(c->n, c->data_len, c->r, inter, c->k, codeword);
    } else {
        qo_fft(c->n, c->data_len, c->r, data, c->k, codeword);
    }
}

/* ------------------------------------------------------------------ */
/* Block API */

static void oor_add(uint32_t* list, uint32_t* count, uint32_t cap,
                    uint32_t off)
{
    if (*count < cap)
        list[*count] = off;
    (*count)++;
}

/* encode_blocks_vertical: src/fec_base.h:1066-1151 with
 * encode_post_process src/fec_rs_fnt.h:253-269 (OOR = value 65536, stored
 * as 0 by vec::unpack's u16 truncation src/vec_cast.h:133-163). */
void qo_encode_blocks(const qo_codec* c, uint8_t* const* data,
                      uint8_t* const* outputs, size_t block_bytes,
                      uint32_t* oor, uint32_t* oor_count, uint32_t oor_cap)
{
    size_t words = block_bytes / 2, j;
    int k = c->k, n = c->n, i, first = c->sys ? k : 0;
    qo_ctx* ctx = NULL;
    uint32_t in[QO_KMAX];
    uint32_t* cw = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);

    if (c->sys) {
        uint32_t ids[QO_KMAX];
        ctx = (qo_ctx*)malloc(sizeof(qo_ctx));
        for (i = 0; i < k; i++)
            ids[i] = (uint32_t)i;
        qo_ctx_init(c, ctx, ids); /* src/fec_rs_fnt.h:141-156 */
    }
    for (i = 0; i < c->n_outputs; i++)
        oor_count[i] = 0;
    for (j = 0; j < words; j++) {
        for (i = 0; i < k; i++)
            in[i] = (uint32_t)data[i][2 * j] |
                    ((uint32_t)data[i][2 * j + 1] << 8);
        qo_encode_column(c, ctx, in, cw);
        for (i = 0; i < c->n_outputs; i++) {
            uint32_t v = cw[first + i];
            if (v & 65536u)
                oor_add(oor + (size_t)i * oor_cap, &oor_count[i], oor_cap,
                        (uint32_t)j);
            if (outputs[i]) {
                outputs[i][2 * j] = (uint8_t)v;
                outputs[i][2 * j + 1] = (uint8_t)(v >> 8);
            }
        }
    }
    free(cw);
    free(ctx);
}

static int cmp_u32(const void* a, const void* b)
{
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}

/* decode_blocks_vertical: src/fec_base.h:1177-1321, decode_prepare
 * src/fec_base.h:1361-1404. */
int qo_decode_blocks(const qo_codec* c, uint8_t* const* data,
                     uint8_t* const* parities, const uint32_t* oor,
                     const uint32_t* oor_count, uint32_t oor_cap,
                     const int* missing, const int* wanted,
                     size_t block_bytes)
{
    int k = c->k, i, fi = 0, avail_data = 0;
    uint32_t ids[QO_KMAX] = {0};
    const uint8_t* src[QO_KMAX];
    const uint32_t* marks[QO_KMAX];
    uint32_t nmarks[QO_KMAX];
    uint32_t* sorted[QO_KMAX];
    uint32_t pos[QO_KMAX];
    size_t words = block_bytes / 2, j;
    qo_ctx* ctx;
    uint32_t in[QO_KMAX], out[QO_KMAX];

    if (c->sys) {
        for (i = 0; i < k; i++) {
            if (!missing[i]) {
                ids[fi] = (uint32_t)i;
                src[fi] = data[i];
                marks[fi] = NULL; /* systematic data rows skipped :1375 */
                nmarks[fi] = 0;
                fi++;
            }
            avail_data = fi;
            if (fi == k)
                return 1; /* src/fec_base.h:1208-1211 */
        }
    }
    (void)avail_data;
    for (i = 0; i < c->n_outputs && fi < k; i++) {
        int id = c->sys ? k + i : i;
        if (!missing[id]) {
            ids[fi] = (uint32_t)id;
            src[fi] = parities[i];
            marks[fi] = oor + (size_t)i * oor_cap;
            nmarks[fi] = oor_count[i] < oor_cap ? oor_count[i] : oor_cap;
            fi++;
        }
    }
    if (fi < k)
        return 0;
    /* ids are already ascending (fragments_ids.sort(), :1236) */

    ctx = (qo_ctx*)malloc(sizeof(qo_ctx));
    qo_ctx_init(c, ctx, ids);
    /* props.sort() src/fec_context.h:93-97 */
    for (i = 0; i < k; i++) {
        sorted[i] = (uint32_t*)malloc(sizeof(uint32_t) * (nmarks[i] + 1));
        if (nmarks[i])
            memcpy(sorted[i], marks[i], sizeof(uint32_t) * nmarks[i]);
        qsort(sorted[i], nmarks[i], sizeof(uint32_t), cmp_u32);
        pos[i] = 0;
    }
    for (j = 0; j < words; j++) {
        for (i = 0; i < k; i++) {
            in[i] = (uint32_t)src[i][2 * j] |
                    ((uint32_t)src[i][2 * j + 1] << 8);
            /* restore OOR symbols (value q-1 = 65536) */
            while (pos[i] < nmarks[i] && sorted[i][pos[i]] < j)
                pos[i]++;
            while (pos[i] < nmarks[i] && sorted[i][pos[i]] == j) {
                in[i] = 65536u;
                pos[i]++;
            }
        }
        qo_decode_column(c, ctx, in, out);
        for (i = 0; i < k; i++) {
            if (wanted[i]) {
                data[i][2 * j] = (uint8_t)out[i];
                data[i][2 * j + 1] = (uint8_t)(out[i] >> 8);
            }
        }
    }
    for (i = 0; i < k; i++)
        free(sorted[i]);
    free(ctx);
    return 1;
}

/* ------------------------------------------------------------------ */
/* RS-NF4: src/fec_rs_nf4.h.  NF4<T> (src/gf_nf4.h:116-132) is the ring of
 * gf_n = word_size/2 tuples over GF(65537) with componentwise arithmetic
 * (:214-316); the code uses the prime field's n-th root replicated in every
 * component (get_nth_root :450-455) and the same Radix2 transforms as RsFnt
 * (src/fec_rs_nf4.h:78-96).  So component c of word j -- the 16-bit lane
 * j*g + c of the byte stream (vec::pack word_size bytes per word, then
 * NF4::pack :355-365) -- is one RS-FNT column.  encode_post_process
 * (src/fec_rs_nf4.h:271-289, NF4::unpack :391-446) records, per output and
 * word, the bitmask of components equal to 65536 (stored as 0);
 * decode_prepare (:291-317, NF4::pack(a, flag) :372-383) restores them. */

void qo_nf4_encode_blocks(const qo_codec* c, int word_size,
                          uint8_t* const* data, uint8_t* const* outputs,
                          size_t block_bytes, uint32_t* oor, uint32_t* flags,
                          uint32_t* oor_count, uint32_t oor_cap)
{
    const int g = word_size / 2, k = c->k, no = c->n_outputs;
    const size_t words = block_bytes / (size_t)word_size; /* fec_base.h:1083 */
    uint32_t in[QO_KMAX];
    uint32_t* cw = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)c->n);
    uint32_t* mask = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)no);
    size_t j;
    int comp, i;

    for (i = 0; i < no; i++)
        oor_count[i] = 0;
    for (j = 0; j < words; j++) {
        for (i = 0; i < no; i++)
            mask[i] = 0;
        for (comp = 0; comp < g; comp++) {
            const size_t lane = j * (size_t)g + (size_t)comp;
            for (i = 0; i < k; i++)
                in[i] = (uint32_t)data[i][2 * lane] |
                        ((uint32_t)data[i][2 * lane + 1] << 8);
            qo_encode_column(c, NULL, in, cw);
            for (i = 0; i < no; i++) {
                const uint32_t v = cw[i];
                if (v & 65536u)
                    mask[i] |= 1u << comp;
                if (outputs[i]) {
                    outputs[i][2 * lane] = (uint8_t)v;
                    outputs[i][2 * lane + 1] = (uint8_t)(v >> 8);
                }
            }
        }
        for (i = 0; i < no; i++) {
            if (!mask[i])
                continue;
            if (oor_count[i] < oor_cap) {
                oor[(size_t)i * oor_cap + oor_count[i]] = (uint32_t)j;
                flags[(size_t)i * oor_cap + oor_count[i]] = mask[i];
            }
            oor_count[i]++;
        }
    }
    free(mask);
    free(cw);
}

static int cmp_u64(const void* a, const void* b)
{
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

int qo_nf4_decode_blocks(const qo_codec* c, int word_size,
                         uint8_t* const* data, uint8_t* const* parities,
                         const uint32_t* oor, const uint32_t* flags,
                         const uint32_t* oor_count, uint32_t oor_cap,
                         const int* missing, const int* wanted,
                         size_t block_bytes)
{
    const int g = word_size / 2, k = c->k;
    const size_t words = block_bytes / (size_t)word_size;
    uint32_t ids[QO_KMAX] = {0};
    const uint8_t* src[QO_KMAX];
    uint64_t* marks[QO_KMAX]; /* word << 8 | component mask, sorted */
    uint32_t nmarks[QO_KMAX], pos[QO_KMAX], cur[QO_KMAX];
    uint32_t in[QO_KMAX], out[QO_KMAX];
    int i, fi = 0, comp;
    size_t j, e;
    qo_ctx* ctx;

    /* first k present fragments (src/fec_base.h:1217-1236, non-systematic) */
    for (i = 0; i < c->n_outputs && fi < k; i++) {
        if (!missing[i]) {
            const uint32_t n = oor_count[i] < oor_cap ? oor_count[i] : oor_cap;
            ids[fi] = (uint32_t)i;
            src[fi] = parities[i];
            marks[fi] = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
            for (e = 0; e < n; e++)
                marks[fi][e] = ((uint64_t)oor[(size_t)i * oor_cap + e] << 8) |
                               flags[(size_t)i * oor_cap + e];
            qsort(marks[fi], n, sizeof(uint64_t), cmp_u64); /* fec_context.h:93-97 */
            nmarks[fi] = n;
            pos[fi] = 0;
            fi++;
        }
    }
    if (fi < k) {
        for (i = 0; i < fi; i++)
            free(marks[i]);
        return 0;
    }
    ctx = (qo_ctx*)malloc(sizeof(qo_ctx));
    qo_ctx_init(c, ctx, ids);
    for (j = 0; j < words; j++) {
        for (i = 0; i < k; i++) {
            cur[i] = 0;
            while (pos[i] < nmarks[i] && (marks[i][pos[i]] >> 8) < j)
                pos[i]++;
            while (pos[i] < nmarks[i] && (marks[i][pos[i]] >> 8) == j)
                cur[i] |= (uint32_t)(marks[i][pos[i]++] & 0xffu);
        }
        for (comp = 0; comp < g; comp++) {
            const size_t lane = j * (size_t)g + (size_t)comp;
            for (i = 0; i < k; i++) {
                in[i] = (uint32_t)src[i][2 * lane] |
                        ((uint32_t)src[i][2 * lane + 1] << 8);
                if ((cur[i] >> comp) & 1u)
                    in[i] = 65536u; /* NF4::pack(a, flag) */
            }
            qo_decode_column(c, ctx, in, out);
            for (i = 0; i < k; i++) {
                if (wanted[i]) {
                    data[i][2 * lane] = (uint8_t)out[i];
                    data[i][2 * lane + 1] = (uint8_t)(out[i] >> 8);
                }
            }
        }
    }
    for (i = 0; i < k; i++)
        free(marks[i]);
    free(ctx);
    return 1;
}

/* ------------------------------------------------------------------ */
/* C-ABI semantics: src/quadiron_c.cpp */

int qo_metadata_size(size_t block_size)
{
    return (int)(((block_size / 65536) + 16) * 4); /* :61-71 */
}

static uint32_t be32(uint32_t x)
{
    return ((x & 0xffu) << 24) | ((x & 0xff00u) << 8) | ((x >> 8) & 0xff00u) |
           (x >> 24);
}

static void put32(uint8_t* p, uint32_t v)
{
    memcpy(p, &v, 4);
}

static uint32_t get32(const uint8_t* p)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

/* Properties::fnt_serialize src/property.h:104-118 (last dword untouched) */
static int fnt_serialize(uint8_t* hdr, int n_dwords, const uint32_t* offs,
                         uint32_t count)
{
    uint32_t i;
    int d;
    if (2 + (int64_t)count > n_dwords)
        return -1;
    put32(hdr, be32(0x464E5431u));
    for (i = 0; i < count; i++)
        put32(hdr + 4 * (2 + i), be32(offs[i]));
    put32(hdr + 4, be32(count));
    for (d = 2 + (int)count; d < n_dwords - 1; d++)
        put32(hdr + 4 * d, 0);
    return 0;
}

/* Properties::fnt_deserialize src/property.h:125-142 */
static int fnt_deserialize(const uint8_t* hdr, int n_dwords, uint32_t* offs,
                           uint32_t* count, uint32_t cap)
{
    uint32_t n, i;
    if (n_dwords < 2)
        return -1;
    if (be32(get32(hdr)) != 0x464E5431u)
        return -1;
    n = be32(get32(hdr + 4));
    if (2 + (uint64_t)n > (uint64_t)n_dwords)
        return -1;
    for (i = 0; i < n && i < cap; i++)
        offs[i] = be32(get32(hdr + 4 * (2 + i)));
    *count = n;
    return 0;
}

int qo_fnt32_encode(const qo_codec* c, uint8_t** data, uint8_t** parity,
                    const int* wanted_idxs, size_t block_size)
{
    int md = qo_metadata_size(block_size), nd = md / 4, i, k = c->k;
    uint32_t cap = (uint32_t)nd;
    uint8_t* in[QO_KMAX];
    uint8_t* out[QO_NMAX];
    uint32_t* oor = (uint32_t*)malloc(sizeof(uint32_t) * cap *
                                      (size_t)c->n_outputs);
    uint32_t* cnt = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)c->n_outputs);
    int ret = 0;

    /* :92-107 buffer offsets; non-sys outputs 0..k-1 go into data */
    for (i = 0; i < k; i++)
        in[i] = data[i] + md;
    for (i = 0; i < c->n_outputs; i++) {
        uint8_t* b = c->sys ? parity[i]
                            : (i < k ? data[i] : parity[i - k]);
        out[i] = wanted_idxs[i] ? b + md : NULL;
    }
    if (!c->sys) {
        /* outputs 0..k-1 overwrite data in place: compute from a copy */
        size_t bb = block_size;
        for (i = 0; i < k; i++) {
            uint8_t* cp = (uint8_t*)malloc(bb ? bb : 1);
            memcpy(cp, in[i], bb);
            in[i] = cp;
        }
    }
    qo_encode_blocks(c, in, out, block_size, oor, cnt, cap);
    if (!c->sys)
        for (i = 0; i < k; i++)
            free(in[i]);
    /* headers: :112-147 */
    if (c->sys) {
        for (i = 0; i < k && !ret; i++)
            ret = fnt_serialize(data[i], nd, NULL, 0);
        for (i = 0; i < c->m && !ret; i++)
            ret = fnt_serialize(parity[i], nd, oor + (size_t)i * cap, cnt[i]);
    } else {
        for (i = 0; i < k && !ret; i++)
            ret = fnt_serialize(data[i], nd, oor + (size_t)i * cap, cnt[i]);
        for (i = 0; i < c->m && !ret; i++)
            ret = fnt_serialize(parity[i], nd, oor + (size_t)(k + i) * cap,
                                cnt[k + i]);
    }
    free(oor);
    free(cnt);
    return ret;
}

/* Deserialize every present coded fragment header; :160-206 / :246-285 */
static int load_props(const qo_codec* c, uint8_t** data, uint8_t** parity,
                      const int* missing, int nd, uint32_t* oor,
                      uint32_t* cnt, uint32_t cap)
{
    int i, k = c->k;
    for (i = 0; i < c->n_outputs; i++)
        cnt[i] = 0;
    if (c->sys) {
        for (i = 0; i < c->m; i++)
            if (!missing[k + i] &&
                fnt_deserialize(parity[i], nd, oor + (size_t)i * cap, &cnt[i],
                                cap))
                return -1;
    } else {
        for (i = 0; i < k; i++)
            if (!missing[i] &&
                fnt_deserialize(data[i], nd, oor + (size_t)i * cap, &cnt[i],
                                cap))
                return -1;
        for (i = 0; i < c->m; i++)
            if (!missing[k + i] &&
                fnt_deserialize(parity[i], nd, oor + (size_t)(k + i) * cap,
                                &cnt[k + i], cap))
                return -1;
    }
    return 0;
}

int qo_fnt32_decode(const qo_codec* c, uint8_t** data, uint8_t** parity,
                    const int* missing_idxs, size_t block_size)
{
    int md = qo_metadata_size(block_size), nd = md / 4, i, k = c->k, res;
    uint32_t cap = (uint32_t)nd;
    uint32_t* oor = (uint32_t*)malloc(sizeof(uint32_t) * cap *
                                      (size_t)c->n_outputs);
    uint32_t* cnt = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)c->n_outputs);
    uint8_t* dv[QO_KMAX];
    uint8_t* pv[QO_NMAX];
    int wanted[QO_KMAX];
    int ret = 0;

    if (load_props(c, data, parity, missing_idxs, nd, oor, cnt, cap)) {
        ret = -1;
        goto out;
    }
    for (i = 0; i < k; i++) {
        dv[i] = data[i] + md;
        wanted[i] = 1;
    }
    for (i = 0; i < c->n_outputs; i++) {
        int id = c->sys ? k + i : i;
        uint8_t* b = c->sys ? parity[i] : (i < k ? data[i] : parity[i - k]);
        pv[i] = missing_idxs[id] ? NULL : b + md;
    }
    if (!c->sys) {
        /* data buffers double as received coded fragments: decode from
         * copies so outputs can be written in place */
        for (i = 0; i < k; i++)
            if (pv[i]) {
                uint8_t* cp = (uint8_t*)malloc(block_size ? block_size : 1);
                memcpy(cp, pv[i], block_size);
                pv[i] = cp;
            }
    }
    res = qo_decode_blocks(c, dv, pv, oor, cnt, cap, missing_idxs, wanted,
                           block_size);
    if (!c->sys)
        for (i = 0; i < k; i++)
            if (!missing_idxs[i])
                free(pv[i]);
    if (!res) {
        ret = -1;
        goto out;
    }
    /* reset metadata of data: :218-226 */
    for (i = 0; i < k && !ret; i++)
        ret = fnt_serialize(data[i], nd, NULL, 0);
out:
    free(oor);
    free(cnt);
    return ret;
}

int qo_fnt32_reconstruct(const qo_codec* c, uint8_t** data, uint8_t** parity,
                         const int* missing_idxs, unsigned destination_idx,
                         size_t block_size)
{
    int md = qo_metadata_size(block_size), nd = md / 4, i, k = c->k, res;
    uint32_t cap = (uint32_t)nd;
    uint32_t* oor = (uint32_t*)malloc(sizeof(uint32_t) * cap *
                                      (size_t)c->n_outputs);
    uint32_t* cnt = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)c->n_outputs);
    uint32_t* eoor = (uint32_t*)malloc(sizeof(uint32_t) * cap *
                                       (size_t)c->n_outputs);
    uint32_t* ecnt = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)c->n_outputs);
    uint8_t* dv[QO_KMAX];
    uint8_t* pv[QO_NMAX];
    uint8_t* ov[QO_NMAX];
    uint8_t* tmp[QO_KMAX];
    int wanted[QO_KMAX];
    int ret = 0, need_decode = 0;

    for (i = 0; i < k; i++)
        tmp[i] = NULL;
    if (load_props(c, data, parity, missing_idxs, nd, oor, cnt, cap)) {
        ret = -1;
        goto out;
    }
    for (i = 0; i < k; i++)
        dv[i] = data[i] ? data[i] + md : NULL;
    for (i = 0; i < c->n_outputs; i++) {
        int id = c->sys ? k + i : i;
        uint8_t* b = c->sys ? parity[i] : (i < k ? data[i] : parity[i - k]);
        pv[i] = (missing_idxs[id] || !b) ? NULL : b + md;
    }
    if (c->sys && destination_idx < (unsigned)k) {
        /* :289-320 */
        for (i = 0; i < k; i++)
            wanted[i] = (unsigned)i == destination_idx;
        res = qo_decode_blocks(c, dv, pv, oor, cnt, cap, missing_idxs, wanted,
                               block_size);
        if (!res) {
            ret = -1;
            goto out;
        }
        ret = fnt_serialize(data[destination_idx], nd, NULL, 0);
        goto out;
    }
    /* :326-352 */
    for (i = 0; i < k; i++)
        wanted[i] = 0;
    if (c->sys) {
        for (i = 0; i < k; i++)
            if (missing_idxs[i]) {
                need_decode = 1;
                wanted[i] = 1;
                tmp[i] = (uint8_t*)calloc(block_size ? block_size : 1, 1);
                dv[i] = tmp[i];
            }
    } else {
        need_decode = 1;
        for (i = 0; i < k; i++) {
            wanted[i] = 1;
            tmp[i] = (uint8_t*)calloc(block_size ? block_size : 1, 1);
            dv[i] = tmp[i];
        }
    }
    if (need_decode) {
        res = qo_decode_blocks(c, dv, pv, oor, cnt, cap, missing_idxs, wanted,
                               block_size);
        if (!res) {
            ret = -1;
            goto out;
        }
    }
    /* :359-406 re-encode the wanted output only */
    for (i = 0; i < c->n_outputs; i++)
        ov[i] = NULL;
    {
        unsigned widx = c->sys ? destination_idx - (unsigned)k
                               : destination_idx;
        if (widx >= (unsigned)c->n_outputs) {
            ret = -1;
            goto out;
        }
        ov[widx] = pv[widx] ? pv[widx] : NULL;
        if (!ov[widx]) {
            uint8_t* b = c->sys ? parity[widx]
                                : (widx < (unsigned)k ? data[widx]
                                                      : parity[widx - k]);
            ov[widx] = b + md;
        }
        qo_encode_blocks(c, dv, ov, block_size, eoor, ecnt, cap);
        {
            uint8_t* b = c->sys ? parity[widx]
                                : (widx < (unsigned)k ? data[widx]
                                                      : parity[widx - k]);
            ret = fnt_serialize(b, nd, eoor + (size_t)widx * cap, ecnt[widx]);
        }
    }
out:
    for (i = 0; i < k; i++)
        free(tmp[i]);
    free(oor);
    free(cnt);
    free(eoor);
    free(ecnt);
    return ret;
}
