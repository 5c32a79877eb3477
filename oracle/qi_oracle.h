/*
 * qi_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of QuadIron's RS-FNT path (Reed-Solomon over GF(65537)
 * with a radix-2 Fermat Number Transform), used as the parity checker for the
 * HIP product path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product library never links it.
 *
 * Parity pinning: checked against golden vectors produced by the reference
 * itself (oracle/_ref, built from /root/reference sources by oracle/Makefile)
 * in tests/golden/ -- see tests/test_oracle_golden.py.
 *
 * Every function cites the reference file:line it restates
 * (paths relative to the reference repository root).
 */
#ifndef QI_ORACLE_H
#define QI_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QO_Q 65537u
/* oracle limits (fixed-size scratch): k <= QO_KMAX, k + m <= 65536 */
#define QO_KMAX 4096
#define QO_NMAX 65536

/* ---- GF(65537) scalar arithmetic: src/gf_ring.h:214-286 ---- */
uint32_t qo_add(uint32_t a, uint32_t b);
uint32_t qo_sub(uint32_t a, uint32_t b);
uint32_t qo_mul(uint32_t a, uint32_t b);
uint32_t qo_exp(uint32_t a, uint32_t e);
uint32_t qo_inv(uint32_t a);
/* src/gf_ring.h:774-781 (root 3 found by src/gf_ring.h:624-660) */
uint32_t qo_nth_root(uint32_t n);
/* src/gf_ring.h:814-822 -> src/arith.h:692-712 */
uint32_t qo_code_len(uint32_t n);

/* Codec parameters: src/fec_rs_fnt.h:69-163, src/fec_base.h:248-271,319-335 */
typedef struct {
    int sys;          /* 1 = SYSTEMATIC */
    int k, m;         /* n_data, n_parities */
    int code_len;     /* k + m */
    int n_outputs;    /* m (sys) or code_len (non-sys)  src/fec_base.h:328-329 */
    int n;            /* FFT length = ceil2(k+m)        src/fec_rs_fnt.h:106 */
    int data_len;     /* ceil2(k): Radix2 data_len      src/fec_rs_fnt.h:111-113 */
    int len_2k;       /* ceil2(2k)                      src/fec_rs_fnt.h:119 */
    uint32_t r;       /* n-th root of unity             src/fec_rs_fnt.h:109 */
} qo_codec;

int qo_codec_init(qo_codec* c, int k, int m, int sys);

/* Radix-2 transforms on one column (src/fft_2n.h:269-352). */
void qo_fft(int n, int data_len, uint32_t w, const uint32_t* in, int in_len,
            uint32_t* out);
void qo_fft_inv(int n, uint32_t w, const uint32_t* in, uint32_t* out);

/* Decode context for a set of k fragment ids (src/fec_context.h:66-274). */
typedef struct {
    int k;
    uint32_t ids[QO_KMAX];
    uint32_t inv_A_i[QO_KMAX];
    uint32_t A_fft_2k[2 * QO_KMAX];
} qo_ctx;

int qo_ctx_init(const qo_codec* c, qo_ctx* ctx, const uint32_t* ids);

/* One column: words[k] (OOR already restored) -> data[k].
 * src/fec_base.h:1336-1355, :1418-1448, src/fec_rs_fnt.h:204-234 */
void qo_decode_column(const qo_codec* c, const qo_ctx* ctx,
                      const uint32_t* words, uint32_t* data);

/* One column encode: data[k] -> out[n] full codeword values (0..65536).
 * src/fec_rs_fnt.h:236-251 (both types; SYS rows 0..k-1 hold the data). */
void qo_encode_column(const qo_codec* c, const qo_ctx* enc_ctx,
                      const uint32_t* data, uint32_t* codeword);

/* ---- Block API (src/fec_base.h:1066-1321) ----
 * data: k pointers to block_bytes each. outputs: n_outputs pointers (NULL =
 * not wanted).  OOR lists: per output, ascending absolute word offsets,
 * capacity oor_cap each (counts may exceed cap: then entries are truncated,
 * count is still exact). */
void qo_encode_blocks(const qo_codec* c, uint8_t* const* data,
                      uint8_t* const* outputs, size_t block_bytes,
                      uint32_t* oor, uint32_t* oor_count, uint32_t oor_cap);

/* data: k pointers (written where wanted[i]); parities: n_outputs pointers;
 * missing: code_len flags (nonzero = missing, src/fec_base.h:1203,1221);
 * oor/oor_count: per n_outputs list as produced by encode.
 * Returns 1 on success, 0 if fewer than k fragments. */
int qo_decode_blocks(const qo_codec* c, uint8_t* const* data,
                     uint8_t* const* parities, const uint32_t* oor,
                     const uint32_t* oor_count, uint32_t oor_cap,
                     const int* missing, const int* wanted,
                     size_t block_bytes);

/* ---- RS-NF4 block API (src/fec_rs_nf4.h:46-334, src/gf_nf4.h) ----
 * word_size in {2, 4, 8}: word j of a fragment packs word_size/2 GF(65537)
 * components (the 16-bit lanes j*g .. j*g+g-1 of the byte stream), each
 * coded like an RS-FNT column.  c: a NON-systematic codec (qo_codec_init
 * with sys = 0).  OOR marks per output: ascending word offsets in `oor`,
 * component bitmasks in `flags` (cap entries each, counts exact).  Only
 * whole words (block_bytes / word_size) are processed. */
void qo_nf4_encode_blocks(const qo_codec* c, int word_size,
                          uint8_t* const* data, uint8_t* const* outputs,
                          size_t block_bytes, uint32_t* oor, uint32_t* flags,
                          uint32_t* oor_count, uint32_t oor_cap);
/* missing: code_len flags (nonzero = missing).  1 decoded, 0 < k present. */
int qo_nf4_decode_blocks(const qo_codec* c, int word_size,
                         uint8_t* const* data, uint8_t* const* parities,
                         const uint32_t* oor, const uint32_t* flags,
                         const uint32_t* oor_count, uint32_t oor_cap,
                         const int* missing, const int* wanted,
                         size_t block_bytes);

/* ---- C-ABI semantics (src/quadiron_c.cpp:37-406) ---- */
int qo_metadata_size(size_t block_size);
int qo_fnt32_encode(const qo_codec* c, uint8_t** data, uint8_t** parity,
                    const int* wanted_idxs, size_t block_size);
int qo_fnt32_decode(const qo_codec* c, uint8_t** data, uint8_t** parity,
                    const int* missing_idxs, size_t block_size);
int qo_fnt32_reconstruct(const qo_codec* c, uint8_t** data, uint8_t** parity,
                         const int* missing_idxs, unsigned destination_idx,
                         size_t block_size);

#ifdef __cplusplus
}
#endif

#endif
