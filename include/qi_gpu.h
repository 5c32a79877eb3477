/*
 * qi_gpu.h -- device-level C-ABI of the MI355X RS-FNT engine.
 *
 * This is the "thin C-ABI shim" below the drop-in quadiron_c.h boundary: plain
 * pointers and sizes, no C++ or torch types.  Device pointers are HIP device
 * memory; `stream` is a hipStream_t passed as void* (NULL = default stream).
 * All calls are asynchronous on `stream` unless stated.  Errors are negative
 * ints.
 *
 * Semantics follow QuadIron's RsFnt<uint32_t> with word_size 2
 * (src/fec_rs_fnt.h:51-270): GF(65537), n = ceil2(k+m), root r = 3^(65536/n).
 *   - NON-SYSTEMATIC encode: outputs 0..k+m-1 = evaluations of the data
 *     polynomial at r^i (the zero-padded n-point NTT, src/fft_2n.h:360-407).
 *   - SYSTEMATIC encode: outputs = the m parities (codeword rows k..k+m-1).
 *   - An output symbol equal to 65536 is stored as 0 and recorded as an
 *     out-of-range (OOR) mark (src/fec_rs_fnt.h:253-269).
 *
 * Device layout: a *stripe* is a set of fragment rows of `words` u16 symbols.
 * Row t of stripe s lives at base + s*stripe_stride + t*row_stride (strides in
 * u16 elements).  One call processes n_stripes stripes; every column of every
 * stripe is an independent codeword.
 *
 * OOR marks are kept in *buckets*: counts[s*slots + slot] (u32) and
 * entries[(s*slots + slot)*cap + e] (u32 word offset within the row).  Encode
 * zeroes nothing: callers clear counts (qi_gpu_oor_clear) before encoding.
 * Entries inside a bucket are unordered; encode keeps counting past cap (the
 * caller detects the overflow from the count and re-runs with a larger
 * cap); a decode reading such a bucket raises qi_gpu_take_error.
 */
#ifndef QI_GPU_H
#define QI_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct qi_plan qi_plan;

/* Number of visible HIP devices (0 when none). */
int qi_gpu_device_count(void);

/* Create an RS-FNT plan (word_size 2 only).  Returns NULL on bad
 * parameters (k < 1, m < 1, k+m > 65536) or when no device is present.
 * Kernels by k:
 *   - k <= 256: the register codelets (non-systematic encode, k <= 32) and
 *     the matrix cores (every decode; the systematic encode; the
 *     non-systematic encode for 32 < k <= 256), dot2 kernels for column
 *     tails;
 *   - 256 < k <= 384: the matrix cores for batches whose width is a
 *     multiple of 1024 columns and whose rows are 8-byte aligned inside
 *     31-bit buffer ranges (the encode only while the generator stays small:
 *     k * n_outputs <= 2^21, 2^18 systematic); the NTT engine otherwise;
 *   - 384 < k <= 640, n - k > 64: the decode as above on the matrix cores
 *     (k x k contexts, two K chunks), and the systematic encode while its
 *     generator stays small (k * m <= 2^20); the non-systematic encode, and
 *     every other batch, on the NTT engine;
 *   - k > 384 otherwise: the NTT engine (column-batched NTT passes in LDS or
 *     HBM; the erasure decode when n - k <= 64). */
qi_plan* qi_plan_create(int k, int m, int systematic);
/* The same with flags: QI_PLAN_ENC_MATRIX / QI_PLAN_ENC_CODELETS force the
 * matrix-core or the register-codelet non-systematic encode for k <= 64
 * (both bit-exact; the default picks the faster: codelets up to k = 32).
 * NULL on unknown or contradictory flags. */
#define QI_PLAN_ENC_MATRIX 1
#define QI_PLAN_ENC_CODELETS 2
qi_plan* qi_plan_create_ex(int k, int m, int systematic, int flags);
void qi_plan_destroy(qi_plan* plan);
/* n (FFT length) and n_outputs (m if systematic, k+m otherwise) */
int qi_plan_n(const qi_plan* plan);
int qi_plan_n_outputs(const qi_plan* plan);

/* Zero n u32 OOR counters. */
int qi_gpu_oor_clear(uint32_t* d_counts, size_t n, void* stream);

/* Batch encode (device resident).  data: k rows per stripe.  out: n_outputs
 * rows per stripe.  OOR buckets: slots = n_outputs, slot = output index.
 * Pass d_oor_counts = NULL to skip OOR recording. */
int qi_gpu_encode(qi_plan* plan, const uint16_t* d_data,
                  long long data_stripe_stride, long long data_row_stride,
                  uint16_t* d_out, long long out_stripe_stride,
                  long long out_row_stride, long long words, int n_stripes,
                  uint32_t* d_oor_counts, uint32_t* d_oor_entries, int oor_cap,
                  void* stream);

/* Bytes of device workspace for n_stripes decode contexts of `words`
 * columns each -- enough for any width up to `words`.  A context is valid
 * only for the `words` it was built with (its format and per-stripe stride
 * follow the width: for 256 < k <= 384 (and the non-systematic 384 < k <=
 * 640 codes with n - k > 64), matrix contexts at multiples of 1024 columns,
 * the NTT engine's otherwise). */
size_t qi_gpu_decode_ctx_bytes(const qi_plan* plan, int n_stripes,
                               long long words);

/* Build per-stripe decode contexts from the received fragment ids:
 * d_ids[s*k + i] (u16, distinct, < k+m; ascending as the reference passes
 * them, any order accepted) -- the k fragments the decoder uses
 * (FecCode::decode_blocks_vertical picks the first k present,
 * src/fec_base.h:1199-1236; a systematic context lists them data fragments
 * first, so that the matrix kernel reads each of its two source regions in
 * one run) -- and route the OOR marks of those fragments
 * (buckets as produced by qi_gpu_encode) into per-tile tables.  With NULL
 * counts the context is built from the ids alone (init_context_dec,
 * src/fec_base.h:758-793: before the fragments' data and marks exist, e.g.
 * on another stream while they are produced); a decode given buckets then
 * reads the marks from them directly (slightly slower per tile than routed
 * tables).  Built on the device, asynchronously on `stream`, for every k:
 * matrix contexts (the interpolation matrix, up to ~780 KB per stripe at
 * k = 256) for k <= 256, and for 256 < k <= 640 at widths that are a
 * multiple of 1024 columns (then followed by the NTT engine's context, used
 * when the decode's rows are not addressable by the matrix cores); the NTT
 * decode's per-pattern constants (src/fec_context.h:232-274, whose decode
 * reads the OOR buckets directly) otherwise; for 256 < k <= 640 the NTT
 * engine's half is built by the first decode that needs it.  h_ids is
 * unused (kept for ABI stability; may be NULL). */
int qi_gpu_decode_ctx(qi_plan* plan, const uint16_t* d_ids,
                      const uint16_t* h_ids, int n_stripes,
                      const uint32_t* d_oor_counts,
                      const uint32_t* d_oor_entries, int oor_cap,
                      long long words, void* d_ctx, void* stream);

/* Batch decode.  Received fragment id f of stripe s is read from
 *   f <  k (systematic data rows):  d_data + s*dss + f*drs
 *   otherwise (coded row / parity): d_coded + s*css + slot*crs
 * with slot = f - k (systematic) or f (non-systematic).
 * OOR buckets of the coded rows are indexed by the same slot (slots =
 * n_outputs); pass NULL counts when there are none.  Output: k data rows.
 * The context is not const in effect: a decode whose rows the matrix cores
 * cannot address fills the context's lazily built sections (the dot2
 * kernel's packed rows for k <= 256, the NTT engine's half for 256 < k <=
 * 640) the first time, on `stream`, and records that in the context.  Every
 * word such a fill writes gets the value it already holds when the section
 * was filled before, so a context may serve any number of decodes, on one
 * stream or on several at once (two decodes may then both fill it), once
 * the qi_gpu_decode_ctx call that built it is ordered before them. */
int qi_gpu_decode(qi_plan* plan, const void* d_ctx, const uint16_t* d_ids,
                  const uint16_t* d_data, long long dss, long long drs,
                  const uint16_t* d_coded, long long css, long long crs,
                  const uint32_t* d_oor_counts, const uint32_t* d_oor_entries,
                  int oor_cap, uint16_t* d_out, long long out_stripe_stride,
                  long long out_row_stride, long long words, int n_stripes,
                  void* stream);

/* Packed-row decode (the staging layout of a host pipeline, where the k
 * received fragments of a stripe are copied back to back): row i of stripe s
 * is read from d_recv + s*rss + i*rrs and holds fragment d_ids[s*k + i].  The
 * OOR buckets are indexed by that position i (slots = k).  Contexts for this
 * layout come from qi_gpu_decode_ctx_packed (same size as
 * qi_gpu_decode_ctx_bytes). */
int qi_gpu_decode_ctx_packed(qi_plan* plan, const uint16_t* d_ids,
                             const uint16_t* h_ids, int n_stripes,
                             const uint32_t* d_oor_counts,
                             const uint32_t* d_oor_entries, int oor_cap,
                             long long words, void* d_ctx, void* stream);
int qi_gpu_decode_packed(qi_plan* plan, const void* d_ctx,
                         const uint16_t* d_recv, long long rss, long long rrs,
                         const uint32_t* d_oor_counts,
                         const uint32_t* d_oor_entries, int oor_cap,
                         uint16_t* d_out, long long out_stripe_stride,
                         long long out_row_stride, long long words,
                         int n_stripes, void* stream);

/* Non-zero if an OOR bucket read by a decode context or a decode held more
 * marks than its capacity (oor_cap), i.e. some out-of-range symbols could
 * not be restored and the affected stripes are wrong (bit 1), or if a decode
 * context was built from ids that were not distinct or not below n (bit 2;
 * every context builder checks: a repeated id makes A'(x_i) = 0, and the
 * erasure decode of k > 384, n - k <= 64, derives its erased set from the
 * ids).  Sticky per plan; reset by
 * reading.  Synchronous.  Tiles with many marks need no capacity of their
 * own: they are decoded by a slower path, never refused. */
int qi_gpu_take_error(qi_plan* plan);

/* Names of the kernels an encode and a decode of `words` columns launch on
 * this plan (rows at 8-byte aligned offsets), as
 * "encode=<kernels>; decode=<kernels>" -- diagnostics for bench lines and
 * profiles.  The string is per calling thread, valid until its next call. */
const char* qi_gpu_kernels(const qi_plan* plan, long long words);

/* Build identification: "<git describe>+src:<hash of the library sources>". */
const char* qi_build_id(void);


/* ---- Block API over host buffers (C view of qi::fec::RsFnt, see
 * include/qi_fec.hpp; semantics of FecCode::encode_blocks_vertical /
 * decode_blocks_vertical, src/fec_base.h:1066-1321).  OOR marks are returned
 * as per-output ascending offset lists of capacity oor_cap (counts exact). */
typedef struct qi_fec qi_fec;
qi_fec* qi_fec_new(int systematic, int k, int m);
void qi_fec_delete(qi_fec* f);
int qi_fec_n_outputs(const qi_fec* f);
/* outputs: n_outputs pointers (NULL = not wanted). 0 or -1 */
int qi_fec_encode_blocks(qi_fec* f, uint8_t** data, uint8_t** outputs,
                         size_t block_bytes, uint32_t* oor, uint32_t* oor_count,
                         uint32_t oor_cap);
/* returns 1 decoded, 0 fewer than k fragments, -1 error */
int qi_fec_decode_blocks(qi_fec* f, uint8_t** data, uint8_t** parities,
                         const uint32_t* oor, const uint32_t* oor_count,
                         uint32_t oor_cap, const int* missing,
                         const int* wanted, size_t block_bytes);

/* Stream API (encode_streams_vertical / decode_streams_vertical,
 * src/fec_base.h:463-542, 898-1048) over caller memory: each fragment is a
 * stream of `bytes` bytes.  The streams go through the two-slot pinned
 * pipeline of qi::fec::RsFnt (chunks of whole packets, host reads/writes
 * overlapping the transfers and kernels).  Encode: all outputs required;
 * 0 or -1.  Decode: data[i] / parities[i] NULL = missing (data may be NULL
 * as a whole for non-systematic codes), out_data[i] NULL = not wanted;
 * 1 decoded, 0 fewer than k fragments, -1 error. */
int qi_fec_encode_streams(qi_fec* f, const uint8_t** data, size_t bytes,
                          uint8_t** outputs, uint32_t* oor, uint32_t* oor_count,
                          uint32_t oor_cap);
int qi_fec_decode_streams(qi_fec* f, const uint8_t** data,
                          const uint8_t** parities, size_t bytes,
                          const uint32_t* oor, const uint32_t* oor_count,
                          uint32_t oor_cap, uint8_t** out_data);

/* ---- RS-NF4 block API (C view of qi::fec::RsNf4; RsNf4<T>,
 * src/fec_rs_nf4.h:46-334).  word_size 2, 4 or 8 (NULL otherwise): every
 * word packs word_size/2 GF(65537) components, each coded like an RS-FNT
 * column on the device.  Non-systematic: n_outputs = k + m.  OOR marks per
 * output: ascending word offsets in `oor` with the component bitmask in
 * `flags` (oor_cap entries each, counts exact).  Whole words only. */
typedef struct qi_nf4 qi_nf4;
qi_nf4* qi_nf4_new(int word_size, int k, int m);
void qi_nf4_delete(qi_nf4* f);
int qi_nf4_n_outputs(const qi_nf4* f);
/* 0 or -1 */
int qi_nf4_encode_blocks(qi_nf4* f, uint8_t** data, uint8_t** outputs,
                         size_t block_bytes, uint32_t* oor, uint32_t* flags,
                         uint32_t* oor_count, uint32_t oor_cap);
/* missing: k + m flags.  1 decoded, 0 fewer than k fragments, -1 error */
int qi_nf4_decode_blocks(qi_nf4* f, uint8_t** data, uint8_t** parities,
                         const uint32_t* oor, const uint32_t* flags,
                         const uint32_t* oor_count, uint32_t oor_cap,
                         const int* missing, const int* wanted,
                         size_t block_bytes);

#ifdef __cplusplus
}
#endif

#endif
