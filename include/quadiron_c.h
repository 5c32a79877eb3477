/*
 * quadiron_c.h -- drop-in C-ABI of the MI355X RS-FNT engine.
 *
 * Same entry points, argument meaning and error behaviour as QuadIron's
 * src/quadiron_c.h:34-160 (each prototype below cites the reference
 * declaration it replaces).  Link against quadiron_amd/libquadiron_amd.so.
 *
 * Deviation (documented in DESIGN.md, quirk Q6): only word_size 2
 * (GF(65537)) is accepted; quadiron_fnt32_new(1, ...) returns NULL.  The
 * reference's word_size-1 path returns wrong data (AVX2 build) or -1 (scalar
 * build).
 */
#ifndef __QUAD_QUADIRON_C_H__
#define __QUAD_QUADIRON_C_H__

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src/quadiron_c.h:49-50 (impl. src/quadiron_c.cpp:37-54) */
struct QuadironFnt32*
quadiron_fnt32_new(int word_size, int n_data, int n_parities, int systematic);

/* src/quadiron_c.h:56 (src/quadiron_c.cpp:56-59) */
void quadiron_fnt32_delete(struct QuadironFnt32* fecp);

/* src/quadiron_c.h:69-71 (src/quadiron_c.cpp:61-71):
 * ((block_size / 65536) + 16) * 4 */
int quadiron_fnt32_get_metadata_size(
    struct QuadironFnt32* fecp,
    size_t block_size);

/* src/quadiron_c.h:90-95 (src/quadiron_c.cpp:73-150) */
int quadiron_fnt32_encode(
    struct QuadironFnt32* fecp,
    uint8_t** data,
    uint8_t** parity,
    int* wanted_idxs,
    size_t block_size);

/* src/quadiron_c.h:119-124 (src/quadiron_c.cpp:152-229) */
int quadiron_fnt32_decode(
    struct QuadironFnt32* fecp,
    uint8_t** data,
    uint8_t** parity,
    int* missing_idxs,
    size_t block_size);

/* src/quadiron_c.h:145-151 (src/quadiron_c.cpp:231-406) */
int quadiron_fnt32_reconstruct(
    struct QuadironFnt32* fecp,
    uint8_t** data,
    uint8_t** parity,
    int* missing_idxs,
    unsigned int destination_idx,
    size_t block_size);

/* src/quadiron_c.h:158 (src/quadiron_c.cpp:408-411) */
void quadiron_hex_dump(uint8_t* buf, size_t size);

#ifdef __cplusplus
}
#endif

#endif
