// Drop-in C-ABI (include/quadiron_c.h) over the GPU RsFnt block API.
// Glue semantics follow src/quadiron_c.cpp:37-411; every C++ exception is
// caught at the boundary (-1 / NULL), never propagated into C callers.
#include <cctype>
#include <cstdio>
#include <exception>
#include <vector>

#include "../../include/qi_fec.hpp"
#include "../../include/quadiron_c.h"

using qi::Properties;
using qi::fec::FecType;
using qi::fec::RsFnt;

namespace {

RsFnt* as_fec(QuadironFnt32* p)
{
    return reinterpret_cast<RsFnt*>(p);
}

int md_size(size_t block_size)
{
    return static_cast<int>(((block_size / 65536) + 16) * 4);
}

uint32_t* hdr(uint8_t* p)
{
    return reinterpret_cast<uint32_t*>(p);
}

// deserialize the FNT1 headers of every present coded fragment and point the
// coded-fragment vector at the payloads (src/quadiron_c.cpp:160-206,246-285)
int load_props(RsFnt* fec, uint8_t** data, uint8_t** parity, const int* missing,
               int md, std::vector<uint8_t*>& par_vec,
               std::vector<Properties>& props, bool all_ptrs)
{
    const unsigned k = fec->n_data, m = fec->n_parities;
    if (fec->type == FecType::SYSTEMATIC) {
        for (unsigned i = 0; i < m; i++) {
            if (!missing[k + i] &&
                props[i].fnt_deserialize(hdr(parity[i]), md / 4) == -1)
                return -1;
            if (!missing[k + i] || all_ptrs)
                par_vec[i] = parity[i] ? parity[i] + md : nullptr;
        }
    } else {
        for (unsigned i = 0; i < k; i++) {
            if (!missing[i] && props[i].fnt_deserialize(hdr(data[i]), md / 4) == -1)
                return -1;
            if (!missing[i] || all_ptrs)
                par_vec[i] = data[i] ? data[i] + md : nullptr;
        }
        for (unsigned i = 0; i < m; i++) {
            if (!missing[k + i] &&
                props[k + i].fnt_deserialize(hdr(parity[i]), md / 4) == -1)
                return -1;
            if (!missing[k + i] || all_ptrs)
                par_vec[k + i] = parity[i] ? parity[i] + md : nullptr;
        }
    }
    return 0;
}

}  // namespace

extern "C" {

struct QuadironFnt32*
quadiron_fnt32_new(int word_size, int n_data, int n_parities, int systematic)
{
    if (word_size != 2)
        return nullptr;  // quirk Q6: GF(257) path not provided
    try {
        return reinterpret_cast<QuadironFnt32*>(new RsFnt(
            systematic ? FecType::SYSTEMATIC : FecType::NON_SYSTEMATIC,
            static_cast<unsigned>(word_size), static_cast<unsigned>(n_data),
            static_cast<unsigned>(n_parities), 1024));
    } catch (...) {
        return nullptr;
    }
}

void quadiron_fnt32_delete(struct QuadironFnt32* fecp)
{
    delete as_fec(fecp);
}

int quadiron_fnt32_get_metadata_size(struct QuadironFnt32* /*fecp*/,
                                     size_t block_size)
{
    return md_size(block_size);
}

int quadiron_fnt32_encode(struct QuadironFnt32* fecp, uint8_t** data,
                          uint8_t** parity, int* wanted_idxs, size_t block_size)
{
    try {
        RsFnt* fec = as_fec(fecp);
        const unsigned k = fec->n_data, m = fec->n_parities, no = fec->n_outputs;
        std::vector<uint8_t*> data_vec(k), par_vec(no);
        std::vector<Properties> props(no);
        std::vector<bool> wanted(no);
        const int md = md_size(block_size);
        for (unsigned i = 0; i < no; i++)
            wanted[i] = wanted_idxs[i] != 0;
        const bool sys = fec->type == FecType::SYSTEMATIC;
        for (unsigned i = 0; i < k; i++) {
            data_vec[i] = data[i] + md;
            if (!sys)
                par_vec[i] = data[i] + md;
        }
        for (unsigned i = 0; i < m; i++)
            par_vec[sys ? i : k + i] = parity[i] ? parity[i] + md : nullptr;
        fec->encode_blocks_vertical(data_vec, par_vec, props, wanted, block_size);
        Properties null_prop;
        for (unsigned i = 0; i < k; i++)
            if ((sys ? null_prop : props[i]).fnt_serialize(hdr(data[i]), md / 4) ==
                -1)
                return -1;
        for (unsigned i = 0; i < m; i++)
            if (parity[i] &&
                props[sys ? i : k + i].fnt_serialize(hdr(parity[i]), md / 4) == -1)
                return -1;
        return 0;
    } catch (...) {
        return -1;
    }
}

int quadiron_fnt32_decode(struct QuadironFnt32* fecp, uint8_t** data,
                          uint8_t** parity, int* missing_idxs, size_t block_size)
{
    try {
        RsFnt* fec = as_fec(fecp);
        const unsigned k = fec->n_data, m = fec->n_parities, no = fec->n_outputs;
        std::vector<uint8_t*> data_vec(k), par_vec(no, nullptr);
        std::vector<Properties> props(no);
        std::vector<int> miss(missing_idxs, missing_idxs + k + m);
        std::vector<bool> wanted(k, true);
        const int md = md_size(block_size);
        if (load_props(fec, data, parity, missing_idxs, md, par_vec, props, false))
            return -1;
        for (unsigned i = 0; i < k; i++)
            data_vec[i] = data[i] + md;
        if (!fec->decode_blocks_vertical(data_vec, par_vec, props, miss, wanted,
                                         block_size))
            return -1;
        // reset metadata of data (src/quadiron_c.cpp:218-226; the reference
        // indexes parities_props[i] for i < n_data, past its end when
        // systematic with m < k -- an empty header is what it writes)
        Properties empty;
        for (unsigned i = 0; i < k; i++)
            if (empty.fnt_serialize(hdr(data[i]), md / 4) == -1)
                return -1;
        return 0;
    } catch (...) {
        return -1;
    }
}

int quadiron_fnt32_reconstruct(struct QuadironFnt32* fecp, uint8_t** data,
                               uint8_t** parity, int* missing_idxs,
                               unsigned int dest, size_t block_size)
{
    try {
        RsFnt* fec = as_fec(fecp);
        const unsigned k = fec->n_data, m = fec->n_parities, no = fec->n_outputs;
        const bool sys = fec->type == FecType::SYSTEMATIC;
        std::vector<uint8_t*> data_vec(k), par_vec(no, nullptr);
        std::vector<Properties> props(no);
        std::vector<int> miss(missing_idxs, missing_idxs + k + m);
        const int md = md_size(block_size);
        if (load_props(fec, data, parity, missing_idxs, md, par_vec, props, true))
            return -1;
        for (unsigned i = 0; i < k; i++)
            data_vec[i] = data[i] ? data[i] + md : nullptr;
        if (sys && dest < k) {
            // src/quadiron_c.cpp:289-320
            std::vector<bool> w(k, false);
            w[dest] = true;
            if (!fec->decode_blocks_vertical(data_vec, par_vec, props, miss, w,
                                             block_size))
                return -1;
            Properties null_prop;
            return null_prop.fnt_serialize(hdr(data[dest]), md / 4) == -1 ? -1 : 0;
        }
        // src/quadiron_c.cpp:326-406: decode the data then re-encode the
        // wanted output
        std::vector<std::vector<uint8_t>> blocks(k);
        std::vector<bool> wanted_data(k, false);
        bool need = false;
        for (unsigned i = 0; i < k; i++) {
            if (!sys || missing_idxs[i]) {
                need = true;
                wanted_data[i] = true;
                blocks[i].resize(block_size + 2);
                data_vec[i] = blocks[i].data();
            }
        }
        if (need && !fec->decode_blocks_vertical(data_vec, par_vec, props, miss,
                                                 wanted_data, block_size))
            return -1;
        const unsigned w = sys ? dest - k : dest;
        if (w >= no)
            return -1;
        std::vector<bool> wanted(no, false);
        wanted[w] = true;
        uint8_t* target = sys ? parity[w] : (w < k ? data[w] : parity[w - k]);
        std::vector<uint8_t*> outs(no, nullptr);
        outs[w] = target + md;
        fec->encode_blocks_vertical(data_vec, outs, props, wanted, block_size);
        return props[w].fnt_serialize(hdr(target), md / 4) == -1 ? -1 : 0;
    } catch (...) {
        return -1;
    }
}

// quadiron::hex_dump (src/misc.cpp:83-130) to stderr with printable chars
void quadiron_hex_dump(uint8_t* buf, size_t size)
{
    if (!buf)
        return;
    const size_t maxline = 32;
    char render[maxline + 1];
    size_t rn = 0;
    size_t linecount = maxline;
    for (; size; --size, ++buf) {
        std::fprintf(stderr, "%02x ", static_cast<unsigned>(*buf));
        render[rn++] = std::isprint(*buf) ? static_cast<char>(*buf) : '.';
        if (--linecount == 0) {
            render[rn] = '\0';
            std::fprintf(stderr, " | %s\n", render);
            rn = 0;
            // min(maxline, bufsize) before the loop decrement, as in
            // src/misc.cpp:108-112
            linecount = size < maxline ? size : maxline;
        }
    }
    if (rn) {
        render[rn] = '\0';
        for (size_t i = rn; i < maxline; i++)
            std::fprintf(stderr, "   ");
        std::fprintf(stderr, " | %s\n", render);
    }
}

}  // extern "C"
