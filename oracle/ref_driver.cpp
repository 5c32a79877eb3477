/*
 * ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * A thin extern "C" driver over the *reference* QuadIron library, compiled
 * from the reference sources where they lie (/root/reference/src, see
 * oracle/Makefile) into oracle/_ref/libqiref.so.  It is used to
 *   - generate the golden vectors in tests/golden/ (tests/golden/gen_golden.py)
 *   - time the reference AVX2 CPU path as bench.py's cpu_baseline leg.
 *
 * quadiron_c.cpp itself cannot be built here (it includes the CMake-generated
 * build_info.h), so the ref_c_* functions below re-do its small amount of
 * glue (src/quadiron_c.cpp:73-406) on top of the reference's own
 * FecCode::encode_blocks_vertical / decode_blocks_vertical and
 * Properties::fnt_serialize / fnt_deserialize.
 */
#include <chrono>
#include <memory>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "fec_rs_fnt.h"
#include "fec_rs_nf4.h"
#include "property.h"

using quadiron::Properties;
using quadiron::fec::FecType;
using quadiron::fec::RsFnt;

namespace {

RsFnt<uint32_t>* make(int sys, int k, int m, size_t pkt)
{
    return new RsFnt<uint32_t>(
        sys ? FecType::SYSTEMATIC : FecType::NON_SYSTEMATIC, 2, k, m, pkt);
}

void props_out(const Properties& p, uint32_t* list, uint32_t* count,
               uint32_t cap)
{
    uint32_t c = 0;
    for (auto const& it : p.get_map()) {
        if (c < cap)
            list[c] = static_cast<uint32_t>(it.first);
        c++;
    }
    *count = c;
}

int md_size(size_t block_size)
{
    return static_cast<int>(((block_size / 65536) + 16) * 4);
}

template <typename T>
void nf4_encode(int ws, int k, int m, size_t pkt, uint8_t** data,
                uint8_t** outputs, size_t block_bytes, uint32_t* oor,
                uint32_t* flags, uint32_t* oor_count, uint32_t cap)
{
    quadiron::fec::RsNf4<T> f(ws, k, m, pkt);
    unsigned no = f.n_outputs;
    std::vector<uint8_t*> dv(data, data + k);
    std::vector<uint8_t*> pv(no);
    std::vector<Properties> props(no);
    std::vector<bool> wanted(no);
    std::vector<std::vector<uint8_t>> scratch(no);
    for (unsigned i = 0; i < no; i++) {
        wanted[i] = outputs[i] != nullptr;
        if (!outputs[i]) {
            scratch[i].resize(block_bytes + 16);
            pv[i] = scratch[i].data();
        } else {
            pv[i] = outputs[i];
        }
    }
    f.encode_blocks_vertical(dv, pv, props, wanted, block_bytes);
    for (unsigned i = 0; i < no; i++) {
        uint32_t c = 0;
        for (auto const& it : props[i].get_map()) {
            if (c < cap) {
                oor[static_cast<size_t>(i) * cap + c] =
                    static_cast<uint32_t>(it.first);
                flags[static_cast<size_t>(i) * cap + c] = it.second;
            }
            c++;
        }
        oor_count[i] = c;
    }
}

template <typename T>
int nf4_decode(int ws, int k, int m, size_t pkt, uint8_t** data,
               uint8_t** parities, const uint32_t* oor, const uint32_t* flags,
               const uint32_t* oor_count, uint32_t cap, const int* missing,
               const int* wanted, size_t block_bytes)
{
    quadiron::fec::RsNf4<T> f(ws, k, m, pkt);
    unsigned no = f.n_outputs;
    std::vector<uint8_t*> dv(data, data + k);
    std::vector<uint8_t*> pv(parities, parities + no);
    std::vector<Properties> props(no);
    std::vector<int> miss(missing, missing + no);
    std::vector<bool> want(k);
    for (int i = 0; i < k; i++)
        want[i] = wanted[i] != 0;
    for (unsigned i = 0; i < no; i++) {
        uint32_t c = oor_count[i] < cap ? oor_count[i] : cap;
        for (uint32_t e = 0; e < c; e++)
            props[i].add(oor[static_cast<size_t>(i) * cap + e],
                         flags[static_cast<size_t>(i) * cap + e]);
    }
    return f.decode_blocks_vertical(dv, pv, props, miss, want, block_bytes) ? 1
                                                                            : 0;
}

} // namespace

extern "C" {

int ref_n(int k, int m)
{
    std::unique_ptr<RsFnt<uint32_t>> f(make(0, k, m, 8));
    return static_cast<int>(f->get_n_outputs());
}

/* FecCode::encode_blocks_vertical, src/fec_base.h:1066-1151 */
void ref_encode_blocks(int sys, int k, int m, size_t pkt, uint8_t** data,
                       uint8_t** outputs, size_t block_bytes, uint32_t* oor,
                       uint32_t* oor_count, uint32_t cap)
{
    std::unique_ptr<RsFnt<uint32_t>> f(make(sys, k, m, pkt));
    unsigned no = f->n_outputs;
    std::vector<uint8_t*> dv(data, data + k);
    std::vector<uint8_t*> pv(no);
    std::vector<Properties> props(no);
    std::vector<bool> wanted(no);
    std::vector<std::vector<uint8_t>> scratch(no);
    for (unsigned i = 0; i < no; i++) {
        wanted[i] = outputs[i] != nullptr;
        if (!outputs[i]) {
            scratch[i].resize(block_bytes + 1);
            pv[i] = scratch[i].data();
        } else {
            pv[i] = outputs[i];
        }
    }
    f->encode_blocks_vertical(dv, pv, props, wanted, block_bytes);
    for (unsigned i = 0; i < no; i++)
        props_out(props[i], oor + static_cast<size_t>(i) * cap, &oor_count[i],
                  cap);
}

/* FecCode::decode_blocks_vertical, src/fec_base.h:1177-1321 */
int ref_decode_blocks(int sys, int k, int m, size_t pkt, uint8_t** data,
                      uint8_t** parities, const uint32_t* oor,
                      const uint32_t* oor_count, uint32_t cap,
                      const int* missing, const int* wanted,
                      size_t block_bytes)
{
    std::unique_ptr<RsFnt<uint32_t>> f(make(sys, k, m, pkt));
    unsigned no = f->n_outputs;
    std::vector<uint8_t*> dv(data, data + k);
    std::vector<uint8_t*> pv(parities, parities + no);
    std::vector<Properties> props(no);
    std::vector<int> miss(missing, missing + k + m);
    std::vector<bool> want(k);
    for (int i = 0; i < k; i++)
        want[i] = wanted[i] != 0;
    for (unsigned i = 0; i < no; i++) {
        uint32_t c = oor_count[i] < cap ? oor_count[i] : cap;
        for (uint32_t e = 0; e < c; e++)
            props[i].add(oor[static_cast<size_t>(i) * cap + e],
                         quadiron::OOR_MARK);
    }
    return f->decode_blocks_vertical(dv, pv, props, miss, want, block_bytes)
               ? 1
               : 0;
}

int ref_metadata_size(size_t block_size)
{
    return md_size(block_size);
}

/* quadiron_fnt32_encode glue: src/quadiron_c.cpp:73-150 (pkt_size 1024) */
int ref_c_encode(int sys, int k, int m, uint8_t** data, uint8_t** parity,
                 const int* wanted_idxs, size_t block_size)
{
    std::unique_ptr<RsFnt<uint32_t>> fec(make(sys, k, m, 1024));
    unsigned no = fec->n_outputs;
    std::vector<uint8_t*> data_vec(k), par_vec(no);
    std::vector<Properties> props(no);
    std::vector<bool> wanted(no);
    int md = md_size(block_size);
    for (unsigned i = 0; i < no; i++)
        wanted[i] = wanted_idxs[i] != 0;
    if (sys) {
        for (int i = 0; i < k; i++)
            data_vec[i] = data[i] + md;
        for (int i = 0; i < m; i++)
            par_vec[i] = parity[i] + md;
    } else {
        for (int i = 0; i < k; i++) {
            data_vec[i] = data[i] + md;
            par_vec[i] = data[i] + md;
        }
        for (int i = 0; i < m; i++)
            par_vec[k + i] = parity[i] + md;
    }
    fec->encode_blocks_vertical(data_vec, par_vec, props, wanted, block_size);
    if (sys) {
        Properties null_prop;
        for (int i = 0; i < k; i++)
            if (null_prop.fnt_serialize(reinterpret_cast<uint32_t*>(data[i]),
                                        md / 4) == -1)
                return -1;
        for (int i = 0; i < m; i++)
            if (props[i].fnt_serialize(reinterpret_cast<uint32_t*>(parity[i]),
                                       md / 4) == -1)
                return -1;
    } else {
        for (int i = 0; i < k; i++)
            if (props[i].fnt_serialize(reinterpret_cast<uint32_t*>(data[i]),
                                       md / 4) == -1)
                return -1;
        for (int i = 0; i < m; i++)
            if (props[k + i].fnt_serialize(
                    reinterpret_cast<uint32_t*>(parity[i]), md / 4) == -1)
                return -1;
    }
    return 0;
}

static int load(RsFnt<uint32_t>* fec, int sys, uint8_t** data,
                uint8_t** parity, const int* missing, int md,
                std::vector<uint8_t*>& par_vec,
                std::vector<Properties>& props, bool all_ptrs)
{
    int k = static_cast<int>(fec->n_data), m = static_cast<int>(fec->n_parities);
    if (sys) {
        for (int i = 0; i < m; i++) {
            if (!missing[k + i]) {
                if (props[i].fnt_deserialize(
                        reinterpret_cast<uint32_t*>(parity[i]), md / 4) == -1)
                    return -1;
            }
            if (!missing[k + i] || all_ptrs)
                par_vec[i] = parity[i] ? parity[i] + md : nullptr;
        }
    } else {
        for (int i = 0; i < k; i++) {
            if (!missing[i]) {
                if (props[i].fnt_deserialize(
                        reinterpret_cast<uint32_t*>(data[i]), md / 4) == -1)
                    return -1;
            }
            if (!missing[i] || all_ptrs)
                par_vec[i] = data[i] ? data[i] + md : nullptr;
        }
        for (int i = 0; i < m; i++) {
            if (!missing[k + i]) {
                if (props[k + i].fnt_deserialize(
                        reinterpret_cast<uint32_t*>(parity[i]), md / 4) == -1)
                    return -1;
            }
            if (!missing[k + i] || all_ptrs)
                par_vec[k + i] = parity[i] ? parity[i] + md : nullptr;
        }
    }
    return 0;
}

/* quadiron_fnt32_decode glue: src/quadiron_c.cpp:152-229 */
int ref_c_decode(int sys, int k, int m, uint8_t** data, uint8_t** parity,
                 const int* missing_idxs, size_t block_size)
{
    std::unique_ptr<RsFnt<uint32_t>> fec(make(sys, k, m, 1024));
    unsigned no = fec->n_outputs;
    std::vector<uint8_t*> data_vec(k), par_vec(no, nullptr);
    std::vector<Properties> props(no);
    std::vector<int> miss(missing_idxs, missing_idxs + k + m);
    std::vector<bool> wanted(k, true);
    int md = md_size(block_size);
    if (load(fec.get(), sys, data, parity, missing_idxs, md, par_vec, props,
             false))
        return -1;
    for (int i = 0; i < k; i++)
        data_vec[i] = data[i] + md;
    if (!fec->decode_blocks_vertical(
            data_vec, par_vec, props, miss, wanted, block_size))
        return -1;
    /* The reference clears parities_props[i] for i < n_data here, which
     * indexes past the end of that vector when systematic and m < k
     * (src/quadiron_c.cpp:219-226, heap overflow under ASan).  The intent
     * -- an empty FNT1 header on every data fragment -- is restated with a
     * local empty Properties instead. */
    for (int i = 0; i < k; i++) {
        Properties empty;
        if (empty.fnt_serialize(reinterpret_cast<uint32_t*>(data[i]),
                                md / 4) == -1)
            return -1;
    }
    return 0;
}

/* quadiron_fnt32_reconstruct glue: src/quadiron_c.cpp:231-406 */
int ref_c_reconstruct(int sys, int k, int m, uint8_t** data, uint8_t** parity,
                      const int* missing_idxs, unsigned dest,
                      size_t block_size)
{
    std::unique_ptr<RsFnt<uint32_t>> fec(make(sys, k, m, 1024));
    unsigned no = fec->n_outputs;
    std::vector<uint8_t*> data_vec(k), par_vec(no, nullptr);
    std::vector<Properties> props(no);
    std::vector<int> miss(missing_idxs, missing_idxs + k + m);
    std::vector<bool> wanted_data(k, false), wanted(no, false);
    int md = md_size(block_size);
    if (load(fec.get(), sys, data, parity, missing_idxs, md, par_vec, props,
             true))
        return -1;
    for (int i = 0; i < k; i++)
        data_vec[i] = data[i] ? data[i] + md : nullptr;
    if (sys && dest < static_cast<unsigned>(k)) {
        wanted[dest] = true;
        std::vector<bool> w(k, false);
        w[dest] = true;
        if (!fec->decode_blocks_vertical(
                data_vec, par_vec, props, miss, w, block_size))
            return -1;
        Properties null_prop;
        return null_prop.fnt_serialize(
                   reinterpret_cast<uint32_t*>(data[dest]), md / 4) == -1
                   ? -1
                   : 0;
    }
    std::vector<std::vector<uint8_t>> blocks(k);
    bool need = false;
    for (int i = 0; i < k; i++) {
        if (!sys || missing_idxs[i]) {
            need = true;
            wanted_data[i] = true;
            blocks[i].resize(block_size);
            data_vec[i] = blocks[i].data();
        }
    }
    if (need &&
        !fec->decode_blocks_vertical(
            data_vec, par_vec, props, miss, wanted_data, block_size))
        return -1;
    unsigned w = sys ? dest - k : dest;
    if (w >= no)
        return -1;
    wanted[w] = true;
    std::vector<std::vector<uint8_t>> scratch(no);
    for (unsigned i = 0; i < no; i++)
        if (!par_vec[i]) {
            scratch[i].resize(block_size + 1);
            par_vec[i] = scratch[i].data();
        }
    uint8_t* target = sys ? parity[w] : (w < static_cast<unsigned>(k) ? data[w] : parity[w - k]);
    par_vec[w] = target + md;
    fec->encode_blocks_vertical(data_vec, par_vec, props, wanted, block_size);
    return props[w].fnt_serialize(reinterpret_cast<uint32_t*>(target),
                                  md / 4) == -1
               ? -1
               : 0;
}

/*
 * RS-NF4 (src/fec_rs_nf4.h): RsNf4<T>(word_size, k, m, pkt) with the word
 * type the reference benchmark picks (benchmark/benchmark.cpp:283-306,
 * 696-718: sizeof(T) >= 2 * word_size), through the same vertical block API.
 * OOR marks are (word offset, component flag) pairs.
 */
int ref_nf4_n_outputs(int ws, int k, int m)
{
    if (ws == 2)
        return quadiron::fec::RsNf4<uint32_t>(ws, k, m, 8).n_outputs;
    if (ws == 4)
        return quadiron::fec::RsNf4<uint64_t>(ws, k, m, 8).n_outputs;
    return quadiron::fec::RsNf4<__uint128_t>(ws, k, m, 8).n_outputs;
}

void ref_nf4_encode_blocks(int ws, int k, int m, size_t pkt, uint8_t** data,
                           uint8_t** outputs, size_t block_bytes, uint32_t* oor,
                           uint32_t* flags, uint32_t* oor_count, uint32_t cap)
{
    if (ws == 2)
        nf4_encode<uint32_t>(ws, k, m, pkt, data, outputs, block_bytes, oor,
                             flags, oor_count, cap);
    else if (ws == 4)
        nf4_encode<uint64_t>(ws, k, m, pkt, data, outputs, block_bytes, oor,
                             flags, oor_count, cap);
    else
        nf4_encode<__uint128_t>(ws, k, m, pkt, data, outputs, block_bytes, oor,
                                flags, oor_count, cap);
}

/* `missing`: code_len (= n_outputs, non-systematic) flags, nonzero = missing */
int ref_nf4_decode_blocks(int ws, int k, int m, size_t pkt, uint8_t** data,
                          uint8_t** parities, const uint32_t* oor,
                          const uint32_t* flags, const uint32_t* oor_count,
                          uint32_t cap, const int* missing, const int* wanted,
                          size_t block_bytes)
{
    if (ws == 2)
        return nf4_decode<uint32_t>(ws, k, m, pkt, data, parities, oor, flags,
                                    oor_count, cap, missing, wanted, block_bytes);
    if (ws == 4)
        return nf4_decode<uint64_t>(ws, k, m, pkt, data, parities, oor, flags,
                                    oor_count, cap, missing, wanted, block_bytes);
    return nf4_decode<__uint128_t>(ws, k, m, pkt, data, parities, oor, flags,
                                   oor_count, cap, missing, wanted, block_bytes);
}

/*
 * CPU baseline: `threads` independent replicas (the reference bench's -g
 * model, benchmark/benchmark.cpp:813-817), each repeatedly encoding one
 * stripe of k fragments x pkt words (one encode_blocks_vertical call,
 * pkt_size = pkt) and decoding it back from a fixed erasure pattern
 * (`missing`), until `min_seconds` of wall time have passed (at least one
 * stripe each).  Returns the wall seconds of the whole job; *stripes
 * receives the stripes done by all threads together, enc_s/dec_s the
 * per-phase thread-seconds summed over all threads.
 */
double ref_bench(int sys, int k, int m, size_t pkt, double min_seconds, int threads,
                 const int* missing, long long* stripes, double* enc_s,
                 double* dec_s)
{
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    std::vector<double> te(threads, 0), td(threads, 0);
    std::vector<long long> done(threads, 0);
    for (int t = 0; t < threads; t++) {
        pool.emplace_back([=, &te, &td, &done]() {
            std::unique_ptr<RsFnt<uint32_t>> f(make(sys, k, m, pkt));
            unsigned no = f->n_outputs;
            size_t bytes = pkt * 2;
            std::vector<std::vector<uint8_t>> d(k, std::vector<uint8_t>(bytes));
            std::vector<std::vector<uint8_t>> o(no, std::vector<uint8_t>(bytes));
            std::vector<std::vector<uint8_t>> r(k, std::vector<uint8_t>(bytes));
            uint64_t s = 0x51D00001ull + static_cast<uint64_t>(t);
            for (int i = 0; i < k; i++)
                for (size_t j = 0; j < bytes; j++) {
                    s = s * 6364136223846793005ull + 1442695040888963407ull;
                    d[i][j] = static_cast<uint8_t>(s >> 56);
                }
            std::vector<uint8_t*> dv(k), ov(no), rv(k), pv(no);
            for (int i = 0; i < k; i++) {
                dv[i] = d[i].data();
                rv[i] = r[i].data();
            }
            for (unsigned i = 0; i < no; i++)
                ov[i] = o[i].data();
            std::vector<Properties> props(no);
            std::vector<bool> wanted(no, true), wk(k, true);
            std::vector<int> miss(missing, missing + k + m);
            for (unsigned i = 0; i < no; i++) {
                unsigned id = sys ? k + i : i;
                pv[i] = miss[id] ? nullptr : ov[i];
            }
            for (;;) {
                auto a = std::chrono::steady_clock::now();
                f->encode_blocks_vertical(dv, ov, props, wanted, bytes);
                auto b = std::chrono::steady_clock::now();
                if (sys)
                    for (int i = 0; i < k; i++)
                        rv[i] = miss[i] ? r[i].data() : d[i].data();
                f->decode_blocks_vertical(rv, pv, props, miss, wk, bytes);
                auto c = std::chrono::steady_clock::now();
                te[t] += std::chrono::duration<double>(b - a).count();
                td[t] += std::chrono::duration<double>(c - b).count();
                done[t]++;
                if (std::chrono::duration<double>(c - t0).count() >= min_seconds)
                    break;
            }
        });
    }
    for (auto& th : pool)
        th.join();
    auto t1 = std::chrono::steady_clock::now();
    long long total = 0;
    for (long long v : done)
        total += v;
    if (stripes)
        *stripes = total;
    // thread-seconds spent in encode / decode, summed over the threads
    // (per stripe: / *stripes)
    double se = 0, sd = 0;
    for (int t = 0; t < threads; t++) {
        se += te[t];
        sd += td[t];
    }
    if (enc_s)
        *enc_s = se;
    if (dec_s)
        *dec_s = sd;
    return std::chrono::duration<double>(t1 - t0).count();
}

} // extern "C"
