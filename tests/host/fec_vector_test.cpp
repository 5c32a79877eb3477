// The reference's FEC round-trip unit test (test/fec_utest.cpp:38-95
// run_test, run by TestFnt / TestFntSys at :132-156) ported onto
// qi::fec::RsFnt's horizontal API -- encode(Vector), init_context_dec,
// decode(context, Vector) -- plus a Buffers round trip checked against the
// block API (itself pinned to the reference's golden vectors).  Test
// infrastructure: built by quadiron_amd/csrc/Makefile next to the library,
// run on the GPU by tests/test_fec_vector.py.  Exit status 0 = pass.
#include <algorithm>
#include <cstdio>
#include <memory>
#include <numeric>
#include <random>
#include <vector>

#include "../../include/qi_fec.hpp"

using qi::Properties;
using qi::fec::FecType;
using qi::fec::RsFnt;
namespace vec = qi::vec;

static int fails = 0;

#define EXPECT(cond, ...)                                \
    do {                                                 \
        if (!(cond)) {                                   \
            std::fprintf(stderr, "FAIL %s: ", #cond);    \
            std::fprintf(stderr, __VA_ARGS__);           \
            std::fprintf(stderr, "\n");                  \
            fails++;                                     \
        }                                                \
    } while (0)

// test/fec_utest.cpp:45-95: 1000 random data vectors, each encoded, then
// decoded from the first n_data of a random shuffle of the code_len ids
static void run_test(FecType type, unsigned seed)
{
    const unsigned n_data = 3, n_parities = 3, code_len = n_data + n_parities;
    RsFnt fec(type, 2, n_data, n_parities);
    vec::Vector data_frags(n_data), copied(n_data), encoded(fec.n), received(n_data),
        decoded(n_data), fragments_ids(n_data);
    std::vector<int> ids(code_len);
    std::iota(ids.begin(), ids.end(), 0);
    std::vector<Properties> props(code_len);
    std::mt19937 rng(seed);
    std::uniform_int_distribution<uint32_t> sym(0, 65535);
    unsigned marked = 0;
    for (int j = 0; j < 1000; j++) {
        for (unsigned i = 0; i < code_len; i++)
            props[i] = Properties();
        for (unsigned i = 0; i < n_data; i++)
            data_frags[i] = sym(rng);
        // every 50th vector: data whose first output is 65536 (an OOR mark
        // through encode and decode), as the reference's random data hits
        // rarely: output 0 = sum of the data symbols
        if (j % 50 == 0) {
            uint32_t s = 0;
            for (unsigned i = 1; i < n_data; i++)
                s = (s + data_frags[i]) % 65537u;
            const uint32_t d0 = (65536u + 65537u - s) % 65537u;
            if (d0 < 65536u)
                data_frags[0] = d0;
        }
        copied = data_frags;
        fec.encode(encoded, props, 0, data_frags);
        for (unsigned i = 0; i < code_len; i++)
            marked += static_cast<unsigned>(props[i].get_map().size());
        std::shuffle(ids.begin(), ids.end(), rng);
        for (unsigned i = 0; i < n_data; i++) {
            fragments_ids[i] = static_cast<uint32_t>(ids[i]);
            received[i] = encoded[ids[i]];
        }
        std::unique_ptr<qi::fec::DecodeContext> context =
            fec.init_context_dec(fragments_ids, props);
        fec.decode(*context, decoded, props, 0, received);
        EXPECT(copied == decoded, "type %d iteration %d", static_cast<int>(type), j);
    }
    EXPECT(marked >= 10, "only %u OOR marks exercised", marked);
}

// Buffers: encode(Buffers) equals the block API's outputs and marks (which
// keep 65536 as 0 + mark), and decode(context, Buffers) from a random k
// subset of the fragments returns the data
static void run_buffers(FecType type, unsigned k, unsigned m, size_t size, unsigned seed)
{
    const bool sys = type == FecType::SYSTEMATIC;
    RsFnt fec(type, 2, k, m);
    const unsigned rows = sys ? m : fec.n;  // Buffers encode: n outputs (non-sys)
    std::mt19937 rng(seed);
    std::uniform_int_distribution<uint32_t> sym(0, 65535);
    vec::Buffers words(static_cast<int>(k), size), out(static_cast<int>(rows), size);
    for (unsigned i = 0; i < k; i++)
        for (size_t j = 0; j < size; j++)
            words.get(static_cast<int>(i))[j] = sym(rng);
    // crafted: output row 0 (non-sys: the sum of the data) = 65536 at column 7
    if (!sys) {
        uint32_t s = 0;
        for (unsigned i = 1; i < k; i++)
            s = (s + words.get(static_cast<int>(i))[7]) % 65537u;
        const uint32_t d0 = (65536u + 65537u - s) % 65537u;
        if (d0 < 65536u)
            words.get(0)[7] = d0;
    }
    std::vector<Properties> props(fec.n_outputs);
    fec.encode(out, props, 100, words);
    // the block API on the same data
    std::vector<std::vector<uint16_t>> d16(k, std::vector<uint16_t>(size)),
        o16(fec.n_outputs, std::vector<uint16_t>(size));
    std::vector<uint8_t*> dp(k), op(fec.n_outputs);
    for (unsigned i = 0; i < k; i++) {
        for (size_t j = 0; j < size; j++)
            d16[i][j] = static_cast<uint16_t>(words.get(static_cast<int>(i))[j]);
        dp[i] = reinterpret_cast<uint8_t*>(d16[i].data());
    }
    for (unsigned i = 0; i < fec.n_outputs; i++)
        op[i] = reinterpret_cast<uint8_t*>(o16[i].data());
    std::vector<Properties> bprops(fec.n_outputs);
    std::vector<bool> wanted(fec.n_outputs, true);
    fec.encode_blocks_vertical(dp, op, bprops, wanted, 2 * size);
    unsigned marks = 0;
    for (unsigned i = 0; i < fec.n_outputs; i++) {
        const uint32_t* o = out.get(static_cast<int>(i));
        for (size_t j = 0; j < size; j++)
            EXPECT((o[j] & 0xffffu) == o16[i][j] && o[j] <= 65536u, "encode row %u col %zu", i, j);
        EXPECT(props[i].get_map().size() == bprops[i].get_map().size(), "marks of row %u", i);
        for (size_t e = 0; e < std::min(props[i].get_map().size(), bprops[i].get_map().size());
             e++) {
            EXPECT(props[i].get_map()[e].first == 100 + bprops[i].get_map()[e].first,
                   "mark %zu of row %u", e, i);
            EXPECT(out.get(static_cast<int>(i))[bprops[i].get_map()[e].first] == 65536u,
                   "marked value of row %u", i);
        }
        marks += static_cast<unsigned>(props[i].get_map().size());
    }
    if (!sys)
        EXPECT(marks >= 1, "no OOR mark exercised");
    // decode from a random k subset of the fragments: data rows (sys) and
    // coded rows; the decode restores the marked 65536s from props itself,
    // so the received coded rows carry them as 0 (the byte form)
    const unsigned code_len = k + m;
    std::vector<unsigned> all(code_len);
    std::iota(all.begin(), all.end(), 0u);
    std::shuffle(all.begin(), all.end(), rng);
    vec::Vector ids(all.begin(), all.begin() + k);
    vec::Buffers recv(static_cast<int>(k), size), dec(static_cast<int>(k), size);
    for (unsigned i = 0; i < k; i++) {
        const unsigned id = ids[i];
        uint32_t* r = recv.get(static_cast<int>(i));
        for (size_t j = 0; j < size; j++) {
            if (sys && id < k)
                r[j] = words.get(static_cast<int>(id))[j];
            else
                r[j] = o16[sys ? id - k : id][j];
        }
    }
    auto ctx = fec.init_context_dec(ids, props, size);
    fec.decode(*ctx, dec, props, 100, recv);
    for (unsigned i = 0; i < k; i++)
        for (size_t j = 0; j < size; j++)
            EXPECT(dec.get(static_cast<int>(i))[j] == words.get(static_cast<int>(i))[j],
                   "decode row %u col %zu (type %d)", i, j, static_cast<int>(type));
}

// A block wider than one pipeline chunk (4 MiB per fragment) goes through
// the two-slot pipeline chunk by chunk, yet counts as ONE operation per
// block call, as the reference counts it (src/fec_base.h:1136, 1304;
// ADVICE r4), and round-trips.
static void run_block_ops()
{
    const unsigned k = 4, m = 4;
    const size_t bytes = 10u << 20;  // three chunks
    RsFnt fec(FecType::NON_SYSTEMATIC, 2, k, m);
    const unsigned no = static_cast<unsigned>(fec.get_n_outputs());
    std::vector<std::vector<uint8_t>> data(k, std::vector<uint8_t>(bytes)),
        coded(no, std::vector<uint8_t>(bytes)), out(k, std::vector<uint8_t>(bytes));
    std::mt19937 rng(7);
    for (auto& d : data)
        for (auto& b : d)
            b = static_cast<uint8_t>(rng());
    std::vector<uint8_t*> dp(k), cp(no), op(k);
    for (unsigned i = 0; i < k; i++) {
        dp[i] = data[i].data();
        op[i] = out[i].data();
    }
    for (unsigned i = 0; i < no; i++)
        cp[i] = coded[i].data();
    std::vector<Properties> props(no);
    std::vector<bool> wanted(no, true);
    fec.encode_blocks_vertical(dp, cp, props, wanted, bytes);
    EXPECT(fec.n_encode_ops == 1, "encode ops %llu", (unsigned long long)fec.n_encode_ops);
    std::vector<int> missing(k + m, 0);
    missing[0] = missing[2] = missing[5] = 1;  // decode from 1, 3, 4, 6
    std::vector<bool> want(k, true);
    fec.reset_stats_dec();
    EXPECT(fec.decode_blocks_vertical(op, cp, props, missing, want, bytes), "decode");
    EXPECT(fec.n_decode_ops == 1, "decode ops %llu", (unsigned long long)fec.n_decode_ops);
    for (unsigned i = 0; i < k; i++)
        EXPECT(out[i] == data[i], "block round trip, row %u", i);
}

int main()
{
    run_test(FecType::NON_SYSTEMATIC, 1);  // TestFnt
    run_test(FecType::SYSTEMATIC, 2);      // TestFntSys
    run_buffers(FecType::NON_SYSTEMATIC, 3, 3, 1000, 3);
    run_buffers(FecType::SYSTEMATIC, 3, 3, 1000, 4);
    run_buffers(FecType::NON_SYSTEMATIC, 16, 48, 4096, 5);
    run_buffers(FecType::SYSTEMATIC, 10, 6, 3000, 6);
    run_block_ops();
    if (fails) {
        std::fprintf(stderr, "%d failures\n", fails);
        return 1;
    }
    std::printf("fec_vector_test: ok\n");
    return 0;
}
