// qi_fec.hpp -- C++ FecCode-style API of the MI355X RS-FNT engine.
//
// Mirrors the part of QuadIron's C++ surface that the C-ABI, the benchmark and
// ec_driver use (src/fec_base.h:93-294, src/fec_rs_fnt.h:51-270,
// src/property.h:61-198): RsFnt<uint32_t>(type, word_size, k, m, pkt_size)
// with the vertical block and stream APIs and the OOR Properties side channel.
// Every transform runs on the GPU through include/qi_gpu.h; there is no CPU
// compute path.  word_size 2 (GF(65537)) only.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <istream>
#include <memory>
#include <ostream>
#include <utility>
#include <vector>

#include <sys/types.h>

struct qi_plan;

namespace qi {

static constexpr unsigned OOR_MARK = 1;  // src/property.h:49

// Sparse (location, marker) list of out-of-range symbols of one fragment.
class Properties {
  public:
    enum { FNT1 = 0x464E5431 };
    void add(size_t location, uint32_t marker)
    {
        props.emplace_back(location, marker);
    }
    void clear() { props.clear(); }
    void sort();
    const std::vector<std::pair<size_t, uint32_t>>& get_map() const
    {
        return props;
    }
    // FNT1 header (src/property.h:104-142): 0 on success, -1 on error
    int fnt_serialize(uint32_t* dwords, unsigned n_dwords) const;
    int fnt_deserialize(const uint32_t* dwords, unsigned n_dwords);

    friend std::istream& operator>>(std::istream& is, Properties& p);
    friend std::ostream& operator<<(std::ostream& os, const Properties& p);

  private:
    std::vector<std::pair<size_t, uint32_t>> props;
};

namespace vec {

// Containers of the horizontal API (QuadIron's vec::Vector<T> /
// vec::Buffers<T>, src/vec_vector.h, src/vec_buffers.h, with T = uint32_t):
// GF(65537) symbols 0 .. 65536 held in 32 bits.
using Vector = std::vector<uint32_t>;

class Buffers {
  public:
    Buffers(int n, size_t size)
        : n_(n), size_(size), mem_(static_cast<size_t>(n) * size, 0u)
    {
    }
    int get_n() const { return n_; }
    size_t get_size() const { return size_; }
    uint32_t* get(int i) { return mem_.data() + static_cast<size_t>(i) * size_; }
    const uint32_t* get(int i) const { return mem_.data() + static_cast<size_t>(i) * size_; }

  private:
    int n_;
    size_t size_;
    std::vector<uint32_t> mem_;
};

}  // namespace vec

namespace fec {

enum class FecType { SYSTEMATIC, NON_SYSTEMATIC };

// What FecCode::init_context_dec returns (src/fec_base.h:758-793,
// src/fec_context.h:66-274): the fragment ids a decode uses.  The
// per-pattern constants themselves are built on the device by every decode
// call, together with that call's OOR marks (decode_prepare).
class DecodeContext {
  public:
    explicit DecodeContext(const vec::Vector& ids, size_t size) : ids_(ids), size_(size) {}
    const vec::Vector& get_fragments_id() const { return ids_; }
    size_t get_size() const { return size_; }

  private:
    vec::Vector ids_;
    size_t size_;
};

class RsFnt {
  public:
    // throws std::invalid_argument (bad parameters / word_size != 2) or
    // std::runtime_error (no HIP device)
    RsFnt(FecType type, unsigned word_size, unsigned n_data,
          unsigned n_parities, size_t pkt_size = 8);
    ~RsFnt();
    RsFnt(const RsFnt&) = delete;
    RsFnt& operator=(const RsFnt&) = delete;

    FecType type;
    unsigned word_size, n_data, n_parities, code_len, n_outputs;
    size_t pkt_size, buf_size;
    unsigned n;

    uint64_t n_encode_ops = 0, n_decode_ops = 0;
    uint64_t total_enc_usec = 0, total_dec_usec = 0;

    int get_n_outputs() const;  // n (non-systematic) or m (systematic)

    void encode_blocks_vertical(std::vector<uint8_t*>& data_bufs,
                                std::vector<uint8_t*>& parities_bufs,
                                std::vector<Properties>& parities_props,
                                std::vector<bool>& wanted_idxs,
                                size_t block_size_bytes);

    bool decode_blocks_vertical(std::vector<uint8_t*>& data_bufs,
                                std::vector<uint8_t*>& parities_bufs,
                                std::vector<Properties>& parities_props,
                                std::vector<int>& missing_idxs,
                                std::vector<bool>& wanted_idxs,
                                size_t block_size_bytes);

    void encode_streams_vertical(
        const std::vector<std::istream*>& input_data_bufs,
        std::vector<std::ostream*>& output_parities_bufs,
        std::vector<Properties>& output_parities_props);

    bool decode_streams_vertical(
        const std::vector<std::istream*>& input_data_bufs,
        const std::vector<std::istream*>& input_parities_bufs,
        std::vector<Properties>& input_parities_props,
        std::vector<std::ostream*>& output_data_bufs);

    // Horizontal API (src/fec_base.h:129-178, 409-460, 740-878,
    // src/fec_rs_fnt.h:178-270): one codeword per Vector call, get_size()
    // codewords (columns) per Buffers call, all on the device.  As in the
    // reference, the Vector calls use the non-systematic code of length n
    // for both types (RsFnt::encode(Vector) is fft(output, words) then the
    // post-process over n_outputs; decode(Vector) returns the polynomial's
    // coefficients), and props are indexed by fragment id; the Buffers calls
    // follow the type (systematic: m parities out, the data rows decoded)
    // with props indexed by output / parity.  Data symbols must be < 65536
    // (16-bit input; std::invalid_argument otherwise).
    void encode(vec::Vector& output, std::vector<Properties>& props, off_t offset,
                const vec::Vector& words);
    void encode(vec::Buffers& output, std::vector<Properties>& props, off_t offset,
                const vec::Buffers& words);
    std::unique_ptr<DecodeContext> init_context_dec(const vec::Vector& fragments_ids,
                                                    std::vector<Properties>& input_props,
                                                    size_t size = 0);
    void decode(DecodeContext& context, vec::Vector& output,
                const std::vector<Properties>& props, off_t offset, vec::Vector& words);
    void decode(DecodeContext& context, vec::Buffers& output,
                const std::vector<Properties>& props, off_t offset, vec::Buffers& words);

    void reset_stats_enc()
    {
        n_encode_ops = 0;
        total_enc_usec = 0;
    }
    void reset_stats_dec()
    {
        n_decode_ops = 0;
        total_dec_usec = 0;
    }

    qi_plan* plan() const { return plan_; }

  private:
    // device encode of `words` columns on plan pl; outputs[i] NULL = not
    // wanted (pl's n_outputs of them)
    void encode_columns(qi_plan* pl, const uint8_t* const* data, uint8_t* const* outputs,
                        size_t words, std::vector<Properties>& props,
                        size_t offset);
    // device decode of `words` columns from the k selected fragments
    void decode_columns(qi_plan* pl, const std::vector<int>& ids,
                        const std::vector<const uint8_t*>& rows,
                        const std::vector<const Properties*>& props,
                        uint8_t* const* outputs, size_t words, size_t offset);
    bool select_fragments(const std::vector<int>& present,
                          std::vector<int>& ids) const;
    // the two-slot pinned pipeline behind the stream API and the blocks
    // wider than one chunk: read(h, pitch, cont) fills the next chunk's
    // input rows (pitch bytes apart) and returns the bytes per row (0: no
    // more); write(h, pitch, got, byte_offset) takes a finished chunk's
    // output rows, in chunk order
    using RowReader = std::function<size_t(uint8_t*, size_t, bool&)>;
    using RowWriter = std::function<void(const uint8_t*, size_t, size_t, size_t)>;
    void encode_pipe(const RowReader& read, const RowWriter& write,
                     std::vector<Properties>& props);
    void decode_pipe(const std::vector<int>& ids, const std::vector<const Properties*>& props,
                     const RowReader& read, const RowWriter& write);
    bool encode_blocks_pipe(const std::vector<uint8_t*>& data_bufs,
                            const std::vector<uint8_t*>& outs, std::vector<Properties>& props,
                            size_t words);
    bool decode_blocks_pipe(const std::vector<int>& ids, const std::vector<const uint8_t*>& rows,
                            const std::vector<const Properties*>& props,
                            const std::vector<uint8_t*>& outs, size_t words);

    // the non-systematic plan of length n behind the Vector calls (created
    // on first use)
    qi_plan* hplan();
    qi_plan* plan_ = nullptr;
    qi_plan* hplan_ = nullptr;
    // pinned two-slot pipeline of the stream API, kept across calls
    struct StreamPipe;
    std::unique_ptr<StreamPipe> pipe_;
};

// RS-NF4 (src/fec_rs_nf4.h:46-334, src/gf_nf4.h).  A word of word_size bytes
// packs gf_n = word_size / 2 GF(65537) components that are coded
// independently with RS-FNT's root and transform (NF4::get_nth_root
// replicates the prime-field root, gf_nf4.h:450-455; Radix2 as RsFnt,
// fec_rs_nf4.h:78-96).  So every 16-bit lane of the byte stream is one
// RS-FNT codeword and the device path is RS-FNT's.  Non-systematic only.
// OOR marks are (word offset, component bitmask) pairs (NF4::unpack,
// gf_nf4.h:391-446; restored by NF4::pack(a, flag), :372-383).  word_size 2,
// 4 or 8: the reference benchmark's T = uint32 / uint64 / __uint128_t
// (benchmark/benchmark.cpp:283-306, 696-718).
class RsNf4 {
  public:
    // throws std::invalid_argument (bad parameters / word_size) or
    // std::runtime_error (no HIP device)
    RsNf4(unsigned word_size, unsigned n_data, unsigned n_parities,
          size_t pkt_size = 8);
    RsNf4(const RsNf4&) = delete;
    RsNf4& operator=(const RsNf4&) = delete;

    unsigned word_size, n_data, n_parities, code_len, n_outputs, gf_n;
    size_t pkt_size, buf_size;
    unsigned n;

    int get_n_outputs() const { return static_cast<int>(n); }  // :115-118

    // only whole words are coded (block_size = bytes / word_size,
    // src/fec_base.h:1083); trailing bytes of a partial word are untouched
    void encode_blocks_vertical(std::vector<uint8_t*>& data_bufs,
                                std::vector<uint8_t*>& parities_bufs,
                                std::vector<Properties>& parities_props,
                                std::vector<bool>& wanted_idxs,
                                size_t block_size_bytes);
    bool decode_blocks_vertical(std::vector<uint8_t*>& data_bufs,
                                std::vector<uint8_t*>& parities_bufs,
                                std::vector<Properties>& parities_props,
                                std::vector<int>& missing_idxs,
                                std::vector<bool>& wanted_idxs,
                                size_t block_size_bytes);
    void encode_streams_vertical(
        const std::vector<std::istream*>& input_data_bufs,
        std::vector<std::ostream*>& output_parities_bufs,
        std::vector<Properties>& output_parities_props);
    bool decode_streams_vertical(
        const std::vector<std::istream*>& input_data_bufs,
        const std::vector<std::istream*>& input_parities_bufs,
        std::vector<Properties>& input_parities_props,
        std::vector<std::ostream*>& output_data_bufs);

    const RsFnt& lanes() const { return lanes_; }

  private:
    RsFnt lanes_;  // the 16-bit lane code (RsFnt NON_SYSTEMATIC, word_size 2)
};

// (16-bit lane, OOR_MARK) marks <-> (word, component mask) marks of gf_n
// lanes per word; lane marks must be ascending (as the encoders emit them)
void nf4_marks_from_lanes(const Properties& lanes, unsigned gf_n,
                          Properties& words);
void nf4_marks_to_lanes(const Properties& words, unsigned gf_n,
                        Properties& lanes);

}  // namespace fec
}  // namespace qi
