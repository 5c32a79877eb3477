// C++ FecCode-style API (include/qi_fec.hpp) on top of the device engine.
//
// The block/stream methods keep the reference's observable behaviour
// (fragment selection, tail handling, OOR side channel, offsets) while the
// per-packet loop of src/fec_base.h:1103-1150 becomes ONE device call over
// the whole block: outputs do not depend on the packet size.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <arpa/inet.h>
#include <chrono>
#include <memory>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>

#include "../../include/qi_fec.hpp"
#include "../../include/qi_gpu.h"
#include "qi_internal.h"
#include "qi_plan.h"

namespace qi {

// ------------------------------------------------------------- Properties

void Properties::sort()
{
    std::sort(props.begin(), props.end());
}

int Properties::fnt_serialize(uint32_t* dwords, unsigned n_dwords) const
{
    // src/property.h:104-118 (the last dword is left untouched)
    if ((2 + props.size()) > n_dwords)
        return -1;
    dwords[0] = htonl(FNT1);
    unsigned i = 2;
    for (auto const& it : props)
        dwords[i++] = htonl(static_cast<uint32_t>(it.first));
    dwords[1] = htonl(i - 2);
    for (unsigned d = i; d + 1 < n_dwords; d++)
        dwords[d] = 0;
    return 0;
}

int Properties::fnt_deserialize(const uint32_t* dwords, unsigned n_dwords)
{
    // src/property.h:125-142
    if (n_dwords < 2)
        return -1;
    if (ntohl(dwords[0]) != FNT1)
        return -1;
    const uint32_t n = ntohl(dwords[1]);
    if ((2 + static_cast<uint64_t>(n)) > n_dwords)
        return -1;
    for (uint32_t i = 0; i < n; i++)
        add(static_cast<size_t>(ntohl(dwords[i + 2])), OOR_MARK);
    return 0;
}

// text form of ec_driver's .props files (src/property.cpp:37-78)
std::istream& operator>>(std::istream& is, Properties& p)
{
    std::string line;
    while (std::getline(is, line)) {
        auto b = line.find_first_not_of(" \f\t\v");
        if (b == std::string::npos)
            continue;
        if (line[b] == '#' || line[b] == ';')
            continue;
        auto e = line.find('=', b);
        std::string key = line.substr(b, e - b);
        key.erase(key.find_last_not_of(" \f\t\v") + 1);
        if (key.empty())
            continue;
        b = line.find_first_not_of(" \f\n\r\t\v", e + 1);
        e = line.find_last_not_of(" \f\n\r\t\v") + 1;
        p.add(std::stoul(key), static_cast<uint32_t>(std::stoul(line.substr(b, e - b))));
    }
    return is;
}

std::ostream& operator<<(std::ostream& os, const Properties& p)
{
    for (auto const& it : p.get_map())
        os << it.first << " = " << it.second << '\n';
    return os;
}

namespace fec {

namespace {

constexpr size_t kAlign = 64;  // row stride granule (u16 words)

size_t pad_words(size_t w)
{
    return std::max<size_t>(kAlign, (w + kAlign - 1) / kAlign * kAlign);
}

void check(hipError_t e, const char* what)
{
    if (e != hipSuccess)
        throw std::runtime_error(std::string("HIP error in ") + what + ": " +
                                 hipGetErrorString(e));
}

void check_rc(int rc, const char* what)
{
    if (rc != 0)
        throw std::runtime_error(std::string(what) + " failed: " +
                                 std::to_string(rc));
}

struct Timer {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    uint64_t usec() const
    {
        return static_cast<uint64_t>(
            std::chrono::duration_cast<std::chrono::microseconds>(
                std::chrono::steady_clock::now() - t0)
                .count());
    }
};

}  // namespace

RsFnt::RsFnt(FecType t, unsigned ws, unsigned k, unsigned m, size_t pkt)
    : type(t), word_size(ws), n_data(k), n_parities(m), code_len(k + m),
      n_outputs(t == FecType::SYSTEMATIC ? m : k + m), pkt_size(pkt),
      buf_size(pkt * ws), n(0)
{
    if (ws != 2)
        throw std::invalid_argument(
            "RsFnt: only word_size 2 (GF(65537)) is supported");
    if (k < 1 || m < 1 || pkt < 1)
        throw std::invalid_argument("RsFnt: bad parameters");
    plan_ = qi_plan_create(static_cast<int>(k), static_cast<int>(m),
                           t == FecType::SYSTEMATIC ? 1 : 0);
    if (!plan_)
        throw std::runtime_error(
            "RsFnt: cannot create the GPU plan (no HIP device)");
    n = static_cast<unsigned>(qi_plan_n(plan_));
    const hipError_t e =
        hipStreamCreateWithFlags(&plan_->host.stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        // the destructor does not run for a throwing constructor
        qi_plan_destroy(plan_);
        plan_ = nullptr;
        check(e, "hipStreamCreate");
    }
}

RsFnt::~RsFnt()
{
    pipe_.reset();
    qi_plan_destroy(hplan_);
    qi_plan_destroy(plan_);
}

qi_plan* RsFnt::hplan()
{
    if (hplan_)
        return hplan_;
    qi_plan* p = qi_plan_create(static_cast<int>(n_data), static_cast<int>(n - n_data), 0);
    if (!p)
        throw std::runtime_error("RsFnt: cannot create the GPU plan");
    const hipError_t e = hipStreamCreateWithFlags(&p->host.stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        qi_plan_destroy(p);
        check(e, "hipStreamCreate");
    }
    hplan_ = p;
    return p;
}

int RsFnt::get_n_outputs() const
{
    // src/fec_rs_fnt.h:165-168
    return type == FecType::SYSTEMATIC ? static_cast<int>(n_parities)
                                       : static_cast<int>(n);
}

void RsFnt::encode_columns(qi_plan* pl, const uint8_t* const* data, uint8_t* const* outputs,
                           size_t words, std::vector<Properties>& props,
                           size_t offset)
{
    if (words == 0)
        return;
    HostState& h = pl->host;
    hipStream_t s = h.stream;
    const size_t P = pad_words(words);
    const size_t no = static_cast<size_t>(pl->n_outputs);
    size_t cap = 64 + words / 512;
    check(h.in.reserve(static_cast<size_t>(pl->k) * P * 2) ? hipSuccess : hipErrorOutOfMemory,
          "alloc");
    check(h.out.reserve(no * P * 2) ? hipSuccess : hipErrorOutOfMemory, "alloc");
    check(h.counts.reserve(no * 4) ? hipSuccess : hipErrorOutOfMemory, "alloc");
    uint16_t* din = static_cast<uint16_t*>(h.in.p);
    uint16_t* dout = static_cast<uint16_t*>(h.out.p);
    uint32_t* dcnt = static_cast<uint32_t*>(h.counts.p);
    for (int t = 0; t < pl->k; t++)
        check(hipMemcpyAsync(din + t * P, data[t], words * 2,
                             hipMemcpyHostToDevice, s),
              "H2D");
    std::vector<uint32_t> cnt(no);
    for (int attempt = 0; attempt < 2; attempt++) {
        check(h.entries.reserve(no * cap * 4) ? hipSuccess : hipErrorOutOfMemory,
              "alloc");
        check_rc(qi_gpu_oor_clear(dcnt, no, s), "oor_clear");
        check_rc(qi_gpu_encode(pl, din, 0, static_cast<long long>(P), dout, 0,
                               static_cast<long long>(P),
                               static_cast<long long>(words), 1, dcnt,
                               static_cast<uint32_t*>(h.entries.p),
                               static_cast<int>(cap), s),
                 "qi_gpu_encode");
        check(hipMemcpyAsync(cnt.data(), dcnt, no * 4, hipMemcpyDeviceToHost, s),
              "D2H");
        check(hipStreamSynchronize(s), "sync");
        const uint32_t mx = *std::max_element(cnt.begin(), cnt.end());
        if (mx <= cap)
            break;
        cap = mx;  // adversarial data: re-run with exact capacity
    }
    std::vector<uint32_t> ent(no * cap);
    check(hipMemcpyAsync(ent.data(), h.entries.p, no * cap * 4,
                         hipMemcpyDeviceToHost, s),
          "D2H");
    for (size_t i = 0; i < no; i++)
        if (outputs[i])
            check(hipMemcpyAsync(outputs[i], dout + i * P, words * 2,
                                 hipMemcpyDeviceToHost, s),
                  "D2H");
    check(hipStreamSynchronize(s), "sync");
    for (size_t i = 0; i < no; i++) {
        uint32_t* b = ent.data() + i * cap;
        std::sort(b, b + cnt[i]);
        for (uint32_t e = 0; e < cnt[i]; e++)
            props[i].add(offset + b[e], OOR_MARK);
    }
}

void RsFnt::decode_columns(qi_plan* pl, const std::vector<int>& ids,
                           const std::vector<const uint8_t*>& rows,
                           const std::vector<const Properties*>& props,
                           uint8_t* const* outputs, size_t words,
                           size_t offset)
{
    if (words == 0)
        return;
    HostState& h = pl->host;
    hipStream_t s = h.stream;
    const size_t P = pad_words(words);
    const int k = pl->k;
    // OOR marks of the received coded rows inside [offset, offset+words)
    std::vector<std::vector<uint32_t>> marks(k);
    size_t cap = 1;
    for (int i = 0; i < k; i++) {
        if (!props[i])
            continue;
        for (auto const& it : props[i]->get_map())
            if (it.first >= offset && it.first < offset + words)
                marks[i].push_back(static_cast<uint32_t>(it.first - offset));
        cap = std::max(cap, marks[i].size());
    }
    std::vector<uint32_t> hcnt(k), hent(static_cast<size_t>(k) * cap, 0);
    for (int i = 0; i < k; i++) {
        hcnt[i] = static_cast<uint32_t>(marks[i].size());
        std::copy(marks[i].begin(), marks[i].end(), hent.begin() + i * cap);
    }
    std::vector<uint16_t> hids(k);
    for (int i = 0; i < k; i++)
        hids[i] = static_cast<uint16_t>(ids[i]);
    const size_t ctx_bytes =
        qi_gpu_decode_ctx_bytes(pl, 1, static_cast<long long>(words));
    const size_t cnt_off = 0, ent_off = 64 * ((k * 4 + 63) / 64);
    if (!h.in.reserve(static_cast<size_t>(k) * P * 2) ||
        !h.out.reserve(static_cast<size_t>(k) * P * 2) ||
        !h.counts.reserve(ent_off + hent.size() * 4) ||
        !h.ids.reserve(k * 2) || !h.ctx.reserve(ctx_bytes))
        throw std::runtime_error("RsFnt: device allocation failed");
    uint16_t* din = static_cast<uint16_t*>(h.in.p);
    uint16_t* dout = static_cast<uint16_t*>(h.out.p);
    uint8_t* dcb = static_cast<uint8_t*>(h.counts.p);
    for (int i = 0; i < k; i++)
        check(hipMemcpyAsync(din + i * P, rows[i], words * 2,
                             hipMemcpyHostToDevice, s),
              "H2D");
    check(hipMemcpyAsync(dcb + cnt_off, hcnt.data(), k * 4, hipMemcpyHostToDevice,
                         s),
          "H2D");
    check(hipMemcpyAsync(dcb + ent_off, hent.data(), hent.size() * 4,
                         hipMemcpyHostToDevice, s),
          "H2D");
    check(hipMemcpyAsync(h.ids.p, hids.data(), k * 2, hipMemcpyHostToDevice, s),
          "H2D");
    // received rows staged by position; OOR buckets by position
    uint32_t* dcnt = reinterpret_cast<uint32_t*>(dcb + cnt_off);
    uint32_t* dent = reinterpret_cast<uint32_t*>(dcb + ent_off);
    check_rc(qi_gpu_decode_ctx_packed(pl, static_cast<uint16_t*>(h.ids.p), hids.data(), 1,
                                      dcnt, dent, static_cast<int>(cap),
                                      static_cast<long long>(words), h.ctx.p, s),
             "decode context");
    check_rc(qi_gpu_decode_packed(pl, h.ctx.p, din, 0, static_cast<long long>(P), dcnt,
                                  dent, static_cast<int>(cap), dout, 0,
                                  static_cast<long long>(P), static_cast<long long>(words), 1,
                                  s),
             "decode");
    for (int t = 0; t < k; t++)
        if (outputs[t])
            check(hipMemcpyAsync(outputs[t], dout + t * P, words * 2,
                                 hipMemcpyDeviceToHost, s),
                  "D2H");
    check(hipStreamSynchronize(s), "sync");
    if (qi_gpu_take_error(pl))
        throw std::runtime_error("RsFnt: OOR marks lost (bucket capacity)");
}

void RsFnt::encode_blocks_vertical(std::vector<uint8_t*>& data_bufs,
                                   std::vector<uint8_t*>& parities_bufs,
                                   std::vector<Properties>& parities_props,
                                   std::vector<bool>& wanted_idxs,
                                   size_t block_size_bytes)
{
    // src/fec_base.h:1066-1151
    for (auto& p : parities_props)
        p.clear();
    reset_stats_enc();
    const size_t words = block_size_bytes / word_size;
    std::vector<uint8_t*> outs(n_outputs, nullptr);
    for (unsigned i = 0; i < n_outputs; i++)
        if (wanted_idxs[i])
            outs[i] = parities_bufs[i];
    Timer tm;
    if (!encode_blocks_pipe(data_bufs, outs, parities_props, words)) {
        encode_columns(plan_, data_bufs.data(), outs.data(), words, parities_props, 0);
        n_encode_ops++;
    }
    total_enc_usec += tm.usec();
}

bool RsFnt::select_fragments(const std::vector<int>& present,
                             std::vector<int>& ids) const
{
    // first k present, data before parities: src/fec_base.h:1199-1236
    ids.clear();
    const bool sys = type == FecType::SYSTEMATIC;
    if (sys)
        for (unsigned i = 0; i < n_data; i++)
            if (present[i])
                ids.push_back(static_cast<int>(i));
    for (unsigned i = 0; i < n_outputs && ids.size() < n_data; i++) {
        const unsigned j = sys ? n_data + i : i;
        if (present[j])
            ids.push_back(static_cast<int>(j));
    }
    return ids.size() == n_data;
}

bool RsFnt::decode_blocks_vertical(std::vector<uint8_t*>& data_bufs,
                                   std::vector<uint8_t*>& parities_bufs,
                                   std::vector<Properties>& parities_props,
                                   std::vector<int>& missing_idxs,
                                   std::vector<bool>& wanted_idxs,
                                   size_t block_size_bytes)
{
    // src/fec_base.h:1177-1321
    const bool sys = type == FecType::SYSTEMATIC;
    std::vector<int> present(code_len);
    for (unsigned i = 0; i < code_len; i++)
        present[i] = missing_idxs[i] ? 0 : 1;
    if (sys) {
        unsigned nd = 0;
        for (unsigned i = 0; i < n_data; i++)
            nd += present[i];
        if (nd == n_data)
            return true;  // data in clear (src/fec_base.h:1208-1211)
    }
    std::vector<int> ids;
    if (!select_fragments(present, ids))
        return false;
    // DecodeContext sorts every input property list (src/fec_context.h:93-97)
    for (auto& p : parities_props)
        p.sort();
    reset_stats_dec();
    std::vector<const uint8_t*> rows(n_data);
    std::vector<const Properties*> props(n_data, nullptr);
    for (unsigned i = 0; i < n_data; i++) {
        const int id = ids[i];
        if (sys && id < static_cast<int>(n_data)) {
            rows[i] = data_bufs[id];
        } else {
            const int slot = sys ? id - static_cast<int>(n_data) : id;
            rows[i] = parities_bufs[slot];
            props[i] = &parities_props[slot];
        }
    }
    std::vector<uint8_t*> outs(n_data, nullptr);
    for (unsigned t = 0; t < n_data; t++)
        if (wanted_idxs[t])
            outs[t] = data_bufs[t];
    Timer tm;
    const size_t words = block_size_bytes / word_size;
    if (!decode_blocks_pipe(ids, rows, props, outs, words)) {
        decode_columns(plan_, ids, rows, props, outs.data(), words, 0);
        n_decode_ops++;
    }
    total_dec_usec += tm.usec();
    return true;
}

namespace {

size_t chunk_bytes(size_t buf_size)
{
    const size_t target = 4u << 20;
    return buf_size * std::max<size_t>(1, target / buf_size);
}

// read up to `len` bytes; returns bytes read (short = end of stream)
size_t read_full(std::istream* is, uint8_t* p, size_t len)
{
    is->read(reinterpret_cast<char*>(p), static_cast<std::streamsize>(len));
    return static_cast<size_t>(is->gcount());
}

}  // namespace

namespace {

// One stage of the pipelined stream API: pinned host staging, device
// buffers and a HIP stream.  Chunk i runs in slot i % 2, so reading chunk i
// from the input streams and writing chunk i-2 to the output streams overlap
// the transfers and kernels of chunk i-1.
struct StreamSlot {
    hipStream_t st = nullptr;
    uint8_t* host = nullptr;
    size_t host_bytes = 0;
    DevBuf in, out, small, ctx;
    size_t got = 0, offset = 0;
    uint32_t cap = 0;
    bool busy = false;
    StreamSlot()
    {
        check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
    }
    ~StreamSlot()
    {
        (void)hipStreamSynchronize(st);
        if (host)
            (void)hipHostFree(host);
        in.release();
        out.release();
        small.release();
        ctx.release();
        (void)hipStreamDestroy(st);
    }
    StreamSlot(const StreamSlot&) = delete;
    StreamSlot& operator=(const StreamSlot&) = delete;
    uint8_t* pinned(size_t n)
    {
        if (n > host_bytes) {
            if (host)
                (void)hipHostFree(host);
            host = nullptr;
            host_bytes = 0;
            check(hipHostMalloc(reinterpret_cast<void**>(&host), n,
                                hipHostMallocDefault),
                  "hipHostMalloc");
            host_bytes = n;
        }
        return host;
    }
    void dev(DevBuf& b, size_t n)
    {
        if (!b.reserve(n))
            throw std::runtime_error("RsFnt: device allocation failed");
    }
};

size_t round64(size_t n)
{
    return (n + 63) / 64 * 64;
}

// fn(i) for i < n on up to 16 threads: the fragments are independent
// streams (shard files, sockets), so they are read and written in parallel
template <typename F>
void parallel_for(size_t n, F fn)
{
    const size_t hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = std::min<size_t>({n, hw, 16});
    if (nt <= 1) {
        for (size_t i = 0; i < n; i++)
            fn(i);
        return;
    }
    std::vector<std::thread> pool;
    for (size_t t = 0; t < nt; t++)
        pool.emplace_back([&, t] {
            for (size_t i = t; i < n; i += nt)
                fn(i);
        });
    for (auto& th : pool)
        th.join();
}

// read `k` streams into rows `pitch` bytes apart: bytes read by every
// stream (short = end of stream), the tail of each row zeroed
size_t read_rows(const std::vector<std::istream*>& src, uint8_t* rows,
                 size_t pitch, bool& cont)
{
    std::vector<size_t> r(src.size());
    parallel_for(src.size(),
                 [&](size_t i) { r[i] = read_full(src[i], rows + i * pitch, pitch); });
    size_t got = pitch;
    for (size_t i = 0; i < src.size(); i++) {
        if (r[i] < pitch) {
            got = std::min(got, r[i]);
            cont = false;
        }
    }
    for (size_t i = 0; i < src.size(); i++)
        std::memset(rows + i * pitch + got, 0, pitch - got);
    return got;
}

}  // namespace

struct RsFnt::StreamPipe {
    StreamSlot slot[2];
};

void RsFnt::encode_streams_vertical(
    const std::vector<std::istream*>& input_data_bufs,
    std::vector<std::ostream*>& output_parities_bufs,
    std::vector<Properties>& output_parities_props)
{
    // src/fec_base.h:463-542: packets of buf_size bytes, zero padded tail,
    // `read_bytes` of every output written for the last packet.  Here whole
    // chunks of packets go through the two-slot pinned pipeline.
    reset_stats_enc();
    Timer tm;
    encode_pipe(
        [&](uint8_t* h, size_t pitch, bool& cont) {
            return read_rows(input_data_bufs, h, pitch, cont);
        },
        [&](const uint8_t* hout, size_t pitch, size_t got, size_t) {
            parallel_for(n_outputs, [&](size_t i) {
                output_parities_bufs[i]->write(reinterpret_cast<const char*>(hout + i * pitch),
                                               static_cast<std::streamsize>(got));
            });
        },
        output_parities_props);
    total_enc_usec += tm.usec();
}

void RsFnt::encode_pipe(const RowReader& read, const RowWriter& write,
                        std::vector<Properties>& output_parities_props)
{
    // chunks of whole packets alternate between two slots (pinned staging,
    // device buffers, a HIP stream each): while one chunk is in H2D ->
    // kernels -> D2H, the host fills the other slot with the next chunk and
    // writes out the previous one
    for (auto& p : output_parities_props)
        p.clear();
    const size_t CH = chunk_bytes(buf_size);  // a multiple of 128 bytes
    const size_t P = CH / 2, k = n_data, no = n_outputs;
    const uint32_t cap = static_cast<uint32_t>(64 + P / 512);
    // pinned: k input rows, no output rows, OOR counts, OOR entries
    const size_t in_b = k * CH, out_b = no * CH, cnt_b = round64(no * 4);
    const size_t ent_b = no * cap * 4;
    if (!pipe_)
        pipe_.reset(new StreamPipe);
    StreamSlot* slot = pipe_->slot;
    auto finish = [&](StreamSlot& sl) {
        check(hipStreamSynchronize(sl.st), "sync");
        sl.busy = false;
        uint8_t* hout = sl.host + in_b;
        const uint32_t* cnt = reinterpret_cast<const uint32_t*>(hout + out_b);
        const uint32_t* ent = reinterpret_cast<const uint32_t*>(hout + out_b + cnt_b);
        const size_t words = (sl.got + 1) / 2;
        const uint32_t mx = *std::max_element(cnt, cnt + no);
        if (mx > cap) {
            // adversarial data: redo this chunk synchronously, exact capacity
            std::vector<const uint8_t*> dp(k);
            std::vector<uint8_t*> op(no);
            for (size_t i = 0; i < k; i++)
                dp[i] = sl.host + i * CH;
            for (size_t i = 0; i < no; i++)
                op[i] = hout + i * CH;
            encode_columns(plan_, dp.data(), op.data(), words, output_parities_props,
                           sl.offset);
        } else {
            for (size_t i = 0; i < no; i++) {
                std::vector<uint32_t> b(ent + i * cap, ent + i * cap + cnt[i]);
                std::sort(b.begin(), b.end());
                for (uint32_t e : b)
                    output_parities_props[i].add(sl.offset + e, OOR_MARK);
            }
        }
        write(hout, CH, sl.got, 2 * sl.offset);
    };
    size_t offset = 0;
    unsigned it = 0;
    bool cont = true;
    while (cont) {
        StreamSlot& sl = slot[it & 1];
        if (sl.busy)
            finish(sl);
        uint8_t* h = sl.pinned(in_b + out_b + cnt_b + ent_b);
        const size_t got = read(h, CH, cont);
        if (got == 0)
            break;
        const size_t words = (got + 1) / 2;
        sl.dev(sl.in, in_b);
        sl.dev(sl.out, out_b);
        sl.dev(sl.small, cnt_b + ent_b);
        uint32_t* dcnt = static_cast<uint32_t*>(sl.small.p);
        uint32_t* dent = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(sl.small.p) + cnt_b);
        check(hipMemcpyAsync(sl.in.p, h, k * CH, hipMemcpyHostToDevice, sl.st), "H2D");
        check_rc(qi_gpu_oor_clear(dcnt, no, sl.st), "oor_clear");
        check_rc(qi_gpu_encode(plan_, static_cast<uint16_t*>(sl.in.p), 0,
                               static_cast<long long>(P),
                               static_cast<uint16_t*>(sl.out.p), 0,
                               static_cast<long long>(P), static_cast<long long>(words),
                               1, dcnt, dent, static_cast<int>(cap), sl.st),
                 "qi_gpu_encode");
        check(hipMemcpyAsync(h + in_b, sl.out.p, out_b, hipMemcpyDeviceToHost, sl.st),
              "D2H");
        check(hipMemcpyAsync(h + in_b + out_b, sl.small.p, cnt_b + ent_b,
                             hipMemcpyDeviceToHost, sl.st),
              "D2H");
        sl.got = got;
        sl.offset = offset;
        sl.busy = true;
        offset += got / 2;
        n_encode_ops++;
        it++;
    }
    // drain in chunk order: the older pending chunk sits in slot it % 2
    if (slot[it & 1].busy)
        finish(slot[it & 1]);
    if (slot[(it + 1) & 1].busy)
        finish(slot[(it + 1) & 1]);
}

bool RsFnt::decode_streams_vertical(
    const std::vector<std::istream*>& input_data_bufs,
    const std::vector<std::istream*>& input_parities_bufs,
    std::vector<Properties>& input_parities_props,
    std::vector<std::ostream*>& output_data_bufs)
{
    // src/fec_base.h:898-1048, through the two-slot pipeline: the k received
    // rows of a chunk are staged back to back (packed decode)
    const bool sys = type == FecType::SYSTEMATIC;
    std::vector<int> present(code_len, 0);
    if (sys)
        for (unsigned i = 0; i < n_data; i++)
            present[i] = input_data_bufs[i] != nullptr;
    for (unsigned i = 0; i < n_outputs; i++)
        present[sys ? n_data + i : i] = input_parities_bufs[i] != nullptr;
    if (sys) {
        unsigned nd = 0;
        for (unsigned i = 0; i < n_data; i++)
            nd += present[i];
        if (nd == n_data)
            return true;
    }
    std::vector<int> ids;
    if (!select_fragments(present, ids))
        return false;
    for (auto& p : input_parities_props)
        p.sort();
    reset_stats_dec();
    const size_t k = n_data;
    std::vector<std::istream*> src(k);
    std::vector<const Properties*> props(k, nullptr);
    for (size_t i = 0; i < k; i++) {
        const int id = ids[i];
        if (sys && id < static_cast<int>(n_data)) {
            src[i] = input_data_bufs[id];
        } else {
            const int s_ = sys ? id - static_cast<int>(n_data) : id;
            src[i] = input_parities_bufs[s_];
            props[i] = &input_parities_props[s_];
        }
    }
    Timer tm;
    decode_pipe(
        ids, props,
        [&](uint8_t* h, size_t pitch, bool& cont) { return read_rows(src, h, pitch, cont); },
        [&](const uint8_t* hout, size_t pitch, size_t got, size_t) {
            parallel_for(k, [&](size_t i) {
                if (output_data_bufs[i])
                    output_data_bufs[i]->write(reinterpret_cast<const char*>(hout + i * pitch),
                                               static_cast<std::streamsize>(got));
            });
        });
    total_dec_usec += tm.usec();
    return true;
}

void RsFnt::decode_pipe(const std::vector<int>& ids, const std::vector<const Properties*>& props,
                        const RowReader& read, const RowWriter& write)
{
    const size_t k = n_data;
    // OOR marks of each received row (ascending), consumed chunk by chunk
    std::vector<std::vector<size_t>> marks(k);
    for (size_t i = 0; i < k; i++)
        if (props[i])
            for (auto const& it : props[i]->get_map())
                marks[i].push_back(it.first);
    std::vector<size_t> mpos(k, 0);
    const size_t CH = chunk_bytes(buf_size);
    const size_t P = CH / 2;
    const size_t io_b = k * CH, ids_b = round64(k * 2), cnt_b = round64(k * 4);
    if (!pipe_)
        pipe_.reset(new StreamPipe);
    StreamSlot* slot = pipe_->slot;
    auto finish = [&](StreamSlot& sl) {
        check(hipStreamSynchronize(sl.st), "sync");
        sl.busy = false;
        if (qi_gpu_take_error(plan_))
            throw std::runtime_error("RsFnt: OOR marks lost (bucket capacity)");
        write(sl.host + io_b, CH, sl.got, 2 * sl.offset);
    };
    size_t offset = 0;
    unsigned it = 0;
    bool cont = true;
    while (cont) {
        StreamSlot& sl = slot[it & 1];
        if (sl.busy)
            finish(sl);
        // the chunk's marks per received row (positions relative to it)
        const size_t words_max = P;
        std::vector<std::vector<uint32_t>> cm(k);
        uint32_t cap = 1;
        for (size_t i = 0; i < k; i++) {
            while (mpos[i] < marks[i].size() && marks[i][mpos[i]] < offset)
                mpos[i]++;
            size_t e = mpos[i];
            while (e < marks[i].size() && marks[i][e] < offset + words_max)
                cm[i].push_back(static_cast<uint32_t>(marks[i][e++] - offset));
            cap = std::max<uint32_t>(cap, static_cast<uint32_t>(cm[i].size()));
        }
        const size_t ent_b = round64(static_cast<size_t>(k) * cap * 4);
        const size_t small_b = ids_b + cnt_b + ent_b;
        uint8_t* h = sl.pinned(2 * io_b + small_b);
        const size_t got = read(h, CH, cont);
        if (got == 0)
            break;
        const size_t words = (got + 1) / 2;
        uint8_t* hs = h + 2 * io_b;
        uint16_t* hids = reinterpret_cast<uint16_t*>(hs);
        uint32_t* hcnt = reinterpret_cast<uint32_t*>(hs + ids_b);
        uint32_t* hent = reinterpret_cast<uint32_t*>(hs + ids_b + cnt_b);
        for (size_t i = 0; i < k; i++) {
            hids[i] = static_cast<uint16_t>(ids[i]);
            hcnt[i] = static_cast<uint32_t>(cm[i].size());
            std::copy(cm[i].begin(), cm[i].end(), hent + i * cap);
        }
        // the context's size follows this chunk's width (a 256 < k <= 384
        // context is larger at whole-tile widths than at ragged ones)
        const size_t ctx_b = qi_gpu_decode_ctx_bytes(plan_, 1, static_cast<long long>(words));
        sl.dev(sl.in, io_b);
        sl.dev(sl.out, io_b);
        sl.dev(sl.small, small_b);
        sl.dev(sl.ctx, ctx_b);
        uint8_t* ds = static_cast<uint8_t*>(sl.small.p);
        const uint16_t* dids = reinterpret_cast<const uint16_t*>(ds);
        const uint32_t* dcnt = reinterpret_cast<const uint32_t*>(ds + ids_b);
        const uint32_t* dent = reinterpret_cast<const uint32_t*>(ds + ids_b + cnt_b);
        check(hipMemcpyAsync(sl.in.p, h, io_b, hipMemcpyHostToDevice, sl.st), "H2D");
        check(hipMemcpyAsync(sl.small.p, hs, small_b, hipMemcpyHostToDevice, sl.st),
              "H2D");
        check_rc(qi_gpu_decode_ctx_packed(plan_, dids, hids, 1, dcnt, dent,
                                          static_cast<int>(cap),
                                          static_cast<long long>(words), sl.ctx.p,
                                          sl.st),
                 "decode context");
        check_rc(qi_gpu_decode_packed(plan_, sl.ctx.p, static_cast<uint16_t*>(sl.in.p),
                                      0, static_cast<long long>(P), dcnt, dent,
                                      static_cast<int>(cap),
                                      static_cast<uint16_t*>(sl.out.p), 0,
                                      static_cast<long long>(P),
                                      static_cast<long long>(words), 1, sl.st),
                 "decode");
        check(hipMemcpyAsync(h + io_b, sl.out.p, io_b, hipMemcpyDeviceToHost, sl.st),
              "D2H");
        sl.got = got;
        sl.offset = offset;
        sl.busy = true;
        offset += got / 2;
        n_decode_ops++;
        it++;
    }
    if (slot[it & 1].busy)
        finish(slot[it & 1]);
    if (slot[(it + 1) & 1].busy)
        finish(slot[(it + 1) & 1]);
}

// Blocks wider than one pipeline chunk (quadiron_fnt32_encode / _decode on
// multi-MiB fragments) go through the same two-slot pinned pipeline as the
// streams: the caller's rows are copied chunk by chunk into pinned staging
// (parallel over the fragments) while the previous chunk is on the device,
// so H2D, kernels, D2H and the host copies overlap.  Returns false for
// blocks of one chunk or less (one synchronous device call).
bool RsFnt::encode_blocks_pipe(const std::vector<uint8_t*>& data_bufs,
                               const std::vector<uint8_t*>& outs,
                               std::vector<Properties>& props, size_t words)
{
    if (words <= chunk_bytes(buf_size) / 2)
        return false;
    const size_t total = 2 * words;
    size_t pos = 0;
    // one operation per block call, as the reference counts it
    // (src/fec_base.h:1136); the pipe counts its chunks
    const uint64_t ops = n_encode_ops;
    encode_pipe(
        [&](uint8_t* h, size_t pitch, bool& cont) {
            const size_t got = std::min(pitch, total - pos);
            parallel_for(n_data, [&](size_t i) {
                std::memcpy(h + i * pitch, data_bufs[i] + pos, got);
                std::memset(h + i * pitch + got, 0, pitch - got);
            });
            pos += got;
            cont = pos < total;
            return got;
        },
        [&](const uint8_t* hout, size_t pitch, size_t got, size_t off) {
            parallel_for(n_outputs, [&](size_t i) {
                if (outs[i])
                    std::memcpy(outs[i] + off, hout + i * pitch, got);
            });
        },
        props);
    n_encode_ops = ops + 1;
    return true;
}

bool RsFnt::decode_blocks_pipe(const std::vector<int>& ids,
                               const std::vector<const uint8_t*>& rows,
                               const std::vector<const Properties*>& props,
                               const std::vector<uint8_t*>& outs, size_t words)
{
    if (words <= chunk_bytes(buf_size) / 2)
        return false;
    const size_t total = 2 * words;
    size_t pos = 0;
    const uint64_t ops = n_decode_ops;  // one per block call (src/fec_base.h:1304)
    decode_pipe(
        ids, props,
        [&](uint8_t* h, size_t pitch, bool& cont) {
            const size_t got = std::min(pitch, total - pos);
            parallel_for(n_data, [&](size_t i) {
                std::memcpy(h + i * pitch, rows[i] + pos, got);
                std::memset(h + i * pitch + got, 0, pitch - got);
            });
            pos += got;
            cont = pos < total;
            return got;
        },
        [&](const uint8_t* hout, size_t pitch, size_t got, size_t off) {
            parallel_for(n_data, [&](size_t i) {
                if (outs[i])
                    std::memcpy(outs[i] + off, hout + i * pitch, got);
            });
        });
    n_decode_ops = ops + 1;
    return true;
}

// ---------------------------------------------------- horizontal API

namespace {

std::vector<unsigned> id_order(const vec::Vector& ids, unsigned k)
{
    std::vector<unsigned> ord(k);
    for (unsigned i = 0; i < k; i++)
        ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](unsigned a, unsigned b) { return ids[a] < ids[b]; });
    for (unsigned i = 1; i < k; i++)
        if (ids[ord[i]] == ids[ord[i - 1]])
            throw std::invalid_argument("RsFnt::decode: repeated fragment id");
    return ord;
}

bool marked_at(const Properties& p, size_t loc)
{
    for (auto const& it : p.get_map())
        if (it.first == loc && it.second == OOR_MARK)
            return true;
    return false;
}

}  // namespace

void RsFnt::encode(vec::Vector& output, std::vector<Properties>& props, off_t offset,
                   const vec::Vector& words)
{
    // src/fec_rs_fnt.h:178-201: fft->fft(output, words) -- the n-point NTT of
    // the zero-padded data whatever the type -- then encode_post_process: an
    // output i < n_outputs equal to 65536 is marked at `offset` and set to 0
    if (words.size() < n_data || output.size() < n || props.size() < n_outputs)
        throw std::invalid_argument("RsFnt::encode: vector sizes");
    std::vector<uint16_t> in(n_data), out(n);
    for (unsigned i = 0; i < n_data; i++) {
        if (words[i] > 65535u)
            throw std::invalid_argument("RsFnt::encode: data symbol >= 65536");
        in[i] = static_cast<uint16_t>(words[i]);
    }
    std::vector<const uint8_t*> dp(n_data);
    std::vector<uint8_t*> op(n);
    for (unsigned i = 0; i < n_data; i++)
        dp[i] = reinterpret_cast<const uint8_t*>(&in[i]);
    for (unsigned i = 0; i < n; i++)
        op[i] = reinterpret_cast<uint8_t*>(&out[i]);
    std::vector<Properties> marks(n);
    encode_columns(hplan(), dp.data(), op.data(), 1, marks, 0);
    for (unsigned i = 0; i < n; i++)
        output[i] = marks[i].get_map().empty() ? out[i] : 65536u;
    for (unsigned i = 0; i < n_outputs; i++) {
        if (output[i] == 65536u) {
            props[i].add(static_cast<size_t>(offset), OOR_MARK);
            output[i] = 0;
        }
    }
    n_encode_ops++;
}

void RsFnt::encode(vec::Buffers& output, std::vector<Properties>& props, off_t offset,
                   const vec::Buffers& words)
{
    // src/fec_rs_fnt.h:231-270: systematic -> the m parities (interpolation
    // + NTT), otherwise the n outputs of the NTT; encode_post_process marks
    // every 65536 of the first n_outputs rows at offset + j (the value stays)
    const bool sys = type == FecType::SYSTEMATIC;
    qi_plan* pl = sys ? plan_ : hplan();
    const unsigned rows = sys ? n_parities : n;
    const size_t size = words.get_size();
    if (words.get_n() < static_cast<int>(n_data) || output.get_n() < static_cast<int>(rows) ||
        output.get_size() < size || props.size() < n_outputs)
        throw std::invalid_argument("RsFnt::encode: buffer sizes");
    std::vector<std::vector<uint16_t>> in(n_data, std::vector<uint16_t>(size));
    std::vector<std::vector<uint16_t>> out(rows, std::vector<uint16_t>(size));
    for (unsigned i = 0; i < n_data; i++)
        for (size_t j = 0; j < size; j++) {
            const uint32_t v = words.get(static_cast<int>(i))[j];
            if (v > 65535u)
                throw std::invalid_argument("RsFnt::encode: data symbol >= 65536");
            in[i][j] = static_cast<uint16_t>(v);
        }
    std::vector<const uint8_t*> dp(n_data);
    std::vector<uint8_t*> op(rows);
    for (unsigned i = 0; i < n_data; i++)
        dp[i] = reinterpret_cast<const uint8_t*>(in[i].data());
    for (unsigned i = 0; i < rows; i++)
        op[i] = reinterpret_cast<uint8_t*>(out[i].data());
    std::vector<Properties> marks(rows);
    encode_columns(pl, dp.data(), op.data(), size, marks, 0);
    for (unsigned i = 0; i < rows; i++) {
        uint32_t* o = output.get(static_cast<int>(i));
        for (size_t j = 0; j < size; j++)
            o[j] = out[i][j];
        for (auto const& it : marks[i].get_map()) {
            o[it.first] = 65536u;
            if (i < n_outputs)
                props[i].add(static_cast<size_t>(offset) + it.first, OOR_MARK);
        }
    }
    n_encode_ops++;
}

std::unique_ptr<DecodeContext> RsFnt::init_context_dec(const vec::Vector& fragments_ids,
                                                       std::vector<Properties>& input_props,
                                                       size_t size)
{
    // src/fec_base.h:758-793 (the props are read by each decode call)
    (void)input_props;
    if (fragments_ids.size() < n_data)
        throw std::invalid_argument("RsFnt::init_context_dec: need n_data ids");
    vec::Vector ids(fragments_ids.begin(), fragments_ids.begin() + n_data);
    for (uint32_t id : ids)
        if (id >= n)
            throw std::invalid_argument("RsFnt::init_context_dec: fragment id >= n");
    return std::make_unique<DecodeContext>(ids, size);
}

void RsFnt::decode(DecodeContext& context, vec::Vector& output,
                   const std::vector<Properties>& props, off_t offset, vec::Vector& words)
{
    // decode_prepare (src/fec_base.h:799-820): a mark at `offset` on fragment
    // ids[i] restores words[i] = 65536; decode_apply (:829-878) interpolates
    // the n-point code: output = the k coefficients
    const vec::Vector& ids = context.get_fragments_id();
    if (words.size() < n_data || output.size() < n_data)
        throw std::invalid_argument("RsFnt::decode: vector sizes");
    std::vector<int> id(n_data);
    std::vector<uint16_t> in(n_data), out(n_data);
    std::vector<Properties> marks(n_data);
    std::vector<const uint8_t*> rows(n_data);
    std::vector<const Properties*> mp(n_data);
    std::vector<uint8_t*> op(n_data);
    // the device takes the received fragments in ascending id order (the
    // interpolation does not depend on the order)
    const std::vector<unsigned> ord = id_order(ids, n_data);
    for (unsigned i = 0; i < n_data; i++) {
        const unsigned r = ord[i];
        if (ids[r] < props.size() && marked_at(props[ids[r]], static_cast<size_t>(offset)))
            words[r] = 65536u;
    }
    for (unsigned i = 0; i < n_data; i++) {
        const unsigned r = ord[i];
        id[i] = static_cast<int>(ids[r]);
        in[i] = static_cast<uint16_t>(words[r] & 0xffffu);
        if (words[r] == 65536u)
            marks[i].add(0, OOR_MARK);
        rows[i] = reinterpret_cast<const uint8_t*>(&in[i]);
        mp[i] = &marks[i];
        op[i] = reinterpret_cast<uint8_t*>(&out[i]);
    }
    decode_columns(hplan(), id, rows, mp, op.data(), 1, 0);
    for (unsigned i = 0; i < n_data; i++)
        output[i] = out[i];
    n_decode_ops++;
}

void RsFnt::decode(DecodeContext& context, vec::Buffers& output,
                   const std::vector<Properties>& props, off_t offset, vec::Buffers& words)
{
    // decode_prepare (src/fec_base.h:1361-1404): the marks of the received
    // coded fragments (props by parity index) inside [offset, offset + size)
    // restore 65536; decode_apply (:1418-1448) + for systematic codes the
    // evaluation at r^t (:1336-1355): output = the k data rows
    const bool sys = type == FecType::SYSTEMATIC;
    const vec::Vector& ids = context.get_fragments_id();
    const size_t size = words.get_size();
    if (words.get_n() < static_cast<int>(n_data) || output.get_n() < static_cast<int>(n_data) ||
        output.get_size() < size)
        throw std::invalid_argument("RsFnt::decode: buffer sizes");
    std::vector<int> id(n_data);
    std::vector<std::vector<uint16_t>> in(n_data, std::vector<uint16_t>(size)),
        out(n_data, std::vector<uint16_t>(size));
    std::vector<Properties> marks(n_data);
    std::vector<const uint8_t*> rows(n_data);
    std::vector<const Properties*> mp(n_data);
    std::vector<uint8_t*> op(n_data);
    const std::vector<unsigned> ord = id_order(ids, n_data);
    for (unsigned i = 0; i < n_data; i++) {
        const unsigned r = ord[i];
        id[i] = static_cast<int>(ids[r]);
        uint32_t* w = words.get(static_cast<int>(r));
        if (!(sys && ids[r] < n_data)) {
            const size_t pi = sys ? ids[r] - n_data : ids[r];
            if (pi < props.size())
                // decode_prepare restores the marks in [offset, offset +
                // pkt_size) (src/fec_base.h:1372), which equals the Buffers'
                // size on the reference's own paths; here the window is the
                // Buffers' size: a Buffers wider than pkt_size keeps every
                // mark (the reference would drop those past pkt_size) and a
                // narrower one is never written past its end (deliberate
                // deviation)
                for (auto const& it : props[pi].get_map())
                    if (it.second == OOR_MARK && it.first >= static_cast<size_t>(offset) &&
                        it.first < static_cast<size_t>(offset) + size)
                        w[it.first - static_cast<size_t>(offset)] = 65536u;
        }
        for (size_t j = 0; j < size; j++) {
            in[i][j] = static_cast<uint16_t>(w[j] & 0xffffu);
            if (w[j] == 65536u)
                marks[i].add(j, OOR_MARK);
        }
        rows[i] = reinterpret_cast<const uint8_t*>(in[i].data());
        mp[i] = &marks[i];
        op[i] = reinterpret_cast<uint8_t*>(out[i].data());
    }
    decode_columns(plan_, id, rows, mp, op.data(), size, 0);
    for (unsigned i = 0; i < n_data; i++) {
        uint32_t* o = output.get(static_cast<int>(i));
        for (size_t j = 0; j < size; j++)
            o[j] = out[i][j];
    }
    n_decode_ops++;
}

// ----------------------------------------------------------------- RS-NF4

void nf4_marks_from_lanes(const Properties& lanes, unsigned g,
                          Properties& words)
{
    // encode_post_process (src/fec_rs_nf4.h:271-289): one mark per word,
    // bit c set when component c was 65536 (NF4::unpack, gf_nf4.h:421-446)
    words.clear();
    size_t cur = 0;
    uint32_t mask = 0;
    for (auto const& it : lanes.get_map()) {
        const size_t w = it.first / g;
        if (mask && w != cur) {
            words.add(cur, mask);
            mask = 0;
        }
        cur = w;
        mask |= 1u << (it.first % g);
    }
    if (mask)
        words.add(cur, mask);
}

void nf4_marks_to_lanes(const Properties& words, unsigned g, Properties& lanes)
{
    // decode_prepare (src/fec_rs_nf4.h:291-317): NF4::pack(a, flag) sets the
    // flagged components to 65536 (gf_nf4.h:372-383)
    lanes.clear();
    for (auto const& it : words.get_map())
        for (unsigned c = 0; c < g; c++)
            if ((it.second >> c) & 1u)
                lanes.add(it.first * g + c, OOR_MARK);
}

namespace {

unsigned nf4_word_size(unsigned ws)
{
    if (ws != 2 && ws != 4 && ws != 8)
        throw std::invalid_argument("RsNf4: word_size must be 2, 4 or 8");
    return ws;
}

}  // namespace

RsNf4::RsNf4(unsigned ws, unsigned k, unsigned m, size_t pkt)
    : word_size(nf4_word_size(ws)), n_data(k), n_parities(m), code_len(k + m),
      n_outputs(k + m), gf_n(ws / 2), pkt_size(pkt), buf_size(pkt * ws), n(0),
      lanes_(FecType::NON_SYSTEMATIC, 2, k, m, pkt * (ws / 2))
{
    n = lanes_.n;
}

void RsNf4::encode_blocks_vertical(std::vector<uint8_t*>& data_bufs,
                                   std::vector<uint8_t*>& parities_bufs,
                                   std::vector<Properties>& parities_props,
                                   std::vector<bool>& wanted_idxs,
                                   size_t block_size_bytes)
{
    std::vector<Properties> lp(n_outputs);
    lanes_.encode_blocks_vertical(data_bufs, parities_bufs, lp, wanted_idxs,
                                  block_size_bytes / word_size * word_size);
    for (unsigned i = 0; i < n_outputs; i++)
        nf4_marks_from_lanes(lp[i], gf_n, parities_props[i]);
}

bool RsNf4::decode_blocks_vertical(std::vector<uint8_t*>& data_bufs,
                                   std::vector<uint8_t*>& parities_bufs,
                                   std::vector<Properties>& parities_props,
                                   std::vector<int>& missing_idxs,
                                   std::vector<bool>& wanted_idxs,
                                   size_t block_size_bytes)
{
    std::vector<Properties> lp(n_outputs);
    for (unsigned i = 0; i < n_outputs; i++) {
        parities_props[i].sort();  // as DecodeContext (src/fec_context.h:93-97)
        nf4_marks_to_lanes(parities_props[i], gf_n, lp[i]);
    }
    return lanes_.decode_blocks_vertical(data_bufs, parities_bufs, lp,
                                         missing_idxs, wanted_idxs,
                                         block_size_bytes / word_size * word_size);
}

void RsNf4::encode_streams_vertical(
    const std::vector<std::istream*>& input_data_bufs,
    std::vector<std::ostream*>& output_parities_bufs,
    std::vector<Properties>& output_parities_props)
{
    std::vector<Properties> lp(n_outputs);
    lanes_.encode_streams_vertical(input_data_bufs, output_parities_bufs, lp);
    for (unsigned i = 0; i < n_outputs; i++)
        nf4_marks_from_lanes(lp[i], gf_n, output_parities_props[i]);
}

bool RsNf4::decode_streams_vertical(
    const std::vector<std::istream*>& input_data_bufs,
    const std::vector<std::istream*>& input_parities_bufs,
    std::vector<Properties>& input_parities_props,
    std::vector<std::ostream*>& output_data_bufs)
{
    std::vector<Properties> lp(n_outputs);
    for (unsigned i = 0; i < n_outputs; i++) {
        input_parities_props[i].sort();
        nf4_marks_to_lanes(input_parities_props[i], gf_n, lp[i]);
    }
    return lanes_.decode_streams_vertical(input_data_bufs, input_parities_bufs,
                                          lp, output_data_bufs);
}

}  // namespace fec
}  // namespace qi

// ---------------------------------------------------------------- C view

struct qi_fec {
    qi::fec::RsFnt* f;
};

extern "C" {

qi_fec* qi_fec_new(int systematic, int k, int m)
{
    try {
        auto* h = new qi_fec;
        h->f = new qi::fec::RsFnt(systematic ? qi::fec::FecType::SYSTEMATIC
                                             : qi::fec::FecType::NON_SYSTEMATIC,
                                  2, static_cast<unsigned>(k),
                                  static_cast<unsigned>(m), 1024);
        return h;
    } catch (...) {
        return nullptr;
    }
}

void qi_fec_delete(qi_fec* h)
{
    if (h) {
        delete h->f;
        delete h;
    }
}

int qi_fec_n_outputs(const qi_fec* h)
{
    return h ? static_cast<int>(h->f->n_outputs) : -1;
}

int qi_fec_encode_blocks(qi_fec* h, uint8_t** data, uint8_t** outputs,
                         size_t block_bytes, uint32_t* oor, uint32_t* oor_count,
                         uint32_t cap)
{
    try {
        qi::fec::RsFnt& f = *h->f;
        std::vector<uint8_t*> dv(data, data + f.n_data);
        std::vector<uint8_t*> pv(outputs, outputs + f.n_outputs);
        std::vector<qi::Properties> props(f.n_outputs);
        std::vector<bool> wanted(f.n_outputs);
        for (unsigned i = 0; i < f.n_outputs; i++)
            wanted[i] = outputs[i] != nullptr;
        f.encode_blocks_vertical(dv, pv, props, wanted, block_bytes);
        for (unsigned i = 0; i < f.n_outputs; i++) {
            uint32_t c = 0;
            for (auto const& it : props[i].get_map()) {
                if (c < cap)
                    oor[static_cast<size_t>(i) * cap + c] =
                        static_cast<uint32_t>(it.first);
                c++;
            }
            oor_count[i] = c;
        }
        return 0;
    } catch (...) {
        return -1;
    }
}

int qi_fec_decode_blocks(qi_fec* h, uint8_t** data, uint8_t** parities,
                         const uint32_t* oor, const uint32_t* oor_count,
                         uint32_t cap, const int* missing, const int* wanted,
                         size_t block_bytes)
{
    try {
        qi::fec::RsFnt& f = *h->f;
        std::vector<uint8_t*> dv(data, data + f.n_data);
        std::vector<uint8_t*> pv(parities, parities + f.n_outputs);
        std::vector<qi::Properties> props(f.n_outputs);
        for (unsigned i = 0; i < f.n_outputs; i++) {
            const uint32_t c = oor_count[i] < cap ? oor_count[i] : cap;
            for (uint32_t e = 0; e < c; e++)
                props[i].add(oor[static_cast<size_t>(i) * cap + e], qi::OOR_MARK);
        }
        std::vector<int> miss(missing, missing + f.code_len);
        std::vector<bool> want(f.n_data);
        for (unsigned i = 0; i < f.n_data; i++)
            want[i] = wanted[i] != 0;
        return f.decode_blocks_vertical(dv, pv, props, miss, want, block_bytes) ? 1
                                                                                : 0;
    } catch (...) {
        return -1;
    }
}

}  // extern "C"

namespace {

// std::streambuf over caller memory (no copies of its own) for the C view
// of the stream API
struct MemIn : std::streambuf {
    MemIn(const uint8_t* p, size_t n)
    {
        char* b = reinterpret_cast<char*>(const_cast<uint8_t*>(p));
        setg(b, b, b + n);
    }
};
struct MemOut : std::streambuf {
    MemOut(uint8_t* p, size_t n)
    {
        char* b = reinterpret_cast<char*>(p);
        setp(b, b + n);
    }
};

struct MemStreams {
    std::vector<std::unique_ptr<std::streambuf>> bufs;
    std::vector<std::unique_ptr<std::iostream>> streams;
    std::iostream* in(const uint8_t* p, size_t n)
    {
        if (!p)
            return nullptr;
        bufs.emplace_back(new MemIn(p, n));
        streams.emplace_back(new std::iostream(bufs.back().get()));
        return streams.back().get();
    }
    std::iostream* out(uint8_t* p, size_t n)
    {
        if (!p)
            return nullptr;
        bufs.emplace_back(new MemOut(p, n));
        streams.emplace_back(new std::iostream(bufs.back().get()));
        return streams.back().get();
    }
};

}  // namespace

extern "C" {

int qi_fec_encode_streams(qi_fec* h, const uint8_t** data, size_t bytes,
                          uint8_t** outputs, uint32_t* oor, uint32_t* oor_count,
                          uint32_t cap)
{
    try {
        qi::fec::RsFnt& f = *h->f;
        MemStreams ms;
        std::vector<std::istream*> in(f.n_data);
        std::vector<std::ostream*> out(f.n_outputs);
        for (unsigned i = 0; i < f.n_data; i++)
            if (!(in[i] = ms.in(data[i], bytes)))
                return -1;
        for (unsigned i = 0; i < f.n_outputs; i++)
            if (!(out[i] = ms.out(outputs[i], bytes)))
                return -1;
        std::vector<qi::Properties> props(f.n_outputs);
        f.encode_streams_vertical(in, out, props);
        for (unsigned i = 0; i < f.n_outputs; i++) {
            uint32_t c = 0;
            for (auto const& it : props[i].get_map()) {
                if (c < cap)
                    oor[static_cast<size_t>(i) * cap + c] =
                        static_cast<uint32_t>(it.first);
                c++;
            }
            oor_count[i] = c;
        }
        return 0;
    } catch (...) {
        return -1;
    }
}

int qi_fec_decode_streams(qi_fec* h, const uint8_t** data,
                          const uint8_t** parities, size_t bytes,
                          const uint32_t* oor, const uint32_t* oor_count,
                          uint32_t cap, uint8_t** out_data)
{
    try {
        qi::fec::RsFnt& f = *h->f;
        MemStreams ms;
        std::vector<std::istream*> din(f.n_data), pin(f.n_outputs);
        std::vector<std::ostream*> dout(f.n_data);
        for (unsigned i = 0; i < f.n_data; i++) {
            din[i] = ms.in(data ? data[i] : nullptr, bytes);
            dout[i] = ms.out(out_data[i], bytes);
        }
        std::vector<qi::Properties> props(f.n_outputs);
        for (unsigned i = 0; i < f.n_outputs; i++) {
            pin[i] = ms.in(parities[i], bytes);
            const uint32_t c = oor_count[i] < cap ? oor_count[i] : cap;
            for (uint32_t e = 0; e < c; e++)
                props[i].add(oor[static_cast<size_t>(i) * cap + e], qi::OOR_MARK);
        }
        return f.decode_streams_vertical(din, pin, props, dout) ? 1 : 0;
    } catch (...) {
        return -1;
    }
}

}  // extern "C"

struct qi_nf4 {
    qi::fec::RsNf4* f;
};

extern "C" {

qi_nf4* qi_nf4_new(int word_size, int k, int m)
{
    try {
        if (word_size < 0 || k < 1 || m < 1)
            return nullptr;
        auto* h = new qi_nf4;
        try {
            h->f = new qi::fec::RsNf4(static_cast<unsigned>(word_size),
                                      static_cast<unsigned>(k),
                                      static_cast<unsigned>(m), 1024);
        } catch (...) {
            delete h;
            return nullptr;
        }
        return h;
    } catch (...) {
        return nullptr;
    }
}

void qi_nf4_delete(qi_nf4* h)
{
    if (h) {
        delete h->f;
        delete h;
    }
}

int qi_nf4_n_outputs(const qi_nf4* h)
{
    return h ? static_cast<int>(h->f->n_outputs) : -1;
}

int qi_nf4_encode_blocks(qi_nf4* h, uint8_t** data, uint8_t** outputs,
                         size_t block_bytes, uint32_t* oor, uint32_t* flags,
                         uint32_t* oor_count, uint32_t cap)
{
    try {
        qi::fec::RsNf4& f = *h->f;
        std::vector<uint8_t*> dv(data, data + f.n_data);
        std::vector<uint8_t*> pv(outputs, outputs + f.n_outputs);
        std::vector<qi::Properties> props(f.n_outputs);
        std::vector<bool> wanted(f.n_outputs);
        for (unsigned i = 0; i < f.n_outputs; i++)
            wanted[i] = outputs[i] != nullptr;
        f.encode_blocks_vertical(dv, pv, props, wanted, block_bytes);
        for (unsigned i = 0; i < f.n_outputs; i++) {
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
        return 0;
    } catch (...) {
        return -1;
    }
}

int qi_nf4_decode_blocks(qi_nf4* h, uint8_t** data, uint8_t** parities,
                         const uint32_t* oor, const uint32_t* flags,
                         const uint32_t* oor_count, uint32_t cap,
                         const int* missing, const int* wanted,
                         size_t block_bytes)
{
    try {
        qi::fec::RsNf4& f = *h->f;
        std::vector<uint8_t*> dv(data, data + f.n_data);
        std::vector<uint8_t*> pv(parities, parities + f.n_outputs);
        std::vector<qi::Properties> props(f.n_outputs);
        for (unsigned i = 0; i < f.n_outputs; i++) {
            const uint32_t c = oor_count[i] < cap ? oor_count[i] : cap;
            for (uint32_t e = 0; e < c; e++)
                props[i].add(oor[static_cast<size_t>(i) * cap + e],
                             flags[static_cast<size_t>(i) * cap + e]);
        }
        std::vector<int> miss(missing, missing + f.code_len);
        std::vector<bool> want(f.n_data);
        for (unsigned i = 0; i < f.n_data; i++)
            want[i] = wanted[i] != 0;
        return f.decode_blocks_vertical(dv, pv, props, miss, want, block_bytes) ? 1
                                                                                : 0;
    } catch (...) {
        return -1;
    }
}

}  // extern "C"
