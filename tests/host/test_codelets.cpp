// Host-side checks of the device arithmetic (compiled by
// tests/test_host_math.py with g++ -fsanitize=signed-integer-overflow):
//  1. fold() range facts used by the kernels,
//  2. the planned NTT codelets dft<K, LO, HI> against an O(K^2) DFT, on
//     random inputs and on inputs pinned at the plan's range extremes (any
//     int32 overflow aborts under UBSan; 24-bit multiply operands are
//     asserted in mul_tw via QI_HOST_CHECK),
//  3. the dot2 matrix path (pack_row + emulated v_dot2_i32_i16) against a
//     plain matrix-vector product, checking the 32-bit accumulator bound,
//  4. the matrix-core path (pack_mf_dword operand tiles x byte planes, the
//     three int32 GEMMs of matrix_mfma_kernel and its epilogue) likewise.
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../quadiron_amd/csrc/fnt_codelets.h"
#include "../../quadiron_amd/csrc/matrix_pack.h"

using namespace qi;

static uint32_t canon64(long long x)
{
    long long r = x % 65537;
    return static_cast<uint32_t>(r < 0 ? r + 65537 : r);
}

static int fails = 0;
#define CHECK(c, ...)                                                        \
    do {                                                                     \
        if (!(c)) {                                                          \
            fails++;                                                         \
            if (fails < 20)                                                  \
                std::printf("FAIL %s:%d ", __FILE__, __LINE__),              \
                    std::printf(__VA_ARGS__), std::printf("\n");             \
        }                                                                    \
    } while (0)

static void test_fold(std::mt19937_64& g)
{
    // exhaustive over the documented input windows (sampled stride 1 near the
    // edges) and random over all int32
    auto chk = [&](long long x, long long lo, long long hi) {
        const int32_t f = fold(static_cast<int32_t>(x));
        CHECK(f >= lo && f <= hi, "fold(%lld)=%d not in [%lld,%lld]", x, f, lo, hi);
        CHECK(canon64(f) == canon64(x), "fold(%lld) not congruent", x);
    };
    for (long long x = -98305; x <= 163840; x++)
        chk(x, -2, 65537);
    for (long long x = -2; x <= 65537; x++)
        chk(x, -1, 65536);
    for (int i = 0; i < 2000000; i++) {
        const long long x = static_cast<int32_t>(g());
        chk(x, -32767, 98303);
    }
    chk(2147483647LL, -32767, 98303);
    chk(-2147483648LL, -32767, 98303);
    // fold_rng matches brute force on random windows
    for (int i = 0; i < 200; i++) {
        long long a = static_cast<int32_t>(g()) / (1 << (g() % 16));
        long long b = a + static_cast<long long>(g() % 300000);
        if (b > 2147483647LL)
            continue;
        Rng r = fold_rng(Rng{a, b});
        long long mn = 1LL << 40, mx = -(1LL << 40);
        for (long long x = a; x <= b; x++) {
            const long long f = fold(static_cast<int32_t>(x));
            mn = f < mn ? f : mn;
            mx = f > mx ? f : mx;
        }
        CHECK(mn == r.lo && mx == r.hi, "fold_rng [%lld,%lld]", a, b);
    }
}

template <int K, long long LO, long long HI>
static void test_dft(std::mt19937_64& g)
{
    const uint32_t w = root_of_unity(K);
    for (int trial = 0; trial < 400; trial++) {
        int32_t x[K];
        for (int i = 0; i < K; i++) {
            const int mode = trial < 200 ? static_cast<int>(g() % 3) : 2;
            const long long span = HI - LO + 1;
            x[i] = static_cast<int32_t>(mode == 0 ? LO : mode == 1 ? HI
                                        : LO + static_cast<long long>(g() % span));
        }
        int32_t y[K];
        for (int i = 0; i < K; i++)
            y[i] = x[i];
        dft<K, LO, HI>(y);
        for (int u = 0; u < K; u++) {
            long long acc = 0;
            uint32_t wp = 1, wu = powmod_c(w, static_cast<uint32_t>(u));
            for (int t = 0; t < K; t++) {
                acc = (acc + static_cast<long long>(canon64(x[t])) * wp) % 65537;
                wp = mulmod_c(wp, wu);
            }
            CHECK(y[u] >= -2 && y[u] <= 65537, "K=%d out of V: %d", K, y[u]);
            CHECK(canon64(y[u]) == static_cast<uint32_t>(acc), "K=%d u=%d", K, u);
        }
    }
    std::printf("dft<%d,[%lld,%lld]> folds=%d ok\n", K, LO, HI,
                plan_folds<K, LO, HI>());
}

static void test_matrix(std::mt19937_64& g)
{
    for (int kin : {1, 2, 3, 16, 33, 64, 128}) {
        const int KP = (kin + 1) / 2, R = kin;
        std::vector<uint32_t> M(static_cast<size_t>(R) * kin);
        for (auto& v : M) {
            const int mode = static_cast<int>(g() % 8);
            // force the residues that need row scaling
            v = mode == 0 ? 32767u + static_cast<uint32_t>(g() % 4)
                          : static_cast<uint32_t>(g() % 65537);
        }
        const MatLayout L{R, kin, KP};
        std::vector<int32_t> blk(L.words());
        for (int t = 0; t < R; t++)
            pack_row(M.data() + static_cast<size_t>(t) * kin, L, t, blk.data());
        for (int trial = 0; trial < 50; trial++) {
            std::vector<uint32_t> x(kin);
            for (auto& v : x)
                v = trial == 0 ? 0u : trial == 1 ? 65535u : static_cast<uint32_t>(g() % 65536);
            for (int t = 0; t < R; t++) {
                // device sequence: acc = kcorr; acc = fold(dot2(x', m, acc))
                long long acc = blk[static_cast<size_t>(R) * KP + t];
                for (int j = 0; j < KP; j++) {
                    const uint32_t pk = static_cast<uint32_t>(blk[static_cast<size_t>(t) * KP + j]);
                    const int16_t m0 = static_cast<int16_t>(pk & 0xffff);
                    const int16_t m1 = static_cast<int16_t>(pk >> 16);
                    const int16_t x0 = static_cast<int16_t>(
                        (2 * j < kin ? x[2 * j] : 0u) ^ 0x8000u);
                    const int16_t x1 = static_cast<int16_t>(
                        (2 * j + 1 < kin ? x[2 * j + 1] : 0u) ^ 0x8000u);
                    const long long s = acc + static_cast<long long>(x0) * m0 +
                                        static_cast<long long>(x1) * m1;
                    CHECK(s >= -2147483648LL && s <= 2147483647LL, "dot2 overflow");
                    acc = fold(static_cast<int32_t>(s));
                }
                int32_t y = fold(static_cast<int32_t>(acc));
                const int32_t rs = blk[static_cast<size_t>(R) * KP + R + t];
                if (rs != 1) {
                    const long long p = static_cast<long long>(y) * rs;
                    CHECK(p >= -2147483648LL && p <= 2147483647LL, "rscale overflow");
                    y = fold(fold(static_cast<int32_t>(p)));
                }
                long long ref = 0;
                for (int i = 0; i < kin; i++)
                    ref = (ref + static_cast<long long>(M[static_cast<size_t>(t) * kin + i]) * x[i]) % 65537;
                CHECK(y >= -1 && y <= 65536, "T range");
                CHECK(canon64(y) == static_cast<uint32_t>(ref), "matrix kin=%d t=%d", kin, t);
            }
        }
    }
    std::printf("matrix dot2 path ok\n");
}

static void test_matrix_mfma(std::mt19937_64& g)
{
    for (int kin : {1, 3, 16, 17, 33, 64, 65, 100, 128, 129, 200, 256, 300, 384, 385, 600, 640}) {
        for (int R : {kin, 48}) {
            int KP = 2;
            while (KP < (kin + 1) / 2)
                KP *= 2;
            const MatLayout L{R, kin, KP};
            if (!L.KS())
                continue;  // small blocks stay on the dot2 kernel
            std::vector<uint32_t> M(static_cast<size_t>(R) * kin);
            for (auto& v : M) {
                const int mode = static_cast<int>(g() % 8);
                // force the residues that need row scaling or sit at the
                // ends of the byte split
                v = mode == 0   ? 32640u
                    : mode == 1 ? 32767u + static_cast<uint32_t>(g() % 4)
                    : mode == 2 ? 65536u - static_cast<uint32_t>(g() % 300)
                                : static_cast<uint32_t>(g() % 65537);
            }
            std::vector<int32_t> blk(L.words());
            for (int t = 0; t < R; t++)
                pack_row(M.data() + static_cast<size_t>(t) * kin, L, t, blk.data());
            for (size_t d = 0; d < L.mf_words(); d++)
                blk[L.mf() + d] = pack_mf_dword(L, blk.data() + L.plain(), d);
            const int KS = L.KS(), KH = 16 * KS;
            auto opb = [&](int rb, int ks, int ty, int lane, int j) {
                const size_t dw = L.mf() +
                                  ((static_cast<size_t>(rb) * KS + ks) * 3 + ty) * 128 +
                                  static_cast<size_t>(lane) * 2 + j / 4;
                return static_cast<int>(static_cast<int8_t>(
                    static_cast<uint32_t>(blk[dw]) >> (8 * (j % 4))));
            };
            // the kernels rebuild [b | a] from the other two tiles at KS >= 2
            // (the contexts do not store it) and read single entries back
            // with mf_entry: both facts, for every dword and entry
            if (KS >= 2)
                for (int rb = 0; rb < L.RB(); rb++)
                    for (int ks = 0; ks < KS; ks++)
                        for (int lane = 0; lane < 64; lane++)
                            for (int j = 0; j < 8; j++) {
                                const int ba = opb(rb, ks, 2, lane, j);
                                const int from = ks < KS / 2 ? opb(rb, ks + KS / 2, 1, lane, j)
                                                             : opb(rb, ks - KS / 2, 0, lane, j);
                                CHECK(ba == from, "[b|a] kin=%d ks=%d lane=%d", kin, ks, lane);
                            }
            for (int t = 0; t < R; t++)
                for (int i = 0; i < kin; i++)
                    CHECK(mf_entry(L, blk.data() + L.mf(), t, i) ==
                              static_cast<uint32_t>(blk[L.plain() + static_cast<size_t>(t) * kin + i]),
                          "mf_entry kin=%d t=%d i=%d", kin, t, i);
            for (int trial = 0; trial < 30; trial++) {
                std::vector<uint32_t> x(kin);
                for (auto& v : x)
                    v = trial == 0 ? 0u : trial == 1 ? 65535u : static_cast<uint32_t>(g() % 65536);
                for (int t = 0; t < R; t++) {
                    const int rb = t / 16;
                    // device: acc1 starts at kmf[t]; rows past kin hold a
                    // clamped row (their operand bytes are 0)
                    long long D[3] = {0, blk[L.kmf() + t], 0};
                    for (int K = 0; K < 2 * KH; K++) {
                        const int ks = K / 32, gg = (K % 32) / 8, j = K % 8;
                        const int lane = 16 * gg + t % 16;
                        const int i = K < KH ? K : K - KH;
                        const uint32_t xi = x[i < kin ? i : kin - 1];
                        const int byte = K < KH ? static_cast<int>(xi >> 8) - 128
                                                : static_cast<int>(xi & 255) - 128;
                        for (int ty = 0; ty < 3; ty++)
                            D[ty] += static_cast<long long>(opb(rb, ks, ty, lane, j)) * byte;
                    }
                    for (long long d : D)
                        CHECK(d >= -2147483648LL && d <= 2147483647LL, "mfma acc overflow");
                    // KS >= 16 (k > 128): the device folds D2 before the shift (KS = 40:
                    // the two K chunks accumulate into the same D0, D1, D2)
                    const long long d2 = KS >= 16 ? fold(static_cast<int32_t>(D[2])) : D[2];
                    const long long v = d2 * 256 + D[1] - D[0];
                    CHECK(v >= -2147483648LL && v <= 2147483647LL, "mfma epilogue overflow");
                    int32_t y = fold(fold(static_cast<int32_t>(v)));
                    const int32_t rs = blk[L.rscale() + t];
                    if (rs != 1)
                        y = fold(fold(static_cast<int32_t>(static_cast<long long>(y) * rs)));
                    long long ref = 0;
                    for (int i = 0; i < kin; i++)
                        ref = (ref + static_cast<long long>(M[static_cast<size_t>(t) * kin + i]) * x[i]) % 65537;
                    CHECK(y >= -1 && y <= 65536, "mfma T range");
                    CHECK(canon64(y) == static_cast<uint32_t>(ref), "mfma kin=%d R=%d t=%d", kin, R, t);
                }
            }
        }
    }
    std::printf("matrix mfma path ok\n");
}

int main()
{
    std::mt19937_64 g(12345);
    test_fold(g);
    test_dft<1, 0, 65535>(g);
    test_dft<2, 0, 65535>(g);
    test_dft<4, 0, 65535>(g);
    test_dft<8, 0, 65535>(g);
    test_dft<16, 0, 65535>(g);
    test_dft<32, 0, 65535>(g);
    test_dft<64, 0, 65535>(g);
    test_dft<2, -32767, 98303>(g);
    test_dft<4, -32767, 98303>(g);
    test_dft<8, -32767, 98303>(g);
    test_dft<16, -32767, 98303>(g);
    test_dft<32, -32767, 98303>(g);
    test_dft<64, -32767, 98303>(g);
    test_matrix(g);
    test_matrix_mfma(g);
    if (fails) {
        std::printf("%d failures\n", fails);
        return 1;
    }
    std::printf("ALL OK\n");
    return 0;
}
