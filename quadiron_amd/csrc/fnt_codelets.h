// Register-resident radix-2 NTT codelets over GF(65537), host + device.
//
// dft<K, LO, HI>(y): in-place natural-order K-point forward transform
//     y[u] <- sum_t y[t] * wK^(u t),   wK = 3^(65536/K)
// as a decimation-in-time radix-2 network (the butterfly of
// src/fft_2n.h:293-316: (a, b) -> (a + r b, a - r b)), fully unrolled with
// compile-time twiddles; the bit-reversal is a compile-time register
// renaming.  Inputs lie in [LO, HI]; outputs lie in V = [-2, 65537].
//
// Lazy reduction.  A constexpr *plan* runs interval arithmetic over the whole
// network at compile time and decides, per butterfly, how many folds
// (gf65537.h) each operand needs before its multiply or add so that no
// int32 product/sum can overflow and every v_mul_i32_i24 operand fits 24
// bits -- and, per output, whether to fold eagerly.  Several eagerness
// thresholds are simulated and the plan with the fewest folds is kept.  The
// plan is exact interval arithmetic, so it is safe for every input in range
// (tests/test_host_math.py also runs the codelets on the host with a checked
// integer type at the range extremes).
#pragma once

#include <utility>

#include "gf65537.h"

namespace qi {

struct Rng {
    long long lo, hi;
};

constexpr long long fdiv65536(long long a)
{
    return a >= 0 ? a / 65536 : -((-a + 65535) / 65536);
}

constexpr long long lmin(long long a, long long b) { return a < b ? a : b; }
constexpr long long lmax(long long a, long long b) { return a > b ? a : b; }
constexpr long long labs_(long long a) { return a < 0 ? -a : a; }

// exact image of fold() over [lo, hi]
constexpr Rng fold_rng(Rng r)
{
    const long long hl = fdiv65536(r.lo), hh = fdiv65536(r.hi);
    if (hl == hh)
        return {r.lo - hl * 65537, r.hi - hh * 65537};
    return {lmin(r.lo - hl * 65537, -hh), lmax(65535 - hl, r.hi - hh * 65537)};
}

constexpr long long kI32Max = 2147483647LL, kI32Min = -2147483648LL;

constexpr bool fits32(Rng r) { return r.lo >= kI32Min && r.hi <= kI32Max; }
constexpr long long mag(Rng r) { return lmax(labs_(r.lo), labs_(r.hi)); }

// v_mul_i32_i24 by constant c: |x| < 2^23 and |x*c| < 2^31
constexpr bool mul_ok(Rng r, long long c)
{
    return mag(r) < (1LL << 23) && mag(r) * labs_(c) <= kI32Max;
}

constexpr Rng mul_rng(Rng r, long long c)
{
    return {lmin(r.lo * c, r.hi * c), lmax(r.lo * c, r.hi * c)};
}

constexpr Rng add_rng(Rng a, Rng b) { return {a.lo + b.lo, a.hi + b.hi}; }
constexpr Rng sub_rng(Rng a, Rng b) { return {a.lo - b.hi, a.hi - b.lo}; }
constexpr Rng join(Rng a, Rng b) { return {lmin(a.lo, b.lo), lmax(a.hi, b.hi)}; }
constexpr bool in_v(Rng r) { return r.lo >= -2 && r.hi <= 65537; }

constexpr int kMaxL = 6;  // K <= 64

struct DftPlan {
    int folds = 0;              // total fold count (the plan's cost)
    signed char fa[kMaxL][32];  // pre-folds of operand a per butterfly
    signed char fb[kMaxL][32];  // pre-folds of operand b
    signed char fo[kMaxL][32][2];  // eager folds of the two outputs
    signed char fout[64];       // final folds into V
};

// twiddle of butterfly (stage s, index B) and its operands
struct Bf {
    int a, b;
    uint32_t c;
};

constexpr Bf bf_at(int K, int s, int B)
{
    const int m = 1 << s;
    int idx = 0;
    for (int j = 0; j < m; j++)
        for (int i = j; i < K; i += 2 * m) {
            if (idx == B)
                return {i, i + m, powmod_c(root_of_unity(static_cast<uint32_t>(K)),
                                           static_cast<uint32_t>(j * (K / (2 * m))))};
            idx++;
        }
    return {0, 0, 1};
}

// t = x * c for a twiddle c (mirrors mul_tw in gf65537.h)
constexpr long long mul_factor(uint32_t c)
{
    const long long cb = balanced(c);
    return (cb == 32768 || cb == -32768) ? cb / 2 : cb;
}

constexpr Rng tw_rng(Rng b, uint32_t c)
{
    const long long cb = balanced(c);
    if (cb == 32768 || cb == -32768) {
        Rng t = fold_rng(mul_rng(b, cb / 2));
        return fold_rng({2 * t.lo, 2 * t.hi});
    }
    return fold_rng(mul_rng(b, cb));
}

constexpr DftPlan make_plan(int K, Rng rin, long long eager)
{
    DftPlan P{};
    Rng r[64] = {};
    for (int i = 0; i < K; i++)
        r[i] = rin;
    int L = 0;
    while ((1 << L) < K)
        L++;
    for (int s = 0; s < L; s++) {
        for (int B = 0; B < K / 2; B++) {
            const Bf f = bf_at(K, s, B);
            Rng ra = r[f.a], rb = r[f.b];
            int fa = 0, fb = 0;
            Rng o0{}, o1{};
            if (f.c == 1u || f.c == 65536u) {
                while (!fits32(add_rng(ra, rb)) || !fits32(sub_rng(ra, rb))) {
                    if (mag(ra) >= mag(rb)) {
                        ra = fold_rng(ra);
                        fa++;
                    } else {
                        rb = fold_rng(rb);
                        fb++;
                    }
                }
                o0 = f.c == 1u ? add_rng(ra, rb) : sub_rng(ra, rb);
                o1 = f.c == 1u ? sub_rng(ra, rb) : add_rng(ra, rb);
            } else {
                while (!mul_ok(rb, mul_factor(f.c))) {
                    rb = fold_rng(rb);
                    fb++;
                }
                const Rng t = tw_rng(rb, f.c);
                while (!fits32(add_rng(ra, t)) || !fits32(sub_rng(ra, t))) {
                    ra = fold_rng(ra);
                    fa++;
                }
                o0 = add_rng(ra, t);
                o1 = sub_rng(ra, t);
            }
            int e0 = 0, e1 = 0;
            while (mag(o0) > eager) {
                o0 = fold_rng(o0);
                e0++;
            }
            while (mag(o1) > eager) {
                o1 = fold_rng(o1);
                e1++;
            }
            P.fa[s][B] = static_cast<signed char>(fa);
            P.fb[s][B] = static_cast<signed char>(fb);
            P.fo[s][B][0] = static_cast<signed char>(e0);
            P.fo[s][B][1] = static_cast<signed char>(e1);
            P.folds += fa + fb + e0 + e1;
            r[f.a] = o0;
            r[f.b] = o1;
        }
    }
    for (int i = 0; i < K; i++) {
        int n = 0;
        while (!in_v(r[i])) {
            r[i] = fold_rng(r[i]);
            n++;
        }
        P.fout[i] = static_cast<signed char>(n);
        P.folds += n;
    }
    return P;
}

constexpr DftPlan best_plan(int K, Rng rin)
{
    constexpr long long cand[] = {65537,     98303,     131072,    163840,
                                  262144,    524288,    1LL << 20, 1LL << 22,
                                  1LL << 24, 1LL << 26, 1LL << 28, kI32Max};
    DftPlan best = make_plan(K, rin, cand[0]);
    for (long long e : cand) {
        const DftPlan p = make_plan(K, rin, e);
        if (p.folds < best.folds)
            best = p;
    }
    return best;
}

template <int K, long long LO, long long HI>
struct PlanHolder {
    static constexpr DftPlan P = best_plan(K, Rng{LO, HI});
};

template <int N>
QI_HD int32_t fold_n(int32_t x)
{
    if constexpr (N <= 0)
        return x;
    else
        return fold_n<N - 1>(fold(x));
}

template <int K, long long LO, long long HI, int S, int B>
QI_HD void bfly_at(int32_t* y)
{
    constexpr const DftPlan& P = PlanHolder<K, LO, HI>::P;
    constexpr Bf f = bf_at(K, S, B);
    const int32_t a = fold_n<P.fa[S][B]>(y[f.a]);
    const int32_t b = fold_n<P.fb[S][B]>(y[f.b]);
    int32_t o0, o1;
    if constexpr (f.c == 1u) {
        o0 = a + b;
        o1 = a - b;
    } else if constexpr (f.c == 65536u) {
        o0 = a - b;
        o1 = a + b;
    } else {
        const int32_t t = mul_tw<f.c>(b);
        o0 = a + t;
        o1 = a - t;
    }
    y[f.a] = fold_n<P.fo[S][B][0]>(o0);
    y[f.b] = fold_n<P.fo[S][B][1]>(o1);
}

template <int K, long long LO, long long HI, int S, int... B>
QI_HD void dit_stage(int32_t* y, std::integer_sequence<int, B...>)
{
    (bfly_at<K, LO, HI, S, B>(y), ...);
}

template <int K, long long LO, long long HI, int... S>
QI_HD void dit_all(int32_t* y, std::integer_sequence<int, S...>)
{
    (dit_stage<K, LO, HI, S>(y, std::make_integer_sequence<int, K / 2>{}), ...);
}

template <int K, long long LO, long long HI, int... I>
QI_HD void fold_outputs(int32_t* y, std::integer_sequence<int, I...>)
{
    constexpr const DftPlan& P = PlanHolder<K, LO, HI>::P;
    ((y[I] = fold_n<P.fout[I]>(y[I])), ...);
}

// natural-order K-point transform; inputs in [LO, HI], outputs in V
template <int K, long long LO, long long HI>
QI_HD void dft(int32_t* x)
{
    constexpr int L = ilog2c(K);
    int32_t y[K];
#pragma unroll
    for (int i = 0; i < K; i++)
        y[bitrev_c(static_cast<uint32_t>(i), L)] = x[i];
    dit_all<K, LO, HI>(y, std::make_integer_sequence<int, L>{});
    fold_outputs<K, LO, HI>(y, std::make_integer_sequence<int, K>{});
#pragma unroll
    for (int i = 0; i < K; i++)
        x[i] = y[i];
}

// fold count of the chosen plan (for reports/tests)
template <int K, long long LO, long long HI>
constexpr int plan_folds()
{
    return PlanHolder<K, LO, HI>::P.folds;
}

}  // namespace qi
