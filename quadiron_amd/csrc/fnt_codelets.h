// Register-resident radix-2 NTT codelets over GF(65537), host + device.
//
// dft<K>(y): in-place natural-order K-point forward transform
//     y[u] <- sum_t y[t] * wK^(u t),   wK = 3^(65536/K)
// as a decimation-in-time radix-2 network (the butterfly of
// src/fft_2n.h:293-316: (a, b) -> (a + r b, a - r b)), fully unrolled with
// compile-time twiddles.  Every value stays in a VGPR; the bit-reversal is a
// compile-time register renaming.
//
// Range contract (see gf65537.h): inputs in V = [-2, 65537], outputs in V.
#pragma once

#include "gf65537.h"

namespace qi {

template <uint32_t C>
QI_HD void bfly(int32_t& a, int32_t& b)
{
    if constexpr (C == 1u) {
        const int32_t s = a + b, d = a - b;
        a = fold(s);
        b = fold(d);
    } else if constexpr (C == 65536u) {
        const int32_t s = a - b, d = a + b;
        a = fold(s);
        b = fold(d);
    } else {
        const int32_t t = mul_tw<C>(b);
        const int32_t s = a + t, d = a - t;
        a = fold(s);
        b = fold(d);
    }
}

template <int K, int M, int J>
QI_HD void dit_stage(int32_t* y)
{
    if constexpr (M < K) {
        if constexpr (J < M) {
            constexpr uint32_t C =
                powmod_c(root_of_unity(K), static_cast<uint32_t>(J * (K / (2 * M))));
#pragma unroll
            for (int i = J; i < K; i += 2 * M)
                bfly<C>(y[i], y[i + M]);
            dit_stage<K, M, J + 1>(y);
        } else {
            dit_stage<K, 2 * M, 0>(y);
        }
    }
}

template <int K>
QI_HD void dft(int32_t* x)
{
    constexpr int L = ilog2c(K);
    int32_t y[K];
#pragma unroll
    for (int i = 0; i < K; i++)
        y[bitrev_c(static_cast<uint32_t>(i), L)] = x[i];
    dit_stage<K, 1, 0>(y);
#pragma unroll
    for (int i = 0; i < K; i++)
        x[i] = y[i];
}

}  // namespace qi
