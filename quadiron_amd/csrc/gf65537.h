// GF(65537) arithmetic for the RS-FNT engine, host + device.
//
// Values live in 32-bit signed registers in *lazy* form: any int32 congruent
// to the residue.  The one reduction primitive is
//
//     fold(x) = (x & 0xffff) - (x >> 16)          (x = hi*2^16 + lo, 2^16 == -1)
//
// which gfx950 executes as ONE `v_sub_u32_sdwa` (src0 WORD_0, src1 WORD_1
// sext).  Range facts used by the kernels (checked exhaustively on the host in
// tests/test_host_math.py):
//   |x| < 2^31          -> fold(x) in [-32767, 98303]
//   x in [-98305,163840] -> fold(x) in [-2, 65537]        ("V" range)
//   x in [-2, 65537]     -> fold(x) in [-1, 65536]        ("T" range)
// T-range values are canonical except -1 and 65536, which both mean 65536
// (the out-of-range symbol of src/fec_rs_fnt.h:253-269).
//
// Constant multiplies use v_mul_i32_i24 with the *balanced* representative
// c in [-32768, 32768]; the callers guarantee |x * c| < 2^31.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define QI_HD __host__ __device__ __forceinline__
#else
#define QI_HD inline
#endif

#if defined(QI_HOST_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
#include <cassert>
// host test builds: v_mul_i32_i24 operands must fit 24 bits
#define QI_ASSERT24(x) assert((x) > -(1 << 23) && (x) < (1 << 23))
#else
#define QI_ASSERT24(x) ((void)0)
#endif

namespace qi {

constexpr int32_t kQ = 65537;

QI_HD int32_t fold(int32_t x)
{
    return (x & 0xffff) - (x >> 16);
}

// balanced representative of a canonical residue
constexpr int32_t balanced(uint32_t c)
{
    return c > 32768u ? static_cast<int32_t>(c) - kQ : static_cast<int32_t>(c);
}

// canonical [0, q) residue of any int32 value (host side helper; slow path)
QI_HD uint32_t canon(int64_t x)
{
    int64_t r = x % kQ;
    return static_cast<uint32_t>(r < 0 ? r + kQ : r);
}

// a * b mod q for a, b in [0, 65536]: with 2^16 = -1 and 2^32 = 1 the
// product p0 + p1 2^16 + p2 2^32 reduces to p0 - p1 + p2 (no 64-bit modulo,
// which is a long software sequence on the GPU)
constexpr uint32_t mulmod_c(uint32_t a, uint32_t b)
{
    const uint64_t p = static_cast<uint64_t>(a % 65537u) * (b % 65537u);
    const int32_t v = static_cast<int32_t>(p & 0xffffu) -
                      static_cast<int32_t>((p >> 16) & 0xffffu) +
                      static_cast<int32_t>(p >> 32);  // [-65535, 65536]
    return static_cast<uint32_t>(v < 0 ? v + 65537 : v);
}

constexpr uint32_t powmod_c(uint32_t a, uint32_t e)
{
    uint32_t r = 1;
    a %= 65537u;
    while (e) {
        if (e & 1u)
            r = mulmod_c(r, a);
        a = mulmod_c(a, a);
        e >>= 1;
    }
    return r;
}

constexpr uint32_t invmod_c(uint32_t a)
{
    return powmod_c(a, 65535u);
}

// principal n-th root of unity for n | 65536: 3^(65536/n)
// (primitive root 3, src/gf_ring.h:624-660, :774-781)
constexpr uint32_t root_of_unity(uint32_t n)
{
    return powmod_c(3u, 65536u / n);
}

constexpr uint32_t ceil2(uint32_t n)
{
    uint32_t x = 1;
    while (x < n)
        x <<= 1;
    return x;
}

constexpr int ilog2c(uint32_t n)
{
    int l = 0;
    while ((1u << l) < n)
        l++;
    return l;
}

constexpr uint32_t bitrev_c(uint32_t i, int bits)
{
    uint32_t r = 0;
    for (int b = 0; b < bits; b++)
        r |= ((i >> b) & 1u) << (bits - 1 - b);
    return r;
}

// 24-bit sign-extension: tells the compiler a value fits v_mul_i32_i24
QI_HD int32_t sext24(int32_t c)
{
    return static_cast<int32_t>(static_cast<uint32_t>(c) << 8) >> 8;
}

// x * cb for a compile-time constant as ONE v_mul_i32_i24 with the constant
// in an SGPR.  The constant is passed through an opaque s_mov so the
// compiler cannot strength-reduce a power-of-two twiddle into shift/and/ashr
// sequences, which would also defeat the single SDWA v_sub of the following
// fold (4 VALU instead of 2).  The s_mov is CSE'd/hoisted (SALU, no VALU).
//
// The multiply itself is also written out: the callers' interval plans
// guarantee |x| < 2^23, but the compiler's own range analysis cannot follow
// lazily reduced sums and fell back to the quarter-rate v_mul_lo_u32 for
// ~20 of the ~150 twiddle multiplies of a 64-point pass.
template <int32_t CB>
QI_HD int32_t mul_const(int32_t x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    int32_t c, r;
    asm("s_mov_b32 %0, %1" : "=s"(c) : "i"(CB));
    asm("v_mul_i32_i24 %0, %1, %2" : "=v"(r) : "s"(c), "v"(x));
    return r;
#else
    return x * CB;
#endif
}

// x * c for a wave-uniform runtime constant c; the caller guarantees |x|,
// |c| < 2^23 and |x*c| < 2^31 (the sign-extension lets the compiler use
// v_mul_i32_i24 instead of the quarter-rate v_mul_lo_u32).
QI_HD int32_t mul_i24_s(int32_t x, int32_t c)
{
    return x * sext24(c);
}

// (w & 0xffff) * c and (w >> 16) * c for a packed pair of u16 columns w and
// a wave-uniform |c| <= 2^15: one SDWA v_mul_i32_i24 each (the 16-bit
// half is zero-extended by the operand select, no unpack instruction)
QI_HD int32_t mul_i24_lo16(uint32_t w, int32_t c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    int32_t r;
    asm("v_mul_i32_i24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 "
        "src1_sel:DWORD"
        : "=v"(r)
        : "v"(w), "s"(c));
    return r;
#else
    return static_cast<int32_t>(w & 0xffffu) * c;
#endif
}
QI_HD int32_t mul_i24_hi16(uint32_t w, int32_t c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    int32_t r;
    asm("v_mul_i32_i24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 "
        "src1_sel:DWORD"
        : "=v"(r)
        : "v"(w), "s"(c));
    return r;
#else
    return static_cast<int32_t>(w >> 16) * c;
#endif
}

// x * c for a compile-time canonical twiddle c, x in V = [-2, 65537].
// Result congruent to x*c, range [-32767, 98303] (or T-range pieces for the
// trivial cases).
template <uint32_t C>
QI_HD int32_t mul_tw(int32_t x)
{
    constexpr int32_t cb = balanced(C);
    QI_ASSERT24(x);
    if constexpr (C == 1u) {
        return x;
    } else if constexpr (cb == 32768 || cb == -32768) {
        // |x * 2^15| may reach 2^31: multiply by half, fold, double.
        // 2*fold(x*cb/2) in [-65534, 196606] -> fold again -> V.
        return fold(2 * fold(mul_const<cb / 2>(x)));
    } else {
        return fold(mul_const<cb>(x));
    }
}

// runtime-constant multiply, x in [0, 65535] (raw data), |c| <= 32768:
// |x*c| <= 2^31 - 2^15.  Result in T-range after the second fold.
QI_HD int32_t mul_data(int32_t x, int32_t cb)
{
    return fold(fold(x * cb));
}

}  // namespace qi
