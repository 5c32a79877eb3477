// Packing of a canonical GF(65537) matrix into the forms the matrix kernels
// read (host + device): the int16-pair rows of the dot2 kernel
// (matrix_kernel) and the i8 operand tiles of the matrix-core kernel
// (matrix_mfma_kernel).
#pragma once

#include <stddef.h>

#include "gf65537.h"

namespace qi {

// Packed matrix block, one per stripe (decode contexts) or shared (plan):
//   packed[R][KP]  int16 pairs (balanced, |c| <= 32766) of the row-scaled
//                  matrix, zero padded past kin
//   kcorr[R]       32768 * sum_i c[t][i] mod q (undoes the x - 32768 offset)
//   rscale[R]      balanced inverse row scale (1 = unscaled)
//   plain[R][kin]  canonical row-scaled entries (OOR corrections)
//   mf[RB][KS][3][64][2]  i8 operand tiles of matrix_mfma_kernel (kin <= 256):
//                  RB = ceil(R / 16) output blocks, KS = K-steps of 32
//                  bytes, 3 operand types, 64 lanes x 8 bytes (pack_mf_dword)
//   kmf[R]         32896 * sum_i c[t][i] mod q (undoes the byte offsets)
//   rscale_mf[R]   the MFMA section's own inverse row scale: its tiles hold
//                  the rows scaled for the i8 split alone (only 32640 is out
//                  of its reach), so a shared generator's Vandermonde rows
//                  that hit +-2^15 need no scale there (decode contexts use
//                  one scale for both: rscale_mf = rscale)
// The MFMA section exists (KS() > 0) when matrix_mfma_kernel takes the
// block: kin <= 256.  |D2| <= 2 kin 128^2: up to k = 128 (2^22) 256 D2 +
// D1 - D0 stays inside int32; at KS = 16 the epilogue folds D2 first.
// A/B on MI355X, k = 16 decode: 1.54 ms on the matrix cores with the
// LDS-transposed streaming stores vs 1.62 ms dot2 (1.65 ms before the
// transpose); the 48 x 16 systematic encode 3.60 vs 3.80 ms and the 64 x 64
// decode 0.35 vs 0.62 ms.
// the largest k the matrix kernels take (256 < k <= 640: whole 1024-column
// tiles only, on the operand-stationary kernel; the NTT engine otherwise;
// 384 < k <= 640: the decodes and the systematic encodes, KS = 40 in two K
// chunks)
constexpr int kMatMaxKin = 640;
// the largest k of the non-systematic matrix-core encodes (KS <= 24)
constexpr int kMatGenMaxKin = 384;

struct MatLayout {
    int R, kin, KP;
    // K-steps of 32 bytes over the [h' ; l'] planes; past 256 inputs only
    // the operand-stationary kernel takes the matrix (KS a multiple of 4,
    // its double-buffered image <= 2 x 61 KB at KS = 24; KS = 40 stages its
    // image in two K chunks of 20 steps)
    QI_HD int KS() const
    {
        if (kin > kMatMaxKin)
            return 0;
        return kin <= 16 ? 1 : kin <= 32 ? 2 : kin <= 64 ? 4 : kin <= 128 ? 8
               : kin <= 256 ? 16 : kin <= 320 ? 20 : kin <= 384 ? 24 : 40;
    }
    QI_HD int RB() const { return KS() ? (R + 15) / 16 : 0; }
    QI_HD size_t packed() const { return 0; }
    QI_HD size_t kcorr() const { return static_cast<size_t>(R) * KP; }
    QI_HD size_t rscale() const { return kcorr() + R; }
    QI_HD size_t plain() const { return rscale() + R; }
    QI_HD size_t mf() const { return plain() + static_cast<size_t>(R) * kin; }
    QI_HD size_t mf_words() const
    {
        return static_cast<size_t>(RB()) * KS() * 3 * 128;
    }
    QI_HD size_t kmf() const { return mf() + mf_words(); }
    QI_HD size_t rscale_mf() const { return kmf() + (KS() ? R : 0); }
    QI_HD size_t words() const { return rscale_mf() + (KS() ? R : 0); }
};

QI_HD int32_t iabs32(int32_t v)
{
    return v < 0 ? -v : v;
}

// Coefficients both kernels can take: v_dot2_i32_i16 accumulates
// acc + x0*c0 + x1*c1 with x in [-32768, 32767] (inputs offset by -32768)
// and acc in [-32767, 98303] (after fold), which stays below 2^31 iff
// |c| <= 32766; the i8 split c = 256 a + b (split_i8) reaches every
// balanced residue but 32640.
QI_HD bool coef_ok(int32_t c)
{
    return iabs32(c) <= 32766 && c != 32640;
}

// Coefficients the i8 split alone can take (the matrix-core section).
QI_HD bool coef_mf_ok(int32_t c)
{
    return c != 32640;
}

// c = 256 a + b (mod q) with a, b in [-128, 127], for a canonical c whose
// balanced form is not 32640 (256 a + b spans [-32896, 32639])
QI_HD void split_i8(uint32_t c, int32_t& a, int32_t& b)
{
    int32_t v = balanced(c);
    if (v > 32639)
        v -= kQ;
    b = ((v + 128) & 255) - 128;
    a = (v - b) / 256;
}

// Pack row t (kin canonical entries) of the block.  Rows holding a
// coefficient that breaks coef_ok are scaled by a unit s first and the
// result is multiplied back by s^-1 (rscale, also |s^-1| <= 32766).
// Returns the row scale s (1 = unscaled).
QI_HD uint32_t pack_row(const uint32_t* row, const MatLayout& L, int t,
                        int32_t* block)
{
    const int kin = L.kin, KP = L.KP;
    // s = 1 almost always (a row needs scaling with probability ~ 5 kin /
    // 65537): test it without multiplications
    bool ok = true;
    for (int i = 0; i < kin && ok; i++)
        ok = coef_ok(balanced(row[i]));
    uint32_t s = 1;
    for (; !ok;) {
        s++;
        const int32_t si = balanced(powmod_c(s, 65535u));
        if (iabs32(si) > 32766)
            continue;
        ok = true;
        for (int i = 0; i < kin && ok; i++)
            ok = coef_ok(balanced(mulmod_c(row[i], s)));
    }
    int32_t* packed = block + static_cast<size_t>(t) * KP;
    int32_t* plain = block + L.plain();
    uint64_t sum = 0;
    for (int j = 0; j < KP; j++) {
        int32_t lo = 0, hi = 0;
        if (2 * j < kin)
            lo = balanced(mulmod_c(row[2 * j], s));
        if (2 * j + 1 < kin)
            hi = balanced(mulmod_c(row[2 * j + 1], s));
        packed[j] = static_cast<int32_t>((static_cast<uint32_t>(lo) & 0xffffu) |
                                         (static_cast<uint32_t>(hi) << 16));
    }
    for (int i = 0; i < kin; i++) {
        const uint32_t c = mulmod_c(row[i], s);
        plain[static_cast<size_t>(t) * kin + i] = static_cast<int32_t>(c);
        sum += c;
    }
    const uint32_t sq = static_cast<uint32_t>(sum % 65537u);
    block[L.kcorr() + t] = static_cast<int32_t>(mulmod_c(sq, 32768u));
    block[L.rscale() + t] = s == 1 ? 1 : balanced(powmod_c(s, 65535u));
    if (L.KS()) {
        block[L.kmf() + t] = static_cast<int32_t>(mulmod_c(sq, 32896u));
        block[L.rscale_mf() + t] = block[L.rscale() + t];
    }
    return s;
}

// Dword d of the MFMA operand tiles, from the `plain` rows pack_row wrote.
// Tile (rb, ks, ty) gives lane l = 16 g + (t & 15), t = 16 rb + (t & 15),
// the B operand bytes B[K][t], K = 32 ks + 8 g + j (j = 0..7 over its two
// dwords), where K < KH = 16 KS is byte plane h' of input K and K >= KH
// is plane l' of input K - KH (x = 256 h' + l' + 32896):
//   ty 0: [a | 0]   ty 1: [0 | b]   ty 2: [b | a]       (c = 256 a + b)
// i.e. D0 = sum a h', D1 = sum b l', D2 = sum (b h' + a l') and
// sum c x = 256 D2 + D1 - D0 + 32896 sum c  (2^16 = -1 mod q).
// `rows`: the row-scaled canonical entries, kin per row (the block's
// `plain` section, or a copy of it in LDS).
QI_HD int32_t pack_mf_dword(const MatLayout& L, const int32_t* rows, size_t d)
{
    const int KS = L.KS(), KH = 16 * KS;  // KS is 1, 2, 4, 8, 16, 20, 24 or 40
    const int tile = static_cast<int>(d >> 7);
    const int rem = static_cast<int>(d & 127), lane = rem >> 1, dw = rem & 1;
    const int ty = tile % 3, rk = tile / 3;
    const int ks = rk % KS, rb = rk / KS;
    const int t = 16 * rb + (lane & 15), g = lane >> 4;
    if (t >= L.R)
        return 0;
    const int32_t* plain = rows + static_cast<size_t>(t) * L.kin;
    uint32_t v = 0;
    for (int jb = 0; jb < 4; jb++) {
        const int K = 32 * ks + 8 * g + 4 * dw + jb;
        const bool hp = K < KH;
        const int i = hp ? K : K - KH;
        int32_t e = 0;
        if (i < L.kin) {
            int32_t a, b;
            split_i8(static_cast<uint32_t>(plain[i]), a, b);
            e = ty == 0 ? (hp ? a : 0) : ty == 1 ? (hp ? 0 : b) : (hp ? b : a);
        }
        v |= (static_cast<uint32_t>(e) & 0xffu) << (8 * jb);
    }
    return static_cast<int32_t>(v);
}

// Entry (t, i) of the row-scaled matrix read back from its operand tiles
// (pack_mf_dword's layout): a from [a | 0] at K = i, b from [0 | b] at
// K = KH + i; 256 a + b, canonical.  The decode paths that need single
// coefficients (the OOR restore of the redo kernel, the dot2 sections
// filled on demand) take them from here, so a context built for whole-tile
// widths holds the matrix only once, as tiles -- and at KS >= 2 without
// its [b | a] tiles, which repeat those two (the kernels rebuild them).
QI_HD uint32_t mf_entry(const MatLayout& L, const int32_t* mf, int t, int i)
{
    const int KS = L.KS(), KH = 16 * KS;
    int32_t e[2];
    for (int h = 0; h < 2; h++) {
        const int K = h ? KH + i : i;
        const int ks = K >> 5, g = (K & 31) >> 3, dw = (K >> 2) & 1, jb = K & 3;
        const size_t d = (static_cast<size_t>((t >> 4) * KS + ks) * 3 + h) * 128 +
                         static_cast<size_t>((16 * g + (t & 15)) * 2 + dw);
        e[h] = static_cast<int8_t>(static_cast<uint32_t>(mf[d]) >> (8 * jb));
    }
    const int32_t c = 256 * e[0] + e[1];
    return static_cast<uint32_t>(c < 0 ? c + kQ : c);
}

}  // namespace qi
