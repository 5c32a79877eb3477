// Packing of a canonical GF(65537) matrix row into the dot2 form used by the
// matrix kernel (host + device).  See qi_internal.h MatLayout.
#pragma once

#include "gf65537.h"

namespace qi {

QI_HD int32_t iabs32(int32_t v)
{
    return v < 0 ? -v : v;
}

// Pack row t (kin canonical entries) of an R-row block with KP pairs.
// v_dot2_i32_i16 accumulates acc + x0*c0 + x1*c1 with x in [-32768, 32767]
// (inputs offset by -32768) and acc in [-32767, 98303] (after fold): the sum
// stays below 2^31 iff |c| <= 32766, so rows holding one of the 4 residues
// {32767, 32768, 32769, 32770} are scaled by a unit s first and the result
// is multiplied back by s^-1 (also kept within |c| <= 32766).
QI_HD void pack_row(const uint32_t* row, int kin, int KP, int R, int t,
                    int32_t* block)
{
    uint32_t s = 1;
    for (;; s++) {
        const int32_t si = balanced(powmod_c(s, 65535u));
        if (iabs32(si) > 32766)
            continue;
        bool ok = true;
        for (int i = 0; i < kin; i++) {
            const int32_t c = balanced(mulmod_c(row[i], s));
            if (iabs32(c) > 32766) {
                ok = false;
                break;
            }
        }
        if (ok)
            break;
    }
    int32_t* packed = block + static_cast<size_t>(t) * KP;
    int32_t* kcorr = block + static_cast<size_t>(R) * KP;
    int32_t* rscale = kcorr + R;
    int32_t* plain = rscale + R;
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
    kcorr[t] = static_cast<int32_t>(mulmod_c(static_cast<uint32_t>(sum % 65537u), 32768u));
    rscale[t] = balanced(powmod_c(s, 65535u));
}

}  // namespace qi
