"""CPU: the index math of the general-path LDS engine (quadiron_amd/csrc/
ntt.hip, ntt_lds_kernel), emulated in Python with exact modular arithmetic.

The kernel runs forward transforms as decimation in frequency (natural order
in, X[j] at pos(j) out) and inverse transforms as the transposed passes in
reverse order (input at pos(t), natural order out), with per-pass twiddle
tables laid out [j][u].  These tests mirror xf_plan / xf_pos / xf_index /
lds_tables / lds_pass and check them against direct DFTs and against the
decode pipeline of FecCode::decode_apply (reference src/fec_base.h:1418-1448):
INTT_n -> NTT_2k -> x C -> INTT_2k.  The GPU parity tests then pin the
kernel itself to the reference's golden vectors."""
import random

import pytest

Q = 65537


def root(n):
    return pow(3, 65536 // n, Q)  # src/gf_ring.h:774-781 (primitive root 3)


def xf_plan(N):
    """ntt.hip xf_plan: radices <= 32, as even as possible; (lgr, sh) per
    pass with s_q = N / (R_0 ... R_q) = 2^sh_q."""
    bits = N.bit_length() - 1
    np_ = max(1, (bits + 4) // 5)
    lgr, sh, left, s = [], [], bits, bits
    for q in range(np_):
        b = (left + (np_ - q) - 1) // (np_ - q)
        lgr.append(b)
        s -= b
        sh.append(s)
        left -= b
    return lgr, sh


def prow(p):
    """ntt.hip prow: the image row of position p (one empty row per 32)."""
    return p + (p >> 5)


def xf_pos(plan, t):
    lgr, sh = plan
    p = 0
    for b, s in zip(lgr, sh):
        p += (t & ((1 << b) - 1)) << s
        t >>= b
    return p


def xf_index(plan, p):
    lgr, sh = plan
    t, b0 = 0, 0
    for b, s in zip(lgr, sh):
        t += ((p >> s) & ((1 << b) - 1)) << b0
        b0 += b
    return t


def tables(plan, nmax, inverse):
    """lds_tables: pass q holds w_L^{+-j u} at j R + u (w_L = w_nmax^(nmax/L))."""
    w = root(nmax)
    out = []
    for b, s in zip(*plan):
        R, sq = 1 << b, 1 << s
        L = R * sq
        wl = pow(w, nmax // L, Q)
        if inverse:
            wl = pow(wl, Q - 2, Q)
        out.append([pow(wl, (j * u) % L, Q) for j in range(sq) for u in range(R)])
    return out


def dft_r(v, inverse):
    R = len(v)
    wr = root(R)
    o = [sum(v[t] * pow(wr, u * t, Q) for t in range(R)) % Q for u in range(R)]
    return [o[(R - u) % R] for u in range(R)] if inverse else o


def lds_transform(buf, N, plan, tabs, dif, inverse):
    """lds_pass over every task, passes in order (DIF) or reversed (DIT)."""
    lgr, sh = plan
    order = range(len(lgr)) if dif else reversed(range(len(lgr)))
    for q in order:
        R, s = 1 << lgr[q], 1 << sh[q]
        L = R * s
        tw = tabs[q]
        for tt in range(N // R):
            j = tt & (s - 1)
            base = (tt // s) * L + j
            v = [buf[base + q2 * s] for q2 in range(R)]
            w = tw[j * R:(j + 1) * R]
            if not dif:
                v = [v[i] * w[i] % Q for i in range(R)]
            v = dft_r(v, inverse)
            if dif:
                v = [v[u] * w[u] % Q for u in range(R)]
            for u in range(R):
                buf[base + u * s] = v[u]


@pytest.mark.parametrize("N", [2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048])
def test_plan_shapes(N):
    lgr, sh = xf_plan(N)
    assert sum(lgr) == N.bit_length() - 1 and max(lgr) <= 5 and sh[-1] == 0
    assert sorted(xf_pos((lgr, sh), t) for t in range(N)) == list(range(N))
    assert all(xf_index((lgr, sh), xf_pos((lgr, sh), t)) == t for t in range(N))


@pytest.mark.parametrize("N", [32, 64, 128, 256, 512, 1024, 2048])
def test_image_rows_and_banks(N):
    """lds_pass_body addresses element q of task (b, j) as prow(b + j) +
    prow(q s): exact for every pass of the plan (no carry into bit 5).  And
    where the unit pass has radix 32 (n = 1024, k1000), its tasks, 32 rows
    apart, sit on distinct banks of the 64 x 4-byte LDS banks at every tile
    width T = 8 .. 64; with a radix-8 / 16 unit pass (n = 2048 / 512) up to
    4 / 2 tasks share banks -- the radix-32 unit-pass plan that avoids it
    measured slower (profiles/r6_ab_notes.txt), so the check is limited to
    radix-32 unit passes."""
    lgr, sh = xf_plan(N)
    for b, s in zip(lgr, sh):
        R, S = 1 << b, 1 << s
        L = R * S
        for tt in range(N // R):
            j = tt & (S - 1)
            x = (tt >> s) * L + j
            for q in range(R):
                assert prow(x + q * S) == prow(x) + prow(q * S), (N, b, s, tt, q)
    R = 1 << lgr[-1]
    if R != 32:
        return
    for lgT in range(3, 7):
        T = 1 << lgT
        tasks = 64 // T
        for t0 in range(0, N // R, tasks):
            for q in range(R):
                banks = {((prow((t0 + i) * R + q) << lgT) + c) % 64
                         for i in range(min(tasks, N // R - t0)) for c in range(T)}
                assert len(banks) == min(tasks, N // R - t0) * T, (N, T, t0, q)


@pytest.mark.parametrize("N", [4, 32, 64, 256, 512])
def test_dif_and_dit_orders(N):
    rng = random.Random(N)
    plan = xf_plan(N)
    nmax = max(N, 512)
    x = [rng.randrange(Q) for _ in range(N)]
    w = root(N)
    X = [sum(x[t] * pow(w, t * k, Q) for t in range(N)) % Q for k in range(N)]
    wi = pow(w, Q - 2, Q)
    Xi = [sum(x[t] * pow(wi, t * k, Q) for t in range(N)) % Q for k in range(N)]
    b = list(x)  # DIF: natural in, X[j] at pos(j)
    lds_transform(b, N, plan, tables(plan, nmax, False), True, False)
    assert [b[xf_pos(plan, k)] for k in range(N)] == X
    b = [0] * N  # inverse DIT: x[t] at pos(t), natural out
    for t in range(N):
        b[xf_pos(plan, t)] = x[t]
    lds_transform(b, N, plan, tables(plan, nmax, True), False, True)
    assert b == Xi


def _ctx(k, n, len2k, ids):
    """DecodeContext::init (src/fec_context.h:232-274): inv_A_i and
    C[j] = -A(w_2k^j) / len_2k."""
    r = root(n)
    x = [pow(r, i, Q) for i in ids]
    A = [1] + [0] * k
    for xi in x:
        A = [((A[d - 1] if d else 0) - xi * A[d]) % Q for d in range(k + 1)]
    inv = []
    for xi in x:
        acc = 0
        for d in range(k, 0, -1):
            acc = (acc * xi + A[d] * d) % Q
        inv.append(pow(acc * xi % Q, Q - 2, Q))
    w2, il = root(len2k), pow(len2k, Q - 2, Q)
    C = []
    for j in range(len2k):
        xj, acc = pow(w2, j, Q), 0
        for d in range(k, -1, -1):
            acc = (acc * xj + A[d]) % Q
        C.append(-acc * il % Q)
    return inv, C


@pytest.mark.parametrize("k,m", [(65, 63), (100, 28), (40, 200)])
@pytest.mark.parametrize("split", [False, True])
def test_decode_pipeline(k, m, split):
    """The kernel's decode order recovers the data polynomial's
    coefficients from any k codeword symbols.  split: NTT_2k / INTT_2k as
    the kernel runs them, two h = len_2k / 2 point transforms each
    (X[2m] = NTT_h(x)[m], X[2m+1] = NTT_h(x_t w^t)[m]; y_t = INTT_h(even)[t]
    + w^-t INTT_h(odd)[t]), C[2m + b] applied to output m of half b."""
    rng = random.Random(k * m)
    n = 1 << (k + m - 1).bit_length()
    len2k = 1 << (2 * k - 1).bit_length()
    nmax = max(n, len2k)
    r = root(n)
    coef = [rng.randrange(65536) for _ in range(k)]
    cw = [sum(c * pow(r, i * t, Q) for t, c in enumerate(coef)) % Q for i in range(n)]
    ids = sorted(rng.sample(range(k + m), k))
    inv, C = _ctx(k, n, len2k, ids)
    pn, p2 = xf_plan(n), xf_plan(len2k)
    buf = [0] * nmax
    for i, z in enumerate(ids):
        buf[xf_pos(pn, z)] = cw[z] * inv[i] % Q
    lds_transform(buf, n, pn, tables(pn, nmax, True), False, True)
    if not split:
        for p in range(k, len2k):
            buf[p] = 0
        lds_transform(buf, len2k, p2, tables(p2, nmax, False), True, False)
        for p in range(len2k):
            buf[p] = buf[p] * C[xf_index(p2, p)] % Q
        lds_transform(buf, len2k, p2, tables(p2, nmax, True), False, True)
        assert buf[:k] == coef
        return
    h = len2k // 2
    w2 = root(len2k)
    even = [buf[t] if t < k else 0 for t in range(h)]
    odd = [even[t] * pow(w2, t, Q) % Q for t in range(h)]
    ph = xf_plan(h)
    out = []
    for b, half in enumerate((even, odd)):
        lds_transform(half, h, ph, tables(ph, nmax, False), True, False)
        for p in range(h):
            half[p] = half[p] * C[2 * xf_index(ph, p) + b] % Q
        lds_transform(half, h, ph, tables(ph, nmax, True), False, True)
        out.append(half)
    w2i = pow(w2, Q - 2, Q)
    y = [(out[0][t] + pow(w2i, t, Q) * out[1][t]) % Q for t in range(k)]
    assert y == coef


# ---------------------------------------------------------------------------
# Erasure decode (ntt.hip, plans with e = n - k <= kErasMax): instead of
# decode_apply's INTT_n -> NTT_2k -> x C -> INTT_2k, the e erased codeword
# symbols are solved from the e "syndromes" the zero-filled codeword leaves
# in the top INTT outputs, then one more INTT_n (non-systematic) or nothing
# (systematic: the data ARE codeword symbols).  The codeword of both types is
# c_j = P(r^j), deg P < k, j < n (positions >= k + m are never sent).

def _lagrange_rows(xs):
    """W[j][u] = coef_u(L_j), L_j = prod_{l != j} (X - x_l) / (x_j - x_l)."""
    e = len(xs)
    A = [1]  # prod (X - x_l), coefficients low to high
    for x in xs:
        A = [(a_lo - x * a) % Q for a, a_lo in zip(A + [0], [0] + A)]
    W = []
    for xj in xs:
        q = [0] * e  # Q_j = A / (X - xj) by synthetic division from the top
        q[e - 1] = 1
        for t in range(e - 1, 0, -1):
            q[t - 1] = (A[t] + xj * q[t]) % Q
        ap = 0
        for t in range(e - 1, -1, -1):
            ap = (ap * xj + q[t]) % Q
        inv = pow(ap, Q - 2, Q)
        W.append([v * inv % Q for v in q])
    return W


@pytest.mark.parametrize("n,k,sys_", [(16, 11, 0), (64, 50, 0), (64, 50, 1), (32, 31, 1),
                                      (128, 100, 0)])
def test_erasure_decode_math(n, k, sys_):
    rng = random.Random(n * 7 + k + sys_)
    r, ri = root(n), pow(root(n), Q - 2, Q)
    P = [rng.randrange(Q) for _ in range(k)]
    c = [sum(P[t] * pow(r, j * t, Q) for t in range(k)) % Q for j in range(n)]
    recv = sorted(rng.sample(range(n), k))
    E = [j for j in range(n) if j not in recv]
    e = len(E)
    # y' = unnormalised INTT_n of the zero-filled codeword
    cz = [c[j] if j in recv else 0 for j in range(n)]
    y = [sum(cz[j] * pow(ri, j * t, Q) for j in range(n)) % Q for t in range(n)]
    # per-pattern constants: B[j][u] = -r^(E_j k) W[j][u], x_j = r^-E_j
    W = _lagrange_rows([pow(ri, j, Q) for j in E])
    B = [[(-pow(r, E[a] * k, Q) * W[a][u]) % Q for u in range(e)] for a in range(e)]
    cE = [sum(B[a][u] * y[k + u] for u in range(e)) % Q for a in range(e)]
    assert cE == [c[j] for j in E]
    if sys_:
        return  # the data rows c_t, t < k: received or in cE
    full = [cz[j] if j in recv else cE[E.index(j)] for j in range(n)]
    ninv = pow(n, Q - 2, Q)
    d = [sum(full[j] * pow(ri, j * t, Q) for j in range(n)) * ninv % Q for t in range(k)]
    assert d == P
    # the kernel's two-pass completion (ntt_eras_kernel, INTT_n in two
    # passes, n = R0 R1): the unit pass of the zero-filled codeword plus its
    # response to c_E, then the last pass alone
    lg = n.bit_length() - 1
    # the kernel's two-pass plan (round 6: the unit pass R1 = 32 from n = 64
    # on; one-pass plans do not take this completion, any split checks the
    # identity)
    lgr, _ = xf_plan(n)
    lg0 = lgr[0] if len(lgr) == 2 else (lg + 1) // 2
    R0, R1 = 1 << lg0, 1 << (lg - lg0)
    w1i = pow(ri, R0, Q)  # w_R1^-1
    # unit pass: group g (elements t = g + R0 q), output u
    Y = [[sum(cz[g + R0 * q] * pow(w1i, q * u, Q) for q in range(R1)) % Q
          for u in range(R1)] for g in range(R0)]
    for a_, t in enumerate(E):
        g, q0 = t % R0, t // R0
        for u in range(R1):
            Y[g][u] = (Y[g][u] + cE[a_] * pow(w1i, q0 * u, Q)) % Q
    # last pass: task j < R1 over the groups v, input twiddle w_n^-jv, then an
    # R0-point inverse DFT; output m is t = j + R1 m
    w0i = pow(ri, R1, Q)  # w_R0^-1
    out = [0] * n
    for j in range(R1):
        for m in range(R0):
            out[j + R1 * m] = sum(Y[v][j] * pow(ri, j * v, Q) * pow(w0i, v * m, Q)
                                  for v in range(R0)) % Q
    assert [out[t] * ninv % Q for t in range(k)] == P
