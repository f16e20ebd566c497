#!/usr/bin/env python3
"""bm_b_identity.py -- the identity rs_bm_k / rs_forney_k rely on when they
replace Omega by B (rs_fast.hip, "Omega or B"):

    after the 2t = 32 Berlekamp-Massey iterations of src/decode.c:49-96
    (Karn's form: B = Lambda / discrepancy at a lengthening, x B otherwise),
    Omega(x0) * B(x0) = x0^(2t-1) at every root x0 of Lambda,
    with Omega = S * Lambda mod x^deg (src/decode.c:147-158).

Pure-Python GF(2^8) restatement (independent of the kernels and the oracle),
checked on random words with 1..16 errors and on fast-path miscorrections
(words 16 symbols from another codeword: 17 of the nonzeros of a shifted
g(x), a weight-33 codeword, added to a codeword), for several fcr / prim.

    python tools/probes/bm_b_identity.py
"""
import random

NR = 32


class Field:
    def __init__(self, poly=0x11D):
        self.exp, self.log = [0] * 512, [255] * 256
        x = 1
        for i in range(255):
            self.exp[i], self.log[x] = x, i
            x <<= 1
            if x & 256:
                x ^= poly
        for i in range(255, 512):
            self.exp[i] = self.exp[i - 255]

    def mul(self, a, b):
        return 0 if a == 0 or b == 0 else self.exp[self.log[a] + self.log[b]]

    def inv(self, a):
        return self.exp[(255 - self.log[a]) % 255]

    def ev(self, p, x):  # p lowest degree first
        r, xp = 0, 1
        for c in p:
            r ^= self.mul(c, xp)
            xp = self.mul(xp, x)
        return r


def generator(F, fcr, prim):
    g = [1]
    for i in range(NR):
        root = F.exp[(prim * (fcr + i)) % 255]
        ng = [0] * (len(g) + 1)
        for j, c in enumerate(g):
            ng[j] ^= F.mul(c, root)
            ng[j + 1] ^= c
        g = ng
    return g  # lowest first, monic


def encode(F, g, msg):  # codeword highest degree first, parity = msg x^32 mod g
    work = list(msg) + [0] * NR
    gh = g[::-1]
    for i in range(len(msg)):
        c = work[i]
        if c:
            for j in range(1, NR + 1):
                work[i + j] ^= F.mul(c, gh[j])
    return list(msg) + work[len(msg):]


def syndromes(F, cw, fcr, prim):
    out = []
    for i in range(NR):
        b, r = F.exp[(prim * (fcr + i)) % 255], 0
        for c in cw:
            r = F.mul(r, b) ^ c
        out.append(r)
    return out


def bm(F, S):
    """src/decode.c:49-96 in value form (Karn: B = Lambda / discr on lengthening)"""
    L, lam, B = 0, [1] + [0] * NR, [1] + [0] * NR
    for r in range(1, NR + 1):
        d = 0
        for i in range(r):
            d ^= F.mul(lam[i], S[r - 1 - i])
        if d == 0:
            B = [0] + B[:-1]
            continue
        T = lam[:]
        for i in range(NR):
            T[i + 1] ^= F.mul(d, B[i])
        if 2 * L <= r - 1:
            L, B = r - L, [F.mul(c, F.inv(d)) for c in lam]
        else:
            B = [0] + B[:-1]
        lam = T
    return lam, B, L


def check(fcr=1, prim=1, trials=100, seed=1):
    """(roots checked, roots where Omega(x0) B(x0) == x0^31, words on the
    fast path that are miscorrections)"""
    F = Field()
    g = generator(F, fcr, prim)
    gh = g[::-1]
    nz = [k for k in range(NR + 1) if gh[k]]
    rng = random.Random(seed)
    tot = good = mis = 0
    for trial in range(trials):
        cw = encode(F, g, [rng.randrange(256) for _ in range(223)])
        bad = cw[:]
        if trial % 2 == 0:
            for p in rng.sample(range(255), rng.randrange(1, 17)):
                bad[p] ^= rng.randrange(1, 256)
        else:
            sh = rng.randrange(0, 255 - NR)
            for k in rng.sample(nz, len(nz) - 16):
                bad[sh + k] ^= gh[k]
        S = syndromes(F, bad, fcr, prim)
        lam, B, L = bm(F, S)
        deg = max(i for i, c in enumerate(lam) if c)
        om = [0] * NR
        for i in range(NR):
            for j in range(i + 1):
                om[i] ^= F.mul(lam[j], S[i - j])
        om = om[:max(deg, 1)]
        roots = [i for i in range(255) if F.ev(lam, F.exp[i]) == 0]
        if len(roots) != deg or deg != L or deg == 0:
            continue  # not the fast path
        mis += trial % 2
        for i in roots:
            x0 = F.exp[i]
            tot += 1
            good += F.mul(F.ev(om, x0), F.ev(B, x0)) == F.exp[(i * (NR - 1)) % 255]
    return tot, good, mis


if __name__ == "__main__":
    for fcr, prim in [(1, 1), (0, 1), (5, 7), (112, 11)]:
        tot, good, mis = check(fcr, prim, trials=120, seed=3)
        print(f"fcr {fcr} prim {prim}: {good} of {tot} roots satisfy Omega(x0) B(x0) = x0^31; "
              f"{mis} fast-path miscorrection words")
