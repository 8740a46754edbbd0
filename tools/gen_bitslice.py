#!/usr/bin/env python3
"""Bitsliced GF(2^16) fragment map: network builder, bit-level simulator and HIP emitter
(experiment for the 8-output passes; see DESIGN.md §4 "C5").

Multiplication by a constant c over GF(2^16) is a 16x16 GF(2) matrix M_c (bit p of c*x is the XOR
of the bits b of x with M_c[p][b] = 1, rs_galois_mult == carry-less multiply mod 0x1100b,
SURVEY.md §0.2).  A lane holds 32 words of each fragment; a 16x16 bit transpose inside each
16-bit half of 16 dwords turns them into 16 bit planes (plane of bit b in register 15 - b, word w
at bit (15 - w/2) + 16*(w%2) -- the same involution maps output planes back to words).  Output
plane (r, p) is then the XOR over inputs j of the input planes b with M_{A[r][j]}[p][b] = 1: pure
VALU XORs, no table lookups.  Per input, common pairs are factored out first (Paar's greedy
algorithm), and the accumulation uses three-input XORs (v_bitop3).
"""
import itertools
import sys

POLY = 0x1100B


def gf_mul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x10000:
            a ^= POLY
    return r


def bitmatrix(c):
    """M[p] = mask over input bits b (bit p of c*(1<<b))."""
    M = [0] * 16
    for b in range(16):
        v = gf_mul(c, 1 << b)
        for p in range(16):
            if (v >> p) & 1:
                M[p] |= 1 << b
    return M


def paar(rows, nin, cap=1 << 30):
    """rows: list of sets of variable ids (< nin).  Returns (temps [(a, b)], rows rewritten): at
    most `cap` temps (each temp is a register the whole input's network may keep live)."""
    R = [set(s) for s in rows]
    temps = []
    nvar = nin
    while len(temps) < cap:
        cnt = {}
        for s in R:
            for a, b in itertools.combinations(sorted(s), 2):
                cnt[(a, b)] = cnt.get((a, b), 0) + 1
        if not cnt:
            break
        (a, b), c = max(cnt.items(), key=lambda kv: (kv[1], -kv[0][0], -kv[0][1]))
        if c < 2:
            break
        temps.append((a, b))
        for s in R:
            if a in s and b in s:
                s.discard(a)
                s.discard(b)
                s.add(nvar)
        nvar += 1
    return temps, R


def build(coeff, cap=1 << 30):
    """coeff: R x K.  Per input j: (temps, rows) with rows[r*16+p] = set of variables, variables
    0..15 = input bit planes (bit b), 16.. = temps."""
    Rn, K = len(coeff), len(coeff[0])
    net = []
    for j in range(K):
        rows = []
        for r in range(Rn):
            M = bitmatrix(coeff[r][j] & 0xFFFF)
            for p in range(16):
                rows.append({b for b in range(16) if (M[p] >> b) & 1})
        net.append(paar(rows, 16, cap))
    return net


def simulate(coeff, inputs):
    """inputs: K lists of 32 words -> R lists of 32 words, through planes and the network."""
    Rn, K = len(coeff), len(coeff[0])
    net = build(coeff)
    acc = [[0] * 16 for _ in range(Rn)]
    for j in range(K):
        planes = [0] * 16
        for w, x in enumerate(inputs[j]):
            for b in range(16):
                if (x >> b) & 1:
                    planes[b] |= 1 << w
        temps, rows = net[j]
        val = list(planes)
        for a, b in temps:
            val.append(val[a] ^ val[b])
        for i, s in enumerate(rows):
            for v in s:
                acc[i // 16][i % 16] ^= val[v]
    out = []
    for r in range(Rn):
        out.append([sum(((acc[r][p] >> w) & 1) << p for p in range(16)) for w in range(32)])
    return out


def emit_net(coeff, fn="bs_net", cap=1 << 30):
    """HIP device functions fn<J>(acc, P): acc[r][15-p] ^= output plane (r, p) contribution of
    input J, P = the 16 plane registers of input J (plane of bit b in P[15-b])."""
    Rn, K = len(coeff), len(coeff[0])
    net = build(coeff, cap)
    out = [f"template <int J> __device__ __forceinline__ void {fn}(uint32_t (&acc)[{Rn}][16], "
           f"const uint32_t (&P)[16]);"]
    for j, (temps, rows) in enumerate(net):
        lines = [f"template <> __device__ __forceinline__ void {fn}<{j}>(uint32_t (&acc)[{Rn}][16], "
                 "const uint32_t (&P)[16])", "{"]

        def ref(v):
            return f"P[{15 - v}]" if v < 16 else f"t{v}"
        for i, (a, b) in enumerate(temps):
            lines.append(f"    const uint32_t t{16 + i} = {ref(a)} ^ {ref(b)};")
        for i, s in enumerate(rows):
            terms = sorted(s)
            if not terms:
                continue
            dst = f"acc[{i // 16}][{15 - i % 16}]"
            while len(terms) >= 2:
                lines.append(f"    {dst} = xor3({dst}, {ref(terms[0])}, {ref(terms[1])});")
                terms = terms[2:]
            if terms:
                lines.append(f"    {dst} ^= {ref(terms[0])};")
        lines.append("}")
        out.append("\n".join(lines))
    return "\n\n".join(out) + "\n"


def _self_test():
    import random
    rnd = random.Random(5)
    coeff = [[rnd.randrange(65536) for _ in range(5)] for _ in range(3)]
    inputs = [[rnd.randrange(65536) for _ in range(32)] for _ in range(5)]
    got = simulate(coeff, inputs)
    for r in range(3):
        for w in range(32):
            want = 0
            for j in range(5):
                want ^= gf_mul(coeff[r][j], inputs[j][w])
            assert got[r][w] == want
    print("bitslice network simulation matches GF(2^16) products")


if __name__ == "__main__":
    _self_test()
