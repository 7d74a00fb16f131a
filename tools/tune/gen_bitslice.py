"""Generate the XOR network of a bitsliced RS(12,8) encode (VERDICT r4 item 4's A/B:
a Cauchy bit-matrix form of ISA-L's parity rows, EC/erasure_coder.c:43, 90 at k=8, m=4).

GF(2^8) multiplication by a constant c is linear over GF(2): with the bytes of a
column split into 8 bit planes P_0..P_7, the planes of c*x are Q_i = XOR over j of
[bit i of c*2^j] P_j.  Parity row a is y_a = XOR_j M[a][j] * x_j, a 32 x 64 binary
matrix from the 64 input planes to the 32 output planes.  Two forms:

- direct: the input planes as they are;
- karatsuba: per group of 4 columns the XOR-circulant sums s = x0^x1^x2^x3,
  u = x1^x3, v = x2^x3, w = x3 (taken in the byte domain before the transpose,
  rs_impl.hpp gf_combine_cauchy4), whose planes feed
  y_a = h_a s ^ c_u(a) u ^ c_v(a) v ^ H w.

Each form's matrix goes through Paar's greedy common-subexpression elimination
(repeatedly XOR the pair of signals that co-occur in the most rows), and the
smaller network is written as straight-line HIP code:

  python tools/tune/gen_bitslice.py > tools/tune/bitslice_net.inc

Prints the XOR counts of both forms on stderr.  The CPU self-check at the end
evaluates the chosen network on random bytes against byte-wise GF products."""
import random
import sys

POLY = 0x11D


def gf_mul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= POLY
        b >>= 1
    return r


def gf_inv(a):
    for b in range(1, 256):
        if gf_mul(a, b) == 1:
            return b
    return 0


K, M = 8, 4
COEF = [[gf_inv((K + a) ^ j) for j in range(K)] for a in range(M)]  # ISA-L gf_gen_cauchy1_matrix parity rows


def mul_rows(c):
    """rows[i] = set of input bit indices j with bit i of c*2^j set"""
    return [{j for j in range(8) if (gf_mul(c, 1 << j) >> i) & 1} for i in range(8)]


def matrix(form):
    """rows: 32 sets of operand-plane indices (operand o, bit j) -> 8*o + j"""
    rows = [set() for _ in range(32)]

    def add(a, o, c):
        if c == 0:
            return
        for i, js in enumerate(mul_rows(c)):
            rows[8 * a + i] ^= {8 * o + j for j in js}

    for g in range(K // 4):
        h = [COEF[0][4 * g + t] for t in range(4)]
        for a in range(M):
            for c in range(4):
                assert COEF[a][4 * g + c] == h[a ^ c]
        H = h[0] ^ h[1] ^ h[2] ^ h[3]
        for a in range(M):
            if form == "direct":
                for c in range(4):
                    add(a, 4 * g + c, COEF[a][4 * g + c])
            else:  # operands 4g+0..3 = s, u, v, w of group g
                add(a, 4 * g + 0, h[a])
                add(a, 4 * g + 1, h[0] ^ h[1] if a in (0, 1) else h[2] ^ h[3])
                add(a, 4 * g + 2, h[0] ^ h[2] if a in (0, 2) else h[1] ^ h[3])
                add(a, 4 * g + 3, H)
    return rows


def paar(rows, nin=64):
    """Greedy CSE: returns (temps [(t, a, b)], rows over signal ids); signal ids < nin are inputs."""
    rows = [set(r) for r in rows]
    temps = []
    nxt = nin
    while True:
        best, cnt = None, 1
        counts = {}
        for r in rows:
            rl = sorted(r)
            for x in range(len(rl)):
                for y in range(x + 1, len(rl)):
                    p = (rl[x], rl[y])
                    counts[p] = counts.get(p, 0) + 1
        for p, c in counts.items():
            if c > cnt or (c == cnt and best is not None and p < best):
                best, cnt = p, c
        if best is None or cnt < 2:
            break
        a, b = best
        temps.append((nxt, a, b))
        for r in rows:
            if a in r and b in r:
                r -= {a, b}
                r.add(nxt)
        nxt += 1
    return temps, rows


def xor_count(temps, rows):
    return len(temps) + sum(max(0, len(r) - 1) for r in rows)


def evaluate(form, temps, rows, cols):
    """cols: K byte values; returns M parity bytes through the network"""
    if form == "karatsuba":
        ops = []
        for g in range(K // 4):
            x = cols[4 * g:4 * g + 4]
            ops += [x[0] ^ x[1] ^ x[2] ^ x[3], x[1] ^ x[3], x[2] ^ x[3], x[3]]
    else:
        ops = list(cols)
    sig = {8 * o + j: (ops[o] >> j) & 1 for o in range(K) for j in range(8)}
    for t, a, b in temps:
        sig[t] = sig[a] ^ sig[b]
    out = []
    for a in range(M):
        v = 0
        for i in range(8):
            bit = 0
            for s in rows[8 * a + i]:
                bit ^= sig[s]
            v |= bit << i
        out.append(v)
    return out


def main():
    res = {}
    for form in ("direct", "karatsuba"):
        rows = matrix(form)
        ones = sum(len(r) for r in rows)
        temps, red = paar(rows)
        n = xor_count(temps, red)
        extra = 4 * 8 * (K // 4) if form == "karatsuba" else 0  # s, u, v per dword: 4 XORs x 8 dwords x groups
        print(f"{form}: {ones} ones, naive {ones - 32} XORs, Paar {n} XORs (+{extra} byte-domain) per 32-byte column",
              file=sys.stderr)
        res[form] = (n + extra, temps, red)
    form = min(res, key=lambda f: res[f][0])
    _, temps, red = res[form]
    rng = random.Random(1)
    for _ in range(2000):
        cols = [rng.randrange(256) for _ in range(K)]
        want = [0] * M
        for a in range(M):
            for j in range(K):
                want[a] ^= gf_mul(COEF[a][j], cols[j])
        assert evaluate(form, temps, red, cols) == want
    print(f"chosen: {form}", file=sys.stderr)
    print(f"// generated by tools/tune/gen_bitslice.py: form {form}, {res[form][0]} XORs per lane and 32-byte column")
    print(f"#define BITSLICE_KARATSUBA {1 if form == 'karatsuba' else 0}")
    print("#define BITSLICE_NET(P, Y) \\")
    lines = [f"    const uint32_t t{t} = {sname(a)} ^ {sname(b)};" for t, a, b in temps]
    for i, r in enumerate(red):
        expr = " ^ ".join(sname(s) for s in sorted(r)) if r else "0u"
        lines.append(f"    Y[{i}] = {expr};")
    print(" \\\n".join(lines))


def sname(s):
    return f"P[{s}]" if s < 64 else f"t{s}"


if __name__ == "__main__":
    main()
