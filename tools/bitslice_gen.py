"""Bitsliced AES inverse round for gfx950, generated and checked here (round 6, VERDICT r05 item 2:
measure a bitsliced decrypt before deciding whether a hybrid with the T-table decrypt can pay).

Layout: a lane holds 32 blocks; plane p = 8 * byte + bit is one 32-bit word whose bit j belongs
to block j.  InvShiftRows is a renaming of planes.  InvSubBytes is a circuit per byte-slice:
    InvS(y) = inv(A^-1 (y ^ 0x63))        (FIPS-197 5.3.2; rijndael.py's tables)
with the GF(2^8) inversion in the tower GF((2^4)^2) (y^2 + y + lambda over GF(2)[z]/(z^4+z+1)):
    a = a1 Y + a0,  D = lambda a1^2 + a1 a0 + a0^2,  a^-1 = (a1 D^-1) Y + ((a0 + a1) D^-1)
the basis change folded into the affine input map and the output map, D^-1 a 4-input function
(each output bit three v_bitop3: two 3-input halves and a select).  InvMixColumns as MixColumns
after the {04}x^2+{05} pre-step.  Every linear map is emitted as 3-input XORs.

The circuit is a DAG of 2-input AND / XOR / XNOR gates; a fusion pass merges single-use gates
into their consumer while the merged function has at most 3 distinct inputs, so each emitted op
is one v_bitop3_b32 with an 8-bit truth table.  The whole round is simulated on 256-bit integers
(every S-box input at once) and on random blocks against a plain AES inverse round, then written
as tools/bs_aes_inv.h (a device function per round).  Diagnostic tool only; not in the product.

Usage: python tools/bitslice_gen.py   (writes tools/bs_aes_inv.h, prints op counts)
"""
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))

# ---------------------------------------------------------------- GF(2^8), AES polynomial basis
def gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = ((a << 1) ^ 0x11B) if a & 0x80 else (a << 1)
        b >>= 1
    return r


def ginv(a):
    if a == 0:
        return 0
    r = 1
    for _ in range(254):
        r = gmul(r, a)
    return r


def affine(x):  # S-box affine map (FIPS-197 5.1.1)
    r = 0
    for i in range(8):
        b = ((x >> i) ^ (x >> ((i + 4) % 8)) ^ (x >> ((i + 5) % 8)) ^ (x >> ((i + 6) % 8)) ^ (x >> ((i + 7) % 8))) & 1
        r |= b << i
    return r ^ 0x63


SBOX = [affine(ginv(x)) for x in range(256)]
INV_SBOX = [0] * 256
for i, v in enumerate(SBOX):
    INV_SBOX[v] = i


# ---------------------------------------------------------------- GF(2) linear algebra
def mat_apply(M, x):  # M: list of 8 row masks; output bit i = parity(M[i] & x)
    return sum(((bin(M[i] & x).count("1") & 1) << i) for i in range(len(M)))


def mat_from_columns(cols):  # column j = image of basis vector j
    return [sum(((cols[j] >> i) & 1) << j for j in range(8)) for i in range(8)]


def mat_inv(M):
    n = len(M)
    A = [(M[i] | (1 << (n + i))) for i in range(n)]
    for c in range(n):
        p = next(r for r in range(c, n) if (A[r] >> c) & 1)
        A[c], A[p] = A[p], A[c]
        for r in range(n):
            if r != c and (A[r] >> c) & 1:
                A[r] ^= A[c]
    return [A[i] >> n for i in range(n)]


# ---------------------------------------------------------------- the tower isomorphism
def g16mul(a, b):  # GF(2)[z]/(z^4 + z + 1)
    r = 0
    for i in range(4):
        if (b >> i) & 1:
            r ^= a << i
    for i in (6, 5, 4):
        if (r >> i) & 1:
            r ^= 0b10011 << (i - 4)
    return r


def find_tower():
    # omega in GF(256) with omega^4 + omega + 1 = 0 (a copy of z); lambda with y^2+y+lambda
    # irreducible over GF(16); beta in GF(256) a root of it
    def gpow(a, e):
        r = 1
        for _ in range(e):
            r = gmul(r, a)
        return r
    omegas = [w for w in range(2, 256) if gpow(w, 4) ^ w ^ 1 == 0]
    w = omegas[0]

    def emb(v):  # GF(16) element (bits of z^k) -> GF(256)
        r = 0
        for k in range(4):
            if (v >> k) & 1:
                r ^= gpow(w, k)
        return r
    for lam in range(1, 16):
        if any(g16mul(y, y) ^ y ^ lam == 0 for y in range(16)):
            continue  # reducible over GF(16)
        L = emb(lam)
        betas = [b for b in range(256) if gmul(b, b) ^ b ^ L == 0]
        if betas:
            beta = betas[0]
            # tower bit t: t < 4 -> a0 coefficient z^t ; t >= 4 -> a1 coefficient z^(t-4) (times beta)
            cols = [gpow(w, t) for t in range(4)] + [gmul(gpow(w, t), beta) for t in range(4)]
            T_inv = mat_from_columns(cols)  # tower bits -> AES bits
            return lam, mat_inv(T_inv), T_inv
    raise RuntimeError("no tower")


LAM, T, T_INV = find_tower()
_A_cols = [affine(1 << j) ^ 0x63 for j in range(8)]
A_M = mat_from_columns(_A_cols)  # affine(x) = A x + 0x63
A_INV_M = mat_inv(A_M)
# InvS(y) = T_inv * towerinv( T * A^-1 * (y ^ 0x63) )


def _check_iso():
    for y in range(256):
        x = mat_apply(A_INV_M, y ^ 0x63)
        assert INV_SBOX[y] == ginv(x)
        t = mat_apply(T, x)
        assert mat_apply(T_INV, t) == x
_check_iso()
M_IN = [0] * 8  # rows of T * A^-1
for i in range(8):
    row = 0
    for j in range(8):
        v = mat_apply(T, mat_apply(A_INV_M, 1 << j))
        row |= ((v >> i) & 1) << j
    M_IN[i] = row
C_IN = mat_apply(T, mat_apply(A_INV_M, 0x63))  # constant after the map (folded as complements)


# ---------------------------------------------------------------- gate DAG
class Circ:
    def __init__(self, ninputs):
        self.ops = []  # (kind, a, b) with node ids; kinds: and, xor, xnor, in, const
        self.n_in = ninputs
        for i in range(ninputs):
            self.ops.append(("in", i, None))

    def add(self, kind, a, b):
        self.ops.append((kind, a, b))
        return len(self.ops) - 1

    def xor(self, a, b):
        return self.add("xor", a, b)

    def and_(self, a, b):
        return self.add("and", a, b)

    def xnor(self, a, b):
        return self.add("xnor", a, b)

    def not_(self, a):
        return self.add("not", a, None)

    def xor_many(self, xs, invert=False):
        xs = list(xs)
        assert xs
        acc = xs[0]
        for x in xs[1:]:
            acc = self.xor(acc, x)
        return self.not_(acc) if invert else acc

    def lin(self, M, inputs, const=0):  # output bit i = parity(M[i] & inputs) ^ const_i
        return [self.xor_many([inputs[j] for j in range(len(inputs)) if (M[i] >> j) & 1], bool((const >> i) & 1))
                for i in range(len(M))]

    def g16mul(self, a, b):
        c = [None] * 7
        for i in range(4):
            for j in range(4):
                t = self.and_(a[i], b[j])
                c[i + j] = t if c[i + j] is None else self.xor(c[i + j], t)
        return [self.xor(c[0], c[4]), self.xor_many([c[1], c[4], c[5]]), self.xor_many([c[2], c[5], c[6]]),
                self.xor(c[3], c[6])]

    def lut4(self, x, table):  # 4-input function by Shannon on x[3]: f = x3 ? hi(x0,x1,x2) : lo(...)
        return self.add("lut4", tuple(x), table)


def g16_lin_matrix(f):  # 4x4 GF(2) matrix of a GF(2)-linear map on GF(16)
    return [sum((((f(1 << j)) >> i) & 1) << j for j in range(4)) for i in range(4)]


def g16sq(v):
    return g16mul(v, v)


def g16inv(v):
    if v == 0:
        return 0
    r = 1
    for _ in range(14):
        r = g16mul(r, v)
    return r


def inv_sbox_circuit(C, y):
    """y: 8 node ids (bit i of the byte) -> 8 node ids of InvS(y)."""
    t = C.lin(M_IN, y, C_IN)            # tower coordinates of A^-1 (y ^ 0x63)
    a0, a1 = t[0:4], t[4:8]
    # D = lambda a1^2 + a1 a0 + a0^2
    Lsq = g16_lin_matrix(lambda v: g16mul(LAM, g16sq(v)))
    Sq = g16_lin_matrix(g16sq)
    p = C.g16mul(a1, a0)
    la = C.lin(Lsq, a1)
    sa = C.lin(Sq, a0)
    D = [C.xor_many([p[i], la[i], sa[i]]) for i in range(4)]
    Dinv = [C.lut4(D, [(g16inv(v) >> i) & 1 for v in range(16)]) for i in range(4)]
    s = [C.xor(a0[i], a1[i]) for i in range(4)]
    r1 = C.g16mul(a1, Dinv)
    r0 = C.g16mul(s, Dinv)
    return C.lin(T_INV, r0 + r1)


# ---------------------------------------------------------------- simulation on integers
def simulate(C, inputs, width_mask):
    val = []
    for kind, a, b in C.ops:
        if kind == "in":
            val.append(inputs[a])
        elif kind == "xor":
            val.append(val[a] ^ val[b])
        elif kind == "xnor":
            val.append(~(val[a] ^ val[b]) & width_mask)
        elif kind == "and":
            val.append(val[a] & val[b])
        elif kind == "not":
            val.append(~val[a] & width_mask)
        elif kind == "lut4":
            xs = [val[i] for i in a]
            out = 0
            for v in range(16):
                if b[v]:
                    m = width_mask
                    for k in range(4):
                        m &= xs[k] if (v >> k) & 1 else ~xs[k]
                    out |= m
            val.append(out & width_mask)
        else:
            raise ValueError(kind)
    return val


def check_sbox():
    C = Circ(8)
    out = inv_sbox_circuit(C, list(range(8)))
    W = (1 << 256) - 1
    ins = [sum(((x >> i) & 1) << x for x in range(256)) for i in range(8)]
    v = simulate(C, ins, W)
    for i in range(8):
        want = sum(((INV_SBOX[x] >> i) & 1) << x for x in range(256))
        assert v[out[i]] == want, i
    return C, out


# ---------------------------------------------------------------- fusion into 3-input ops
OPS = {"xor": lambda a, b: a ^ b, "xnor": lambda a, b: ~(a ^ b) & 0xff, "and": lambda a, b: a & b}
VARS = (0xF0, 0xCC, 0xAA)  # truth-table columns of the three bitop3 inputs (a, b, c)


def fuse(C, outputs):
    """-> list of (dst, (src...), tt8) 3-input ops computing `outputs`; srcs are node ids of
    inputs or of earlier ops.  A single-use gate is merged into its consumer while the merged
    function has <= 3 distinct leaves."""
    uses = [0] * len(C.ops)
    for kind, a, b in C.ops:
        if kind in ("xor", "xnor", "and"):
            uses[a] += 1
            uses[b] += 1
        elif kind == "not":
            uses[a] += 1
        elif kind == "lut4":
            for i in a:
                uses[i] += 1
    for o in outputs:
        uses[o] += 1
    memo = {}

    def expr(n):  # -> (leaves tuple, function over leaves as a python callable on bit masks)
        if n in memo:
            return memo[n]
        kind, a, b = C.ops[n]
        if kind == "in" or kind == "lut4":
            r = ((n,), lambda env, n=n: env[n])
        elif kind == "not":
            la, fa = leaf_or_expr(a)
            r = (la, lambda env, fa=fa: ~fa(env) & 0xff)
        else:
            la, fa = leaf_or_expr(a)
            lb, fb = leaf_or_expr(b)
            leaves = tuple(dict.fromkeys(la + lb))
            if len(leaves) > 3:  # cannot merge: both children become leaves
                leaves = tuple(dict.fromkeys((a, b)))
                op = OPS[kind]
                r = (leaves, lambda env, a=a, b=b, op=op: op(env[a], env[b]))
                memo[n] = r
                return r
            op = OPS[kind]
            r = (leaves, lambda env, fa=fa, fb=fb, op=op: op(fa(env), fb(env)))
        memo[n] = r
        return r

    def leaf_or_expr(m):
        kind = C.ops[m][0]
        if kind in ("in", "lut4") or uses[m] > 1:
            return (m,), (lambda env, m=m: env[m])
        return expr(m)

    emitted = {}
    prog = []

    def emit(n):
        if n in emitted:
            return
        kind, a, b = C.ops[n]
        if kind == "in":
            emitted[n] = True
            return
        if kind == "lut4":
            for i in a:
                emit(i)
            prog.append((n, tuple(a), b, "lut4"))
            emitted[n] = True
            return
        leaves, f = expr(n)
        for l in leaves:
            emit(l)
        env = {l: VARS[k] for k, l in enumerate(leaves)}
        tt = f(env) & 0xff
        prog.append((n, leaves, tt, "bop3"))
        emitted[n] = True

    # make every multi-use / output node its own op
    order = list(range(len(C.ops)))
    for n in order:
        if C.ops[n][0] != "in" and (uses[n] > 1 or n in outputs):
            pass
    for o in outputs:
        emit(o)
    return prog


def prog_cost(prog):
    n = 0
    for _, leaves, tt, kind in prog:
        n += 3 if kind == "lut4" else 1
    return n


def sim_prog(prog, env0, mask):
    env = dict(env0)
    for dst, leaves, tt, kind in prog:
        if kind == "lut4":
            xs = [env[i] for i in leaves]
            out = 0
            for v in range(16):
                if tt[v]:
                    m = mask
                    for k in range(4):
                        m &= xs[k] if (v >> k) & 1 else ~xs[k]
                    out |= m
            env[dst] = out & mask
        else:
            xs = [env[l] for l in leaves] + [0] * (3 - len(leaves))
            out = 0
            for bit in range(8):
                if (tt >> bit) & 1:
                    m = mask
                    for k in range(3):
                        m &= xs[k] if (VARS[k] >> bit) & 1 else ~xs[k]
                    out |= m
            env[dst] = out & mask
    return env


# ---------------------------------------------------------------- InvMixColumns
def xtime_planes(C, b):  # b: 8 node ids (bit i) -> x * b
    return [b[7], C.xor(b[0], b[7]), b[1], C.xor(b[2], b[7]), C.xor(b[3], b[7]), b[4], b[5], b[6]]


def inv_mix_column(C, col):  # col: 4 bytes x 8 planes
    u = xtime_planes(C, xtime_planes(C, [C.xor(col[0][i], col[2][i]) for i in range(8)]))
    v = xtime_planes(C, xtime_planes(C, [C.xor(col[1][i], col[3][i]) for i in range(8)]))
    b = [[C.xor(col[0][i], u[i]) for i in range(8)], [C.xor(col[1][i], v[i]) for i in range(8)],
         [C.xor(col[2][i], u[i]) for i in range(8)], [C.xor(col[3][i], v[i]) for i in range(8)]]
    out = []
    for r in range(4):
        x = xtime_planes(C, [C.xor(b[r][i], b[(r + 1) % 4][i]) for i in range(8)])
        out.append([C.xor_many([x[i], b[(r + 1) % 4][i], b[(r + 2) % 4][i], b[(r + 3) % 4][i]]) for i in range(8)])
    return out


def mix_circuit():
    C = Circ(32)
    col = [[8 * r + i for i in range(8)] for r in range(4)]
    out = inv_mix_column(C, col)
    return C, [p for byte in out for p in byte]


def ref_inv_mix(col):
    a = col
    return [gmul(a[0], 14) ^ gmul(a[1], 11) ^ gmul(a[2], 13) ^ gmul(a[3], 9),
            gmul(a[0], 9) ^ gmul(a[1], 14) ^ gmul(a[2], 11) ^ gmul(a[3], 13),
            gmul(a[0], 13) ^ gmul(a[1], 9) ^ gmul(a[2], 14) ^ gmul(a[3], 11),
            gmul(a[0], 11) ^ gmul(a[1], 13) ^ gmul(a[2], 9) ^ gmul(a[3], 14)]


def check_mix(prog, outs):
    rng = random.Random(1)
    cols = [[rng.randrange(256) for _ in range(4)] for _ in range(32)]
    env = {}
    for r in range(4):
        for i in range(8):
            env[8 * r + i] = sum((((cols[j][r] >> i) & 1) << j) for j in range(32))
    e = sim_prog(prog, env, 0xFFFFFFFF)
    for j in range(32):
        want = ref_inv_mix(cols[j])
        got = [sum((((e[outs[8 * r + i]] >> j) & 1) << i) for i in range(8)) for r in range(4)]
        assert got == want, (j, got, want)


# ---------------------------------------------------------------- emission
def emit_c(name, prog, n_in, outs, lut_helper="bs_lut4"):
    lines = ["__host__ __device__ __forceinline__ void %s(const uint32_t* __restrict__ in, uint32_t* __restrict__ out) {"
             % name]
    names = {i: "in[%d]" % i for i in range(n_in)}
    for k, (dst, leaves, tt, kind) in enumerate(prog):
        v = "t%d" % k
        if kind == "lut4":
            lo = sum(tt[v2] << v2 for v2 in range(16))
            lines.append("    const uint32_t %s = %s<0x%04x>(%s);" % (v, lut_helper, lo, ", ".join(names[l] for l in leaves)))
        else:
            args = [names[l] for l in leaves] + ["0u"] * (3 - len(leaves))
            lines.append("    const uint32_t %s = BS_BOP3(%s, %s, %s, 0x%02x);" % (v, args[0], args[1], args[2], tt))
        names[dst] = v
    for i, o in enumerate(outs):
        lines.append("    out[%d] = %s;" % (i, names[o]))
    lines.append("}")
    return "\n".join(lines)


def main():
    Cs, souts = check_sbox()
    sprog = fuse(Cs, souts)
    env = {i: sum((((x >> i) & 1) << x) for x in range(256)) for i in range(8)}
    e = sim_prog(sprog, env, (1 << 256) - 1)
    for i in range(8):
        assert e[souts[i]] == sum(((INV_SBOX[x] >> i) & 1) << x for x in range(256))
    Cm, mouts = mix_circuit()
    mprog = fuse(Cm, mouts)
    check_mix(mprog, mouts)
    sc, mc = prog_cost(sprog), prog_cost(mprog)
    per_round = 16 * sc + 4 * mc + 128
    print("tower lambda=%d; InvS %d ops (2-input gates %d), InvMixColumns %d per column, round %d ops "
          "(+128 key XORs) per 32 x 64 = 2048 blocks: %.3f per block-round"
          % (LAM, sc, sum(1 for k, _, _ in Cs.ops if k not in ("in",)), mc, per_round, per_round / 2048.0))
    hdr = ["// bs_aes_inv.h -- GENERATED by tools/bitslice_gen.py (checked there: the inverse S-box on all",
           "// 256 inputs, InvMixColumns on random columns).  Diagnostic microbenchmark only.",
           "// Plane p = 8 * byte + bit of a 32-bit word, bit j of the word = block j.",
           "#pragma once",
           "#include <stdint.h>",
           "#include <hip/hip_runtime.h>",
           "// v_bitop3_b32 on the device; the same truth table evaluated on the host (the microbenchmark",
           "// checks the GPU's output against a host run of these functions)",
           "__host__ __device__ inline uint32_t bs_bop3_ref(uint32_t a, uint32_t b, uint32_t c, unsigned t) {",
           "    uint32_t r = 0;",
           "    for (unsigned k = 0; k < 8; k++)",
           "        if ((t >> k) & 1u)",
           "            r |= (((0xF0u >> k) & 1u) ? a : ~a) & (((0xCCu >> k) & 1u) ? b : ~b) & (((0xAAu >> k) & 1u) ? c : ~c);",
           "    return r;",
           "}",
           "#if defined(__HIP_DEVICE_COMPILE__)",
           "#define BS_BOP3(a, b, c, t) __builtin_amdgcn_bitop3_b32((a), (b), (c), (t))",
           "#else",
           "#define BS_BOP3(a, b, c, t) bs_bop3_ref((a), (b), (c), (t))",
           "#endif",
           "// 4-input function (truth table bit v = f(x0..x3 = bits of v)) as two 3-input halves + a select",
           "template <unsigned TT>",
           "__host__ __device__ __forceinline__ uint32_t bs_lut4(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {",
           "    // table over (x0, x1, x2) for x3 = 0 / 1, in bitop3's column order (a = x2, b = x1, c = x0)",
           "    constexpr unsigned lo = BS_LUT3(TT & 0xffu), hi = BS_LUT3((TT >> 8) & 0xffu);",
           "    const uint32_t f0 = BS_BOP3(x2, x1, x0, lo), f1 = BS_BOP3(x2, x1, x0, hi);",
           "    return BS_BOP3(x3, f1, f0, 0xCA);  // x3 ? f1 : f0",
           "}"]
    # BS_LUT3: reorder an 8-entry table indexed by v = x0 + 2 x1 + 4 x2 into bitop3's bit order
    # (bit k of the immediate: a = bit 2 of k... ) -- bitop3 column for (a,b,c) = (F0,CC,AA) masks
    lut3 = ["constexpr unsigned bs_lut3(unsigned t) {",
            "    unsigned r = 0;",
            "    for (unsigned k = 0; k < 8; k++) {",
            "        const unsigned a = (0xF0u >> k) & 1u, b = (0xCCu >> k) & 1u, c = (0xAAu >> k) & 1u;",
            "        const unsigned v = c | (b << 1) | (a << 2);  // a = x2, b = x1, c = x0",
            "        r |= ((t >> v) & 1u) << k;",
            "    }",
            "    return r;",
            "}",
            "#define BS_LUT3(t) bs_lut3(t)"]
    cut = hdr.index("#endif") + 1
    body = "\n".join(hdr[:cut] + lut3 + hdr[cut:]) + "\n\n" + emit_c("bs_inv_sbox", sprog, 8, souts) + "\n\n" + \
        emit_c("bs_inv_mix_column", mprog, 32, mouts) + "\n"
    out = os.path.join(HERE, "bs_aes_inv.h")
    with open(out, "w") as fh:
        fh.write(body)
    print("wrote", out)


if __name__ == "__main__":
    main()
