"""Map the bitsliced AES round circuit onto gfx950's v_bitop3_b32 (any
boolean function of three 32-bit operands, at most one of them scalar) and
emit tools/bitslice/qpp_bs_gen.h.

The circuit per output column of a round is four S-boxes (the Boyar-Peralta
depth-16 circuit, as in qpp_bitslice.h) followed by MixColumns.  The round key
of the previous round is folded into the S-box inputs: the top linear layer's
XORs of raw inputs take the matching key combination as their (scalar) third
operand, so AddRoundKey costs no instruction.  The last round has no
MixColumns and folds its own round key into the S-box outputs.

Mapping: every gate starts as a 2-input LUT; a LUT whose only consumer can
absorb it (merged support of at most 3 leaves, at most 1 scalar) is merged
into that consumer; a LUT all of whose consumers can absorb it is duplicated
into them.  Several merge orders are tried and the smallest cover is kept.
The result is checked against the unmapped circuit on random inputs.

    python tools/lutmap.py            # writes tools/bitslice/qpp_bs_gen.h
"""

import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "bitslice", "qpp_bs_gen.h")
M32 = 0xFFFFFFFF

# ------------------------------------------------------------------ circuit --


class Circuit:
    def __init__(self):
        self.inputs = []      # (name, kind) kind 'v' or 's'
        self.kind = {}
        self.gates = []       # (name, op, a, b): op in xor, and, xnor
        self.outputs = []

    def inp(self, name, kind="v"):
        self.inputs.append(name)
        self.kind[name] = kind
        return name

    def g(self, name, op, a, b):
        assert a in self.kind and b in self.kind, (name, a, b)
        self.gates.append((name, op, a, b))
        self.kind[name] = "v"
        return name


SBOX_TOP = """y14=x3^x5 y13=x0^x6 y9=x0^x3 y8=x0^x5 t0=x1^x2 y1=t0^x7 y4=y1^x3 y12=y13^y14
y2=y1^x0 y5=y1^x6 y3=y5^y8 t1=x4^y12 y15=t1^x5 y20=t1^x1 y6=y15^x7 y10=y15^t0
y11=y20^y9 y7=x7^y11 y17=y10^y11 y19=y10^y8 y16=t0^y11 y21=y13^y16 y18=x0^y16"""
SBOX_MID = """t2=y12&y15 t3=y3&y6 t4=t3^t2 t5=y4&X7 t6=t5^t2 t7=y13&y16 t8=y5&y1 t9=t8^t7
t10=y2&y7 t11=t10^t7 t12=y9&y11 t13=y14&y17 t14=t13^t12 t15=y8&y10 t16=t15^t12
t17=t4^t14 t18=t6^t16 t19=t9^t14 t20=t11^t16 t21=t17^y20 t22=t18^y19 t23=t19^y21 t24=t20^y18
t25=t21^t22 t26=t21&t23 t27=t24^t26 t28=t25&t27 t29=t28^t22 t30=t23^t24 t31=t22^t26
t32=t31&t30 t33=t32^t24 t34=t23^t33 t35=t27^t33 t36=t24&t35 t37=t36^t34 t38=t27^t36
t39=t29&t38 t40=t25^t39 t41=t40^t37 t42=t29^t33 t43=t29^t40 t44=t33^t37 t45=t42^t41
z0=t44&y15 z1=t37&y6 z2=t33&X7 z3=t43&y16 z4=t40&y1 z5=t29&y7 z6=t42&y11 z7=t45&y17
z8=t41&y10 z9=t44&y12 z10=t37&y3 z11=t33&y4 z12=t43&y13 z13=t40&y5 z14=t29&y2
z15=t42&y9 z16=t45&y14 z17=t41&y8
t46=z15^z16 t47=z10^z11 t48=z5^z13 t49=z9^z10 t50=z2^z12 t51=z2^z5 t52=z7^z8
t53=z0^z3 t54=z6^z7 t55=z16^z17 t56=z12^t48 t57=t50^t53 t58=z4^t46 t59=z3^t54 t60=t46^t57
t61=z14^t57 t62=t52^t58 t63=t49^t58 t64=z4^t59 t65=t61^t62 t66=z1^t63
s0=t59^t63 s6=t56~t62 s7=t48~t60 t67=t64^t65 s3=t53^t66 s4=t51^t66 s5=t47^t65 s1=t64~s3 s2=t55~t67"""
# key bits of the S-box input needed alone / in pairs by the top layer (x_i = bit 7 - i)
KEY_SINGLE = (0, 1, 3, 4, 5, 6, 7)
KEY_PAIR = {"y14": (3, 5), "y13": (0, 6), "y9": (0, 3), "y8": (0, 5), "t0": (1, 2)}
# scalar key words per S-box, in this order (the order of the key table):
KEY_WORDS = [f"p{a}{b}" for a, b in KEY_PAIR.values()] + [f"k{i}" for i in KEY_SINGLE]


def add_sbox(c, pre, x, keyed, out_key):
    """Gates of one S-box; x[i] = input name of x_i (bit 7 - i); returns the
    names of the 8 outputs in bit order (bit 0 first).  keyed: input key
    folded in (scalars pre+k*/p*); out_key: scalars pre+o0..o7 XORed into the
    outputs (bit b)."""
    n = lambda s: pre + s  # noqa: E731
    env = {f"x{i}": x[i] for i in range(8)}
    if keyed:
        for w in KEY_WORDS:
            c.inp(n(w), "s")
    corrected = set()

    def ref(tok):
        return env[tok]

    for stmt in SBOX_TOP.split():
        lhs, rhs = stmt.split("=")
        a, b = rhs.split("^")
        ra, rb = ref(a), ref(b)
        if keyed and lhs in KEY_PAIR:
            i, j = KEY_PAIR[lhs]
            t = c.g(n(lhs + "_d"), "xor", ra, rb)
            env[lhs] = c.g(n(lhs), "xor", t, n(f"p{i}{j}"))
        elif keyed and (a.startswith("x") or b.startswith("x")):
            xi = int((a if a.startswith("x") else b)[1:])
            t = c.g(n(lhs + "_d"), "xor", ra, rb)
            env[lhs] = c.g(n(lhs), "xor", t, n(f"k{xi}"))
        else:
            env[lhs] = c.g(n(lhs), "xor", ra, rb)
        corrected.add(lhs)
    # x7 used raw by two ANDs: corrected copy
    if keyed:
        env["X7"] = c.g(n("x7k"), "xor", env["x7"], n("k7"))
    else:
        env["X7"] = env["x7"]
    for stmt in SBOX_MID.split():
        lhs, rhs = stmt.split("=")
        if "~" in rhs:
            a, b = rhs.split("~")
            op = "xnor"
        elif "&" in rhs:
            a, b = rhs.split("&")
            op = "and"
        else:
            a, b = rhs.split("^")
            op = "xor"
        env[lhs] = c.g(n(lhs), op, env[a], env[b])
    outs = [env[f"s{7 - b}"] for b in range(8)]  # s0 is bit 7
    if out_key:
        res = []
        for b in range(8):
            c.inp(n(f"o{b}"), "s")
            res.append(c.g(n(f"r{b}"), "xor", outs[b], n(f"o{b}")))
        return res
    return outs


def column_circuit(last):
    """Output column of a round: inputs a{r}_{b} (byte in row r after
    ShiftRows, bit b), scalars per S-box; outputs o{r}_{b}."""
    c = Circuit()
    s = []
    for r in range(4):
        x = [c.inp(f"a{r}_{7 - i}") for i in range(8)]  # x_i = bit 7 - i
        s.append(add_sbox(c, f"S{r}", x, True, last))
    if last:
        for r in range(4):
            for b in range(8):
                c.outputs.append(s[r][b])
        return c
    u = [[c.g(f"u{r}_{b}", "xor", s[r][b], s[(r + 1) % 4][b]) for b in range(8)] for r in range(4)]
    for r in range(4):
        xt = [u[r][7], None, u[r][1], None, None, u[r][4], u[r][5], u[r][6]]
        for b, lo in ((1, 0), (3, 2), (4, 3)):
            xt[b] = c.g(f"xt{r}_{b}", "xor", u[r][lo], u[r][7])
        for b in range(8):
            p = c.g(f"m{r}_{b}", "xor", xt[b], s[(r + 1) % 4][b])
            c.outputs.append(c.g(f"o{r}_{b}", "xor", p, u[(r + 2) % 4][b]))
    return c


# ------------------------------------------------------------------- mapper --

def truth(op):
    return {"xor": lambda a, b: a ^ b, "and": lambda a, b: a & b,
            "xnor": lambda a, b: ~(a ^ b) & 1}[op]


def map_luts(c, order_seed):
    """Greedy merge/duplicate mapping; returns {node: (leaves, tt)}."""
    kind = c.kind
    lut = {}
    for name, op, a, b in c.gates:
        f = truth(op)
        lut[name] = ([a, b], [f(i >> 1 & 1, i & 1) for i in range(4)])  # tt over leaves bits

    def consumers():
        cons = {}
        for n, (lv, _) in lut.items():
            for l in lv:
                cons.setdefault(l, []).append(n)
        return cons

    def merged(n, m):
        """LUT of m with its leaf n replaced by n's function; None if too big."""
        lm, tm = lut[m]
        ln, tn = lut[n]
        leaves = [l for l in lm if l != n]
        for l in ln:
            if l not in leaves:
                leaves.append(l)
        if len(leaves) > 3 or sum(kind[l] == "s" for l in leaves) > 1:
            return None
        k = len(leaves)
        tt = []
        for v in range(1 << k):
            val = {leaves[i]: (v >> (k - 1 - i)) & 1 for i in range(k)}
            idx = 0
            for l in ln:
                idx = idx << 1 | val[l]
            val[n] = tn[idx]
            idx = 0
            for l in lm:
                idx = idx << 1 | val[l]
            tt.append(tm[idx])
        return leaves, tt

    outs = set(c.outputs)
    rng = random.Random(order_seed)
    changed = True
    while changed:
        changed = False
        cons = consumers()
        names = list(lut)
        rng.shuffle(names)
        for n in names:
            if n in outs or n not in lut:
                continue
            cs = cons.get(n, [])
            if not cs:
                continue
            news = {}
            for m in set(cs):
                r = merged(n, m)
                if r is None:
                    break
                news[m] = r
            else:
                for m, r in news.items():
                    lut[m] = r
                del lut[n]
                changed = True
                cons = consumers()
    # drop dead LUTs
    live, stack = set(), list(outs)
    while stack:
        x = stack.pop()
        if x in live or x not in lut:
            continue
        live.add(x)
        stack.extend(lut[x][0])
    return {n: v for n, v in lut.items() if n in live}


def simulate_circuit(c, vals):
    env = dict(vals)
    for name, op, a, b in c.gates:
        x, y = env[a], env[b]
        env[name] = {"xor": x ^ y, "and": x & y, "xnor": ~(x ^ y) & M32}[op]
    return [env[o] for o in c.outputs]


def lut_eval(leaves, tt, env):
    k = len(leaves)
    res = 0
    for v in range(1 << k):
        if not tt[v]:
            continue
        term = M32
        for i in range(k):
            bit = (v >> (k - 1 - i)) & 1
            x = env[leaves[i]]
            term &= x if bit else ~x & M32
        res |= term
    return res


def topo(c, lut):
    order, seen = [], set()

    def visit(n):
        if n in seen or n not in lut:
            return
        seen.add(n)
        for l in lut[n][0]:
            visit(l)
        order.append(n)

    for o in c.outputs:
        visit(o)
    return order


def check(c, lut, trials=64):
    rng = random.Random(1)
    order = topo(c, lut)
    for _ in range(trials):
        vals = {i: rng.getrandbits(32) for i in c.inputs}
        want = simulate_circuit(c, vals)
        env = dict(vals)
        for n in order:
            env[n] = lut_eval(lut[n][0], lut[n][1], env)
        got = [env[o] for o in c.outputs]
        assert got == want


def best_map(c, tries=40):
    best = None
    for seed in range(tries):
        m = map_luts(c, seed)
        if best is None or len(m) < len(best):
            best = m
    check(c, best)
    return best


# ------------------------------------------------------------------ emitter --

def bitop3_imm(leaves, tt):
    """v_bitop3_b32 immediate with operands (S0, S1, S2) = leaves padded:
    bit index (S0 << 2) | (S1 << 1) | S2 (vpternlog order, checked on gfx950)."""
    k = len(leaves)
    imm = 0
    for idx in range(8):
        s = [(idx >> 2) & 1, (idx >> 1) & 1, idx & 1]
        v = 0
        for i in range(k):
            v = v << 1 | s[i]
        if tt[v]:
            imm |= 1 << idx
    return imm


def emit_fn(c, lut, fname, args_doc, out_names):
    order = topo(c, lut)
    # scalars first among the operands: VOP3 takes at most one scalar, any slot
    ident = {}
    for i in c.inputs:
        ident[i] = i
    lines = []
    for n in order:
        leaves, tt = lut[n]
        ops = [ident[l] for l in leaves]
        imm = bitop3_imm(leaves, tt)
        while len(ops) < 3:
            ops.append("0u")
        lines.append(f"    const uint32_t {n} = QPP_LUT3({ops[0]}, {ops[1]}, {ops[2]}, 0x{imm:02x});")
        ident[n] = n
    return lines, order


def gen():
    blocks = []
    stats = {}
    for last in (False, True):
        c = column_circuit(last)
        lut = best_map(c)
        name = "column_last" if last else "column"
        stats[name] = (len(c.gates), len(lut))
        order = topo(c, lut)
        # group the LUTs per S-box (in S-box order), MixColumns after; fences between
        groups = {r: [] for r in range(5)}
        for n in order:
            groups[int(n[1]) if n.startswith("S") else 4].append(n)
        body = []
        ident = {i: i for i in c.inputs}
        # map input names onto the C arguments
        for r in range(4):
            for b in range(8):
                ident[f"a{r}_{b}"] = f"a[{r}][{b}]"
            for j, w in enumerate(KEY_WORDS):
                ident[f"S{r}{w}"] = f"k[{r * len(KEY_WORDS) + j}]"
            if last:
                for b in range(8):
                    ident[f"S{r}o{b}"] = f"ko[{8 * r + b}]"
        for g in range(5):
            for n in groups[g]:
                leaves, tt = lut[n]
                ops = [ident[l] for l in leaves]
                imm = bitop3_imm(leaves, tt)
                while len(ops) < 3:
                    ops.append("0u")
                body.append(f"    const uint32_t {n} = QPP_LUT3({ops[0]}, {ops[1]}, {ops[2]}, 0x{imm:02x});")
                ident[n] = n
            body.append("    QPP_BS_FENCE_SBOX();" if g < 3 else "    QPP_BS_FENCE();")
        outs = c.outputs
        for i, o in enumerate(outs):
            body.append(f"    o[{i // 8}][{i % 8}] = {ident[o]};")
        if last:
            sig = (f"QPP_BS_HD void {name}(const uint32_t (&a)[4][8], const uint32_t *k, "
                   f"const uint32_t *ko, uint32_t (&o)[4][8])")
        else:
            sig = f"QPP_BS_HD void {name}(const uint32_t (&a)[4][8], const uint32_t *k, uint32_t (&o)[4][8])"
        blocks.append(f"// {len(lut)} LUTs (from {len(c.gates)} two-input gates)\n{sig}\n{{\n" +
                      "\n".join(body) + "\n}\n")
    hdr = f'''// qpp_bs_gen.h -- GENERATED by tools/lutmap.py; do not edit.
//
// One output column of a bitsliced AES round as v_bitop3_b32 operations
// (QPP_LUT3(s0, s1, s2, imm): bit (s0 << 2 | s1 << 1 | s2) of imm).
// a[r][b]: plane of bit b of the input byte in row r of this output column
// (ShiftRows already applied by the caller); k: the {len(KEY_WORDS)} scalar key
// words of each of the four S-boxes (previous round key folded into the
// S-box inputs: {", ".join(KEY_WORDS)}); ko (last round): this round's key
// bits, XORed into the S-box outputs; o[r][b]: output planes.
// column: S-boxes + MixColumns; column_last: S-boxes + output key.
#pragma once

namespace qpp {{
namespace bs {{

constexpr int kKeyWordsPerSbox = {len(KEY_WORDS)};

{chr(10).join(blocks)}
}}  // namespace bs
}}  // namespace qpp
'''
    open(OUT, "w").write(hdr)
    print("wrote", OUT, stats)


if __name__ == "__main__":
    gen()
