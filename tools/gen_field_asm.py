"""Generator for babble_amd/csrc/field_asm.h — hand-scheduled gfx950 field
arithmetic mod p = 2^256 - 2^32 - 977 (secp256k1, src/crypto/keys/curve.go:21).

Why: the compiled C++ field multiply (field.h mul_512 + fe_reduce) lowers to
347 VALU instructions on gfx950, 153 of them v_mov (64-bit operand pairs for
v_mad_u64_u32) and 30 s_nop (VCC carry-chain hazards); fe_add/fe_sub are
55/66 with 22 s_nop each.  rocprofv3 shows the verify kernels are VALU-issue
bound (profiles/r01_pmc_summary.json), so instruction count is the roofline.

Programs emitted:
  fe_sqr  Comba squaring: 28 off-diagonal products once, doubled, plus the
          8 diagonal squares (36 mads instead of 64), then fe_mul's fold.
  fe_mul  product-scanning (Comba) 8x8 using v_mad_u64_u32's carry-out: each
          column accumulates in a 64-bit pair P_k, carry-outs are counted in
          the high word of the next column's pair, so a product costs one mad
          + one addc and a column one v_mov; then the fold 2^256 = 2^32 + 977
          as two interleaved carry chains and a short tail.
          FAST_FIRST: the first product of each counted column does not
          count its carry-out (it would be one addc); the carries are OR-ed
          into one SALU lane mask instead, and a uniform rare block re-runs
          the whole product phase with full counting when any lane carried
          (P ~ 2^-32 per first product on uniform operands; all-ones
          operands take it, tests/test_field_asm.py).  fe_mul 71 -> 58
          addc, fe_sqr 64 -> 52.
  fe_add  s = a + b, then s + c0 (2^32 + 977) on the carry-out c0 into limbs
          0..1 (13 VALU); the carry past limb 1 (~2^-31) and the
          once-in-2^222 second wrap go to nested uniform slow blocks.
  fe_sub  same with borrows and s - c0 (2^32 + 977).

Each program is written in logical order over named registers, then list-
scheduled: an instruction issues once its register dependences (RAW, WAR,
WAW, pairs split into halves) are met and no SGPR it reads as a carry/mask
was written by a VALU fewer than HAZARD_STATES wait states earlier; s_nop is
inserted only when nothing else can issue.  The scheduled list is both
(1) executed by the interpreter here against Python integers
(tests/test_field_asm.py) and (2) printed as the inline-asm block.

    python tools/gen_field_asm.py            # rewrite the header
    python tools/gen_field_asm.py --check    # exit 1 if the header is stale
"""
from __future__ import annotations

import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "babble_amd", "csrc", "field_asm.h")

M32 = (1 << 32) - 1
M64 = (1 << 64) - 1
P = 2**256 - 2**32 - 977
K = 2**32 + 977  # 2^256 mod p
HAZARD_STATES = 2  # VALU writes SGPR -> VALU reads it: 2 wait states (gfx950)
MUL_BASE = 0       # physical VGPR temporaries of fe_mul: v[MUL_BASE, MUL_BASE+34)
MUL_NREGS = 34
NCARRY = 10        # SGPR lane-mask pairs of fe_mul / fe_sqr (%[c0..9])

# ops: name -> (dst-operand positions, src-operand positions, sgpr-src positions)
#   every op: (op, d, ...); positions index into the tuple
OPS = {
    "mad": ((1, 2), (3, 4, 5), ()),        # d64, cy | a, b, c64
    "addc": ((1, 2), (3, 4, 5), (5,)),     # d, cy | a, b, cin
    "add_co": ((1, 2), (3, 4), ()),
    "subb": ((1, 2), (3, 4, 5), (5,)),
    "sub_co": ((1, 2), (3, 4), ()),
    "add": ((1,), (2, 3), ()),
    "mov": ((1,), (2,), ()),
    "cnd": ((1,), (2, 3, 4), (4,)),        # d = mask ? s1 : s0
    "mul24": ((1,), (2, 3), ()),           # d = a * b (24-bit operands)
    "mul_lo": ((1,), (2, 3), ()),          # d = lo32(a * b)
    "alignbit": ((1,), (2, 3), ()),        # d = lo32(({a, b} 64-bit) >> sh), sh = x[4]
    "nop": ((), (), ()),
    "sor": ((1,), (2, 3), (2, 3)),         # SALU s_or_b64 d, a, b (lane masks)
    "slow": ((), (), (1,)),                # uniform branch into x[2] (a Prog) iff any lane of mask x[1]
}


class Prog:
    """A straight-line VALU program over named registers.

    Names: physical VGPR 'v12'; even-aligned pair 'v[12:13]'; asm operands
    '%[x]' (32-bit VGPR operands; '%[c*]' are 64-bit SGPR lane masks).
    Python ints are inline constants or (977) 32-bit literals in v_mov.
    """

    def __init__(self, name: str):
        self.name = name
        self.ins: list[tuple] = []
        self.slow: tuple[str, "Prog"] | None = None  # (mask, block run iff any lane's mask bit)

    def emit(self, *ins):
        assert ins[0] in OPS, ins
        self.ins.append(tuple(ins))

    def mad(self, d, cy, a, b, c):
        self.emit("mad", d, cy, a, b, c)

    def addc(self, d, cy, a, b, cin):
        self.emit("addc", d, cy, a, b, cin)

    def add_co(self, d, cy, a, b):
        self.emit("add_co", d, cy, a, b)

    def subb(self, d, cy, a, b, bin_):
        self.emit("subb", d, cy, a, b, bin_)

    def sub_co(self, d, cy, a, b):
        self.emit("sub_co", d, cy, a, b)

    def add(self, d, a, b):
        self.emit("add", d, a, b)

    def mov(self, d, s):
        self.emit("mov", d, s)

    def cnd(self, d, s0, s1, mask):
        self.emit("cnd", d, s0, s1, mask)

    def mul24(self, d, a, b):
        self.emit("mul24", d, a, b)

    def mul_lo(self, d, a, b):
        self.emit("mul_lo", d, a, b)

    def alignbit(self, d, hi, lo, sh):
        self.emit("alignbit", d, hi, lo, sh)

    def sor(self, d, a, b):
        self.emit("sor", d, a, b)

    def slow_block(self, mask, blk: "Prog"):
        """Mid-program rare block: run (by the whole wave) iff some lane's
        `mask` bit is set; it must be a no-op for lanes without the bit."""
        self.emit("slow", mask, blk)


# ---------------------------------------------------------------------------
# registers
# ---------------------------------------------------------------------------
def v(n: int) -> str:
    return f"v{n}"


def pair(lo: str) -> str:
    n = int(lo[1:])
    assert lo[0] == "v" and n % 2 == 0, lo
    return f"v[{n}:{n + 1}]"


def is_pair(x) -> bool:
    return isinstance(x, str) and x.startswith("v[")


def halves(x) -> list[str]:
    if is_pair(x):
        a, b = x[2:-1].split(":")
        return [f"v{a}", f"v{b}"]
    if isinstance(x, str):
        return [x]
    return []


def is_sgpr(x) -> bool:
    """SGPR lane masks: %[cN] (and %[zKcN] in zipped programs)."""
    return isinstance(x, str) and re.fullmatch(r"%\[(z\d+)?c\d+\]", x) is not None


def reads(ins) -> list[str]:
    out = []
    for p in OPS[ins[0]][1]:
        out += halves(ins[p])
    return out


def writes(ins) -> list[str]:
    out = []
    for p in OPS[ins[0]][0]:
        out += halves(ins[p])
    return out


def sgpr_reads(ins) -> list[str]:
    return [ins[p] for p in OPS[ins[0]][2] if is_sgpr(ins[p])]


# ---------------------------------------------------------------------------
# list scheduler with the SGPR hazard
# ---------------------------------------------------------------------------
BRANCH_STATES = 2  # s_cmp_lg_u64 + s_cbranch_scc0 between the blocks


def _block_sgpr_writes(blk: Prog) -> set[str]:
    out: set[str] = set()
    for x in blk.ins:
        if x[0] == "slow":
            out |= _block_sgpr_writes(x[2])
            continue
        out |= {x[p] for p in OPS[x[0]][0] if is_sgpr(x[p])}
    if blk.slow is not None:
        out |= _block_sgpr_writes(blk.slow[1])
    return out


SALU_OPS = {"sor"}


def _note_sgpr_writes(x: tuple, wtime: dict[str, int], t: int) -> None:
    """Record the SGPRs x writes: a VALU write starts the hazard window
    (the next VALU or SALU read waits HAZARD_STATES); an SALU write does
    not (SALU results are interlocked), so it clears the entry."""
    for p in OPS[x[0]][0]:
        if is_sgpr(x[p]):
            if x[0] in SALU_OPS:
                wtime.pop(x[p], None)
            else:
                wtime[x[p]] = t


def _sched_segment(ins: list[tuple], out: Prog, t: int, sgpr_wtime: dict[str, int]) -> int:
    """List-schedule a straight-line segment into `out`; returns the clock."""
    n = len(ins)
    preds: list[set[int]] = [set() for _ in range(n)]
    last_w: dict[str, int] = {}
    last_r: dict[str, list[int]] = {}
    for j, x in enumerate(ins):
        for r in reads(x):
            if r in last_w:
                preds[j].add(last_w[r])
        for w in writes(x):
            if w in last_w:
                preds[j].add(last_w[w])
            for i in last_r.get(w, []):
                if i != j:
                    preds[j].add(i)
        for r in reads(x):
            last_r.setdefault(r, []).append(j)
        for w in writes(x):
            last_w[w] = j
            last_r[w] = []
    done = [False] * n
    remaining = n
    while remaining:
        pick = None
        for j in range(n):
            if done[j] or any(not done[i] for i in preds[j]):
                continue
            if all(t - sgpr_wtime.get(s, -99) >= HAZARD_STATES for s in sgpr_reads(ins[j])):
                pick = j
                break
        if pick is None:
            out.emit("nop")
            t += 1
            continue
        x = ins[pick]
        out.ins.append(x)
        t += 1
        _note_sgpr_writes(x, sgpr_wtime, t)
        done[pick] = True
        remaining -= 1
    return t


def schedule(g: Prog, ages: dict[str, int] | None = None) -> Prog:
    """List-schedule g.ins; `ages` = wait states already elapsed since each
    SGPR's last VALU write at entry (for a slow block after a branch).
    Mid-program slow blocks split the program into segments; after one, the
    SGPRs it may write count as written at the resume point (conservative
    for both the taken and the skipped path)."""
    out = Prog(g.name)
    t = 0
    sgpr_wtime: dict[str, int] = {k: -a for k, a in (ages or {}).items()}
    seg: list[tuple] = []
    for x in g.ins + [None]:
        if x is not None and x[0] != "slow":
            seg.append(x)
            continue
        t = _sched_segment(seg, out, t, sgpr_wtime)
        seg = []
        if x is None:
            break
        mask, blk = x[1], x[2]
        entry = {k: t - w + BRANCH_STATES for k, w in sgpr_wtime.items()}
        out.ins.append(("slow", mask, schedule(blk, entry)))
        t += BRANCH_STATES
        for sg in _block_sgpr_writes(blk):
            sgpr_wtime[sg] = t
    if g.slow is not None:
        mask, blk = g.slow
        exit_ages = {k: t - w + BRANCH_STATES for k, w in sgpr_wtime.items()}
        out.slow = (mask, schedule(blk, exit_ages))
    return out


def check_hazards(g: Prog, wt: dict[str, int] | None = None, t: int = 0) -> None:
    wt = dict(wt or {})
    for x in g.ins:
        if x[0] == "slow":
            check_hazards(x[2], wt, t + BRANCH_STATES)
            t += BRANCH_STATES
            for sg in _block_sgpr_writes(x[2]):
                wt[sg] = t
            continue
        t += 1
        if x[0] == "nop":
            continue
        for s in sgpr_reads(x):
            assert t - 1 - wt.get(s, -99) >= HAZARD_STATES, (g.name, x, t, wt.get(s))
        _note_sgpr_writes(x, wt, t)
    if g.slow is not None:
        check_hazards(g.slow[1], wt, t + BRANCH_STATES)


# ---------------------------------------------------------------------------
# interpreter (one lane)
# ---------------------------------------------------------------------------
class Machine:
    def __init__(self):
        self.r: dict[str, int] = {}
        self.hits: dict[str, int] = {}  # mid-program slow blocks entered (by program name)

    def get(self, x) -> int:
        if isinstance(x, int):
            return x & M32  # inline constants -16..64 are 32-bit sign-extended
        if is_pair(x):
            lo, hi = halves(x)
            return self.get(lo) | (self.get(hi) << 32)
        if x not in self.r:
            raise KeyError(f"read of undefined register {x}")
        return self.r[x]

    def put(self, x, val: int):
        if is_pair(x):
            lo, hi = halves(x)
            self.r[lo] = val & M32
            self.r[hi] = (val >> 32) & M32
        else:
            self.r[x] = val

    def run(self, g: Prog, force_slow: bool = False):
        self._run(g, force_slow)
        if g.slow is not None:
            mask, blk = g.slow
            if force_slow or self.get(mask):
                self.run(blk, force_slow)

    def _run(self, g: Prog, force_slow: bool = False):
        for x in g.ins:
            op = x[0]
            if op == "nop":
                continue
            if op == "slow":
                self.hits[g.name] = self.hits.get(g.name, 0) + bool(self.get(x[1]))
                if force_slow or self.get(x[1]):
                    self.run(x[2], force_slow)
                continue
            if op == "sor":
                self.put(x[1], 1 if (self.get(x[2]) or self.get(x[3])) else 0)
                continue
            if op == "mad":
                s = self.get(x[3]) * self.get(x[4]) + self.get(x[5])
                self.put(x[1], s & M64)
                self.put(x[2], s >> 64)
            elif op in ("addc", "add_co"):
                s = self.get(x[3]) + self.get(x[4]) + (self.get(x[5]) if op == "addc" else 0)
                self.put(x[1], s & M32)
                self.put(x[2], s >> 32)
            elif op in ("subb", "sub_co"):
                s = self.get(x[3]) - self.get(x[4]) - (self.get(x[5]) if op == "subb" else 0)
                self.put(x[1], s & M32)
                self.put(x[2], 1 if s < 0 else 0)
            elif op == "add":
                self.put(x[1], (self.get(x[2]) + self.get(x[3])) & M32)
            elif op == "mov":
                self.put(x[1], self.get(x[2]))
            elif op == "cnd":
                self.put(x[1], self.get(x[3]) if self.get(x[4]) else self.get(x[2]))
            elif op == "mul_lo":
                self.put(x[1], (self.get(x[2]) * self.get(x[3])) & M32)
            elif op == "alignbit":
                self.put(x[1], (((self.get(x[2]) << 32) | self.get(x[3])) >> x[4]) & M32)
            elif op == "mul24":
                a, b = self.get(x[2]), self.get(x[3])
                assert a < 2**24 and b < 2**24
                self.put(x[1], (a * b) & M32)
            else:
                raise ValueError(op)


# ---------------------------------------------------------------------------
# programs (logical order; schedule() interleaves)
# ---------------------------------------------------------------------------
CY = ["%[c0]", "%[c1]", "%[c2]", "%[c3]"]


# The carry of a column's FIRST product: its 64-bit addend is the previous
# column's high word plus 2^32 times that column's carry count c, so
# a b + addend < 2^64 unless c >= 2 (or c = 1 with a full high word) AND
# a b is within ~c 2^32 of 2^64 — both limbs within a few units of 2^32.
# Random operands never do that; crafted ones can.  So the fast product
# phase does not count first-product carries (13 of fe_mul's 71 carry
# instructions, 12 of fe_sqr's 64; a carry-writing VALU op costs 4.7-4.9
# cycles, profiles/r03_ubench_ops.txt) but ORs them into RARE (SALU), and a
# uniform rare block re-runs the product phase with every carry counted
# (from the inputs, which are still live: outputs are written in the fold).
FAST_FIRST = True
RARE = "%[c8]"  # free during the product phases (the fold's CANY, written after)


def _mul_product(g: Prog, base: int, fast: bool):
    A = [f"%[a{i}]" for i in range(8)]
    B = [f"%[b{i}]" for i in range(8)]
    Pl = [v(base + 2 * k) for k in range(15)]
    Ph = [v(base + 2 * k + 1) for k in range(15)]
    PP = [pair(x) for x in Pl]
    first = True
    for k in range(15):
        terms = [(i, k - i) for i in range(8) if 0 <= k - i < 8]
        src = 0 if k == 0 else PP[k]
        counted = 0 < k < 14  # col 0 (src 0) and col 14 (top) cannot carry
        c2 = Ph[k + 1] if k < 14 else None
        for j, (i, jj) in enumerate(terms):
            cy = CY[j % 3]
            # first product with a check: the first one writes the mask itself
            direct = fast and counted and j == 0 and k > 1 and first
            g.mad(PP[k], RARE if direct else cy, A[i], B[jj], src)
            src = PP[k]
            if not counted:
                continue
            if fast and j == 0:  # first product: only the rare mask
                # column 1's addend is {w_0 hi, 0} < 2^32: a b + addend < 2^64
                if k > 1 and not direct:
                    g.sor(RARE, cy, RARE)
                first = first and not direct
            else:
                g.addc(c2, cy, 0 if j == (1 if fast else 0) else c2, 0, cy)
        if k < 14:
            g.mov(Pl[k + 1], Ph[k])
            if not counted:
                g.mov(c2, 0)
        if k >= 8:
            g.mov(Ph[k - 8], Pl[k])  # P_(k-8) = {w_(k-8), w_k} for the fold
    g.mov(Ph[7], Ph[14])             # P_7 = {w_7, w_15}
    return Pl, Ph, PP


def gen_mul(base: int = MUL_BASE) -> Prog:
    """r = a * b mod p, weakly reduced (< 2^256).
    Operands %[a0..7], %[b0..7] -> %[r0..7]; physical temporaries
    v[base, base+34); carries %[c0..3]; RARE %[c8] during the product."""
    g = Prog("fe_mul")
    R = [f"%[r{i}]" for i in range(8)]
    Pl, Ph, PP = _mul_product(g, base, FAST_FIRST)
    if FAST_FIRST:
        blk = Prog("fe_mul_recount")
        _mul_product(blk, base, False)
        g.slow_block(RARE, blk)
    return _fold(g, base, R, Pl, Ph, PP)


def _fold(g: Prog, base: int, R, Pl, Ph, PP) -> Prog:
    """Reduce the 512-bit value w_0..w_15 mod p into %[r0..7] (weak).
    Entry: P_i = {w_i, w_(i+8)} for i < 8 (so P_i as a 64-bit value is
    w_i + 2^32 w_(i+8)), and w_(i+8) also in P_(i+8).lo (i < 7) / P_14.hi.

    2^256 = 2^32 + 977 (mod p), so limb i of the folded value collects
    w_i + 977 w_(i+8) + 2^32 w_(i+8): ONE mad per limb,
        Y_i = w_(i+8) * 977 + P_i         (65 bits: carry-out y_i, rare),
    then one carry chain R_i = Y_i.lo + Y_(i-1).hi (+ carry), R_8 = Y_7.hi.
    y_i (weight 2^(32(i+2)); P(set) ~ 2^-22 per limb) is added in a
    uniform rare block entered iff some lane has one.  Then R_8 (+ c9 2^32)
    is folded once more into limbs 0..2 and a rare tail propagates."""
    T0, T1, T2, T3 = v(base + 30), v(base + 31), v(base + 32), v(base + 33)
    K977 = T2
    YC = [f"%[c{i}]" for i in range(8)]
    CANY, cR = "%[c8]", "%[c9]"
    H = [Pl[i + 8] for i in range(7)] + [Ph[14]]

    # logical order interleaves the chain with the mads and the SALU ORs,
    # so each chain link's carry hazard is covered without s_nop
    g.mov(K977, 977)
    g.mad(PP[0], YC[0], H[0], K977, PP[0])
    g.mad(PP[1], YC[1], H[1], K977, PP[1])
    g.sor(CANY, YC[0], YC[1])
    g.add_co(R[1], cR, Pl[1], Ph[0])
    for i in range(2, 8):
        g.mad(PP[i], YC[i], H[i], K977, PP[i])
        g.sor(CANY, CANY, YC[i])
        g.addc(R[i], cR, Pl[i], Ph[i - 1], cR)
    g.addc(T1, cR, Ph[7], 0, cR)            # R_8; cR = c9 (weight 2^288)

    # ---- rare: y_i -> limb i + 2 (limb 8 = R_8 in T1); the carry out of
    # limb 8 and y_7 both have weight 2^288: at most one of c9, y_7 and that
    # carry is set (each forces R_8 small), so c9 |= y_7 | carry.
    s = Prog(g.name + "_ycarry")
    cS = CANY
    limbs = [R[2], R[3], R[4], R[5], R[6], R[7], T1]
    XT = [Ph[8], Ph[9]]                     # free since the product phase
    for i in range(7):
        x = XT[i % 2]
        s.cnd(x, 0, 1, YC[i])
        if i == 0:
            s.add_co(limbs[0], cS, limbs[0], x)
        else:
            s.addc(limbs[i], cS, limbs[i], x, cS)
    s.sor(cR, cR, YC[7])
    s.sor(cR, cR, cS)
    g.slow_block(CANY, s)

    # ---- fold 1: add (R_8 + c9 2^32)(2^32 + 977) ----
    TT = pair(T0)
    cE = CY[0]
    g.mov(T0, 0)
    g.mad(TT, cE, T1, T2, TT)               # E = 977 R_8 + 2^32 R_8 (+ cE 2^64)
    g.cnd(T3, 0, T2, cR)                    # 977 c9 -> limb 1
    g.add(T1, T1, T3)
    g.cnd(T3, 0, 1, cE)                     # limb 2: cE | c9 (exclusive)
    g.cnd(T3, T3, 1, cR)
    cF = CY[1]
    g.add_co(R[0], cF, Pl[0], T0)
    g.addc(R[1], cF, R[1], T1, cF)
    g.addc(R[2], cF, R[2], T3, cF)
    # ---- rare tail (uniform branch, taken iff some lane carried out of
    # limb 2): propagate into limbs 3..7; if that wraps past 2^256 (value is
    # then < 2^66) add 2^32 + 977 once more.  A no-op for lanes without the
    # carry, so the whole wave may run it.
    t = Prog(g.name + "_tail")
    for i in range(3, 8):
        t.addc(R[i], cF, R[i], 0, cF)
    t.cnd(T3, 0, T2, cF)
    t.cnd(T1, 0, 1, cF)
    cG = CY[2]
    t.add_co(R[0], cG, R[0], T3)
    t.addc(R[1], cG, R[1], T1, cG)
    t.addc(R[2], cG, R[2], 0, cG)
    g.slow = (cF, t)
    return g


def _sqr_offdiag(g: Prog, base: int, fast: bool):
    A = [f"%[a{i}]" for i in range(8)]
    Pl = [v(base + 2 * k) for k in range(15)]
    Ph = [v(base + 2 * k + 1) for k in range(15)]
    PP = [pair(x) for x in Pl]
    first = True
    for k in range(1, 14):
        terms = [(i, k - i) for i in range(8) if i < k - i <= 7]
        src = 0 if k == 1 else PP[k]
        counted = k > 1  # column 1: one product, zero addend: no carry
        c2 = Ph[k + 1]
        for j, (i, jj) in enumerate(terms):
            cy = CY[j % 3]
            direct = fast and counted and j == 0 and k > 2 and first
            g.mad(PP[k], RARE if direct else cy, A[i], A[jj], src)
            src = PP[k]
            if not counted:
                continue
            if fast and j == 0:
                # column 2's addend is {column 1 hi, 0} < 2^32: no carry
                if k > 2 and not direct:
                    g.sor(RARE, cy, RARE)
                first = first and not direct
                if len(terms) == 1:
                    g.mov(c2, 0)
            else:
                g.addc(c2, cy, 0 if j == (1 if fast else 0) else c2, 0, cy)
        if not counted:
            g.mov(c2, 0)
        g.mov(Pl[k + 1], Ph[k])


def gen_sqr(base: int = MUL_BASE) -> Prog:
    """r = a^2 mod p, weakly reduced.  Comba squaring: the 28 off-diagonal
    products a_i a_j (i < j) once, in the column scheme of gen_mul; then
    W = 2 D + sum a_i^2 2^(64 i) as a doubling carry chain and a diagonal
    carry chain; then the same fold.  36 mads instead of 64."""
    g = Prog("fe_sqr")
    A = [f"%[a{i}]" for i in range(8)]
    R = [f"%[r{i}]" for i in range(8)]
    Pl = [v(base + 2 * k) for k in range(15)]
    Ph = [v(base + 2 * k + 1) for k in range(15)]
    PP = [pair(x) for x in Pl]
    T01, T23 = pair(v(base + 30)), pair(v(base + 32))

    # ---- off-diagonal D = sum_{i<j} a_i a_j 2^(32(i+j)): columns 1..13
    # (first-product carries as in gen_mul: a rare re-count) ----
    _sqr_offdiag(g, base, FAST_FIRST)
    if FAST_FIRST:
        blk = Prog("fe_sqr_recount")
        _sqr_offdiag(blk, base, False)
        g.slow_block(RARE, blk)
    # D: d_0 = 0, d_m = P_m.lo (1 <= m <= 14), d_15 = P_14.hi
    Dw = [None] + [Pl[m] for m in range(1, 15)] + [Ph[14]]

    # ---- E = 2 D (carry chain, 2 D < 2^512; it interleaves with the
    # diagonal chain below, so the carry hazards need no s_nop) ----
    cE = CY[0]
    g.add_co(Dw[1], cE, Dw[1], Dw[1])
    for m in range(2, 16):
        g.addc(Dw[m], cE, Dw[m], Dw[m], cE)

    # ---- W = E + sum a_i^2 2^(64 i) ----
    cQ = CY[1]
    g.mad(PP[0], CY[3], A[0], A[0], 0)           # w_0, and a_0^2 hi -> w_1
    g.add_co(Dw[1], cQ, Dw[1], Ph[0])
    for i in range(1, 8):
        tp = T01 if i % 2 else T23
        tl, th = halves(tp)
        g.mad(tp, CY[2] if i % 2 else CY[3], A[i], A[i], 0)
        g.addc(Dw[2 * i], cQ, Dw[2 * i], tl, cQ)
        g.addc(Dw[2 * i + 1], cQ, Dw[2 * i + 1], th, cQ)
    for i in range(8):
        g.mov(Ph[i], Dw[i + 8])  # P_i = {w_i, w_(i+8)} for the fold
    return _fold(g, base, R, Pl, Ph, PP)


def _addsub(name: str, sub: bool) -> Prog:
    """r = a +/- b mod p, weakly reduced.  Chain s = a +/- b (carry c0);
    then s -/+ (c0 ? 0 : K)... i.e. on a wrap past 2^256 apply
    K = 2^256 - p = 2^32 + 977 once to limbs 0..1 (carry c1): 13 VALU.  The
    carry past limb 1 (~2^-31 per lane) is propagated through limbs 2..7
    in a uniform rare block entered iff some lane's c1 is set; only a
    result within K of the wrap carries out of limb 7 (probability ~2^-222
    for random operands) and needs K applied once more (a nested rare
    block).  Before the propagation block: 19 VALU."""
    g = Prog(name)
    A = [f"%[a{i}]" for i in range(8)]
    B = [f"%[b{i}]" for i in range(8)]
    R = [f"%[r{i}]" for i in range(8)]
    k0, k1 = "%[k0]", "%[k1]"
    c0, c1, c2 = CY[0], CY[1], CY[2]
    first = g.sub_co if sub else g.add_co
    nxt = g.subb if sub else g.addc
    first(R[0], c0, A[0], B[0])
    for i in range(1, 8):
        nxt(R[i], c0, A[i], B[i], c0)
    g.mov(k1, 977)
    g.cnd(k0, 0, k1, c0)                     # 977 c0
    g.cnd(k1, 0, 1, c0)                      # c0 (limb 1 of K c0)
    first(R[0], c1, R[0], k0)
    nxt(R[1], c1, R[1], k1, c1)
    # The carry of K's two limbs past limb 1 needs limbs 0..1 of the wrapped
    # value within K of 2^64 (~2^-31 per lane): propagating it into limbs
    # 2..7 is a rare block (a no-op for lanes without c1), not six
    # unconditional links of every add / sub.
    p = Prog(name + "_prop")
    pn = p.subb if sub else p.addc
    for i in range(2, 8):
        pn(R[i], c1, R[i], 0, c1)
    s = Prog(name + "_tail")
    sf = s.sub_co if sub else s.add_co
    sn = s.subb if sub else s.addc
    s.mov(k1, 977)
    s.cnd(k0, 0, k1, c1)
    s.cnd(k1, 0, 1, c1)
    sf(R[0], c2, R[0], k0)
    sn(R[1], c2, R[1], k1, c2)
    for i in range(2, 8):
        sn(R[i], c2, R[i], 0, c2)
    p.slow = (c1, s)
    g.slow = (c1, p)
    return g


def gen_add() -> Prog:
    return _addsub("fe_add", sub=False)


def gen_sub() -> Prog:
    return _addsub("fe_sub", sub=True)




# secp256k1 group order N (curve.go:13) and Montgomery constants (R = 2^256)
N_ORDER = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
N_LIMBS = [(N_ORDER >> (32 * i)) & M32 for i in range(8)]
N_C = 2**256 - N_ORDER  # 129 bits
N_C_LIMBS = [(N_C >> (32 * i)) & M32 for i in range(8)]
NINV = (-pow(N_ORDER, -1, 2**32)) % 2**32
MONT_BASE = 0
MONT_NREGS = 32


def _nlimb(j: int):
    """N_j as an operand: the low four limbs come in VGPR operands, the high
    four (0xFFFFFFFE, 0xFFFFFFFF x3) are the inline constants -2 / -1."""
    return f"%[n{j}]" if j < 4 else (-2 if N_LIMBS[j] == 0xFFFFFFFE else -1)


def gen_mont(base: int = MONT_BASE) -> Prog:
    """r = a * b * 2^-256 mod N (Montgomery, product scanning / FIPS), for
    a * b < N 2^256 (a < 2^256, b < N); output < N.  Operands %[a0..7],
    %[b0..7], %[n0..3] (N's low limbs), %[nc0..3] (2^256 - N low limbs),
    %[ninv] (-N^-1 mod 2^32) -> %[r0..7].  Temporaries v[base, base+32):
    column pairs P_0..P_15; m_k lives in P_{k+8}.lo until column k+7 ends."""
    g = Prog("sc_mont")
    A = [f"%[a{i}]" for i in range(8)]
    B = [f"%[b{i}]" for i in range(8)]
    R = [f"%[r{i}]" for i in range(8)]
    Pl = [v(base + 2 * k) for k in range(16)]
    Ph = [v(base + 2 * k + 1) for k in range(16)]
    PP = [pair(x) for x in Pl]
    M = [Pl[k + 8] for k in range(8)]
    for k in range(15):
        ab = [(A[i], B[k - i]) for i in range(8) if 0 <= k - i < 8]
        mn = [(M[i], _nlimb(k - i)) for i in range(8) if 0 <= k - i < 8 and i < k]
        terms = ab + mn
        src = 0 if k == 0 else PP[k]
        c2 = Ph[k + 1]
        nprod = 0
        for j, (x, y) in enumerate(terms):
            cy = CY[nprod % 3]
            g.mad(PP[k], cy, x, y, src)
            if src != 0:
                g.addc(c2, cy, 0 if nprod == 0 or (nprod == 1 and k == 0) else c2, 0, cy)
            elif k == 0:
                pass
            src = PP[k]
            nprod += 1
        if k < 8:
            g.mul_lo(M[k], Pl[k], "%[ninv]")
            cy = CY[nprod % 3]
            g.mad(PP[k], cy, M[k], _nlimb(0), PP[k])   # low word becomes 0
            g.addc(c2, cy, 0 if k == 0 else c2, 0, cy)
        g.mov(Pl[k + 1], Ph[k])
    # T = t_0..t_7 (+ t_8 = P_15.hi in {0,1}), T < 2N; t_j = P_{8+j}.lo, t_7 = P_15.lo
    T = [Pl[8 + j] for j in range(8)]
    t8 = Ph[15]
    # D = T + (2^256 - N): carry-out | t_8  <=>  T >= N; then r = sel ? D : T
    D = [Pl[j] for j in range(8)]
    cD = CY[0]
    NC = ["%[nc0]", "%[nc1]", "%[nc2]", "%[nc3]", 1, 0, 0, 0]
    g.add_co(D[0], cD, T[0], NC[0])
    for j in range(1, 8):
        g.addc(D[j], cD, T[j], NC[j], cD)
    g.addc(Ph[0], cD, t8, 0, cD)                 # t_8 + carry in {0, 1}
    sel = CY[1]
    g.sub_co(Ph[1], sel, 0, Ph[0])                # borrow <=> value != 0
    for j in range(8):
        g.cnd(R[j], T[j], D[j], sel)
    return g


PROGRAMS = {"fe_mul": gen_mul, "fe_sqr": gen_sqr, "fe_add": gen_add, "fe_sub": gen_sub, "sc_mont": gen_mont}


# ---------------------------------------------------------------------------
# zipped programs: K independent multiplies in one asm block (latency-bound
# single-wave chains: the per-key doubling chain of k_table_bases)
# ---------------------------------------------------------------------------
# A lone wave issues a dependent VALU instruction only every ~2x its issue
# cost (tools/ubench_lat.hip); the serial doubling chain of the key-table
# bases runs one wave per 64 keys, so it is latency bound.  Interleaving the
# independent multiplies of one doubling (dbl-2009-l: {X^2, Y^2, Y Z} then
# {B^2, (X+B)^2, E^2}) fills those slots: each program keeps its own
# physical temporaries (v[34 k, 34 k + 34)) and carry SGPRs.  The mixed
# addition's eleven multiplies form five levels the same way
# ({Z^2} -> {x Z1Z1, Z Z1Z1} -> {y t, H^2} -> {H HH, X HH, Z H, R^2} ->
# {R (V - X3), Y HHH}): the verify kernels' latency variant (small batches,
# one or two waves per SIMD) uses them.
ZIP_KINDS = {"mul": gen_mul, "sqr": gen_sqr}
ZIP_COMBOS = [("sqr", "sqr", "mul"), ("sqr", "sqr", "sqr"),      # gej_double_lat
              ("mul", "mul"), ("mul", "sqr"), ("mul", "mul", "mul", "sqr"),  # gej_add_ge_lat
              ("sqr", "sqr"), ("mul", "mul", "mul")]  # gexz_add_ge_lat (with ("mul", "mul"))


def _rename(g: Prog, f) -> Prog:
    """Copy of g with every asm operand name passed through f; the tail
    block becomes a trailing mid-program slow block (same semantics: run iff
    some lane's mask bit is set, a no-op for the other lanes)."""
    def op(x):
        return f(x) if isinstance(x, str) and x.startswith("%[") else x

    out = Prog(g.name)
    for x in g.ins:
        if x[0] == "slow":
            out.ins.append(("slow", op(x[1]), _rename(x[2], f)))
        else:
            out.ins.append(tuple([x[0]] + [op(y) for y in x[1:]]))
    if g.slow is not None:
        out.ins.append(("slow", op(g.slow[0]), _rename(g.slow[1], f)))
    return out


def _segments(g: Prog) -> list[tuple[list, tuple | None]]:
    segs, cur = [], []
    for x in g.ins:
        if x[0] == "slow":
            segs.append((cur, (x[1], x[2])))
            cur = []
        else:
            cur.append(x)
    segs.append((cur, None))
    return segs


def zip_name(kinds) -> str:
    return "fe_" + "_".join(kinds) + "_zip"


def gen_zip(kinds) -> Prog:
    """Programs kinds[k] over operands %[z{k}a*], %[z{k}b*] -> %[z{k}r*],
    carries %[z{k}c*], temporaries v[34 k, 34 k + 34); the instruction
    streams are merged segment by segment in proportion to their lengths
    (the list scheduler keeps that order where dependences allow) and each
    program's rare blocks follow its segment."""
    progs = []
    for k, kind in enumerate(kinds):
        g = ZIP_KINDS[kind](base=MUL_NREGS * k)
        progs.append(_rename(g, lambda x, k=k: f"%[z{k}{x[2:]}"))
    segs = [_segments(p) for p in progs]
    out = Prog(zip_name(kinds))
    for si in range(max(len(s) for s in segs)):
        keyed = []
        for k, s in enumerate(segs):
            part = s[si][0] if si < len(s) else []
            keyed += [((j + 0.5) / len(part), k, x) for j, x in enumerate(part)]
        keyed.sort(key=lambda t: (t[0], t[1]))
        out.ins += [x for _, _, x in keyed]
        for s in segs:
            if si < len(s) and s[si][1] is not None:
                out.ins.append(("slow",) + s[si][1])
    return out


def build(name: str) -> Prog:
    for kinds in ZIP_COMBOS:
        if name == zip_name(kinds):
            g = schedule(gen_zip(kinds))
            check_hazards(g)
            return g
    g = schedule(PROGRAMS[name]())
    check_hazards(g)
    return g


# ---------------------------------------------------------------------------
# printer
# ---------------------------------------------------------------------------
def fmt(x) -> str:
    if isinstance(x, int):
        return str(x)
    return x


def asm_line(x) -> str:
    op = x[0]
    if op == "nop":
        return "s_nop 0"
    if op == "mad":
        return f"v_mad_u64_u32 {fmt(x[1])}, {fmt(x[2])}, {fmt(x[3])}, {fmt(x[4])}, {fmt(x[5])}"
    if op == "addc":
        return f"v_addc_co_u32_e64 {x[1]}, {x[2]}, {fmt(x[3])}, {fmt(x[4])}, {x[5]}"
    if op == "add_co":
        return f"v_add_co_u32_e64 {x[1]}, {x[2]}, {fmt(x[3])}, {fmt(x[4])}"
    if op == "subb":
        return f"v_subb_co_u32_e64 {x[1]}, {x[2]}, {fmt(x[3])}, {fmt(x[4])}, {x[5]}"
    if op == "sub_co":
        return f"v_sub_co_u32_e64 {x[1]}, {x[2]}, {fmt(x[3])}, {fmt(x[4])}"
    if op == "add":
        return f"v_add_u32_e64 {x[1]}, {fmt(x[2])}, {fmt(x[3])}"
    if op == "mov":
        return f"v_mov_b32_e32 {x[1]}, {fmt(x[2])}"
    if op == "cnd":
        return f"v_cndmask_b32_e64 {x[1]}, {fmt(x[2])}, {fmt(x[3])}, {x[4]}"
    if op == "mul24":
        return f"v_mul_u32_u24_e64 {x[1]}, {fmt(x[2])}, {fmt(x[3])}"
    if op == "mul_lo":
        return f"v_mul_lo_u32 {x[1]}, {fmt(x[2])}, {fmt(x[3])}"
    if op == "alignbit":
        return f"v_alignbit_b32 {x[1]}, {fmt(x[2])}, {fmt(x[3])}, {x[4]}"
    if op == "sor":
        return f"s_or_b64 {x[1]}, {x[2]}, {x[3]}"
    raise ValueError(op)


def asm_body(g: Prog) -> str:
    """Consecutive wait states are merged into one s_nop N (N + 1 states):
    one issue slot instead of N + 1."""
    lines = []
    run = 0
    for k, x in enumerate(g.ins + [("end",)]):
        if x[0] == "nop":
            run += 1
            continue
        while run:
            m = min(run, 8)  # s_nop takes 0..7 (1..8 wait states)
            lines.append(f'      "s_nop {m - 1}\\n"')
            run -= m
        if x[0] == "end":
            break
        if x[0] == "slow":
            lbl = f"BV_{g.name.upper()}_S{k}_%="
            lines.append(f'      "s_cmp_lg_u64 {x[1]}, 0\\n"')
            lines.append(f'      "s_cbranch_scc0 {lbl}\\n"')
            lines.append(asm_body(x[2]))
            lines.append(f'      "{lbl}:\\n"')
            continue
        lines.append(f'      "{asm_line(x)}\\n"')
    if g.slow is not None:
        mask, blk = g.slow
        lines.append(f'      "s_cmp_lg_u64 {mask}, 0\\n"')
        lines.append(f'      "s_cbranch_scc0 BV_{g.name.upper()}_SKIP_%=\\n"')
        lines.append(asm_body(blk))
        lines.append(f'      "BV_{g.name.upper()}_SKIP_%=:\\n"')
    return "\n".join(lines)


def stats(g: Prog) -> dict:
    from collections import Counter

    c = Counter(x[0] for x in g.ins if x[0] != "slow")
    out = dict(c)
    mids = [len(x[2].ins) for x in g.ins if x[0] == "slow"]
    if mids:
        out["rare_mid"] = mids
    if g.slow is not None:
        out["rare_tail"] = len(g.slow[1].ins)
    return out


def _all_reads(g: Prog) -> list[tuple]:
    out = []
    for x in g.ins:
        if x[0] == "slow":
            out += _all_reads(x[2])
        else:
            out.append(x)
    if g.slow is not None:
        out += _all_reads(g.slow[1])
    return out


def outputs_after_inputs(g: Prog) -> bool:
    """True when every read of an input operand (%[a*] / %[b*], zipped
    %[zKa*] / %[zKb*]) precedes every write of an output (%[r*] / %[zKr*])
    in program order (rare blocks included, at their position).  The
    outputs may then share registers with inputs that die at the asm
    statement (no early-clobber "&"): the register allocator gets up to 8
    VGPRs per multiply back at the verify kernels' 128-VGPR budget."""
    seq = _all_reads(g)
    is_in = re.compile(r"%\[(z\d+)?[ab]\d+\]")
    is_out = re.compile(r"%\[(z\d+)?r\d+\]")
    last_in = max((i for i, x in enumerate(seq) if any(is_in.fullmatch(r) for r in reads(x))), default=-1)
    first_out = min((i for i, x in enumerate(seq) if any(is_out.fullmatch(w) for w in writes(x))), default=len(seq))
    return last_in < first_out


def zip_wrapper(kinds) -> str:
    """C++ wrapper of a zipped program: fe_<kinds>_zip_asm(r0, a0[, b0], r1, ...)."""
    g = build(zip_name(kinds))
    ec = "=v" if outputs_after_inputs(g) else "=&v"
    params, outs, ins, cys = [], [], [], []
    for k, kind in enumerate(kinds):
        params.append(f"fe &r{k}, const fe &a{k}" + (f", const fe &b{k}" if kind == "mul" else ""))
        outs += [f'[z{k}r{i}] "{ec}"(r{k}.v[{i}])' for i in range(8)]
        outs += [f'[z{k}c{i}] "=&s"(c{k}_{i})' for i in range(NCARRY)]
        cys += [f"c{k}_{i}" for i in range(NCARRY)]
        ins += [f'[z{k}a{i}] "v"(a{k}.v[{i}])' for i in range(8)]
        if kind == "mul":
            ins += [f'[z{k}b{i}] "v"(b{k}.v[{i}])' for i in range(8)]
    clob = ", ".join(f'"v{i}"' for i in range(MUL_NREGS * len(kinds)))
    return f"""// {", ".join(kinds)} interleaved (independent operands): {stats(g)}
__device__ __forceinline__ void {zip_name(kinds)}_asm({", ".join(params)}) {{
  uint64_t {", ".join(cys)};
  asm volatile(
{asm_body(g)}
      : {", ".join(outs)}
      : {", ".join(ins)}
      : {clob}, "scc");
}}
"""


def header() -> str:
    mul = build("fe_mul")
    sqr = build("fe_sqr")
    add = build("fe_add")
    sub = build("fe_sub")
    mont = build("sc_mont")
    clob_m = ", ".join(f'"v{MONT_BASE + i}"' for i in range(MONT_NREGS))
    n_in = ", ".join(f'[n{i}] "v"({hex(N_LIMBS[i])}u)' for i in range(4))
    nc_in = ", ".join(f'[nc{i}] "v"({hex(N_C_LIMBS[i])}u)' for i in range(4))
    st = {k: stats(build(k)) for k in PROGRAMS}
    clob = ", ".join(f'"v{MUL_BASE + i}"' for i in range(MUL_NREGS))
    a_in = ", ".join(f'[a{i}] "v"(a.v[{i}])' for i in range(8))
    b_in = ", ".join(f'[b{i}] "v"(b.v[{i}])' for i in range(8))
    r_out = ", ".join(f'[r{i}] "=&v"(r.v[{i}])' for i in range(8))
    assert outputs_after_inputs(mul) and outputs_after_inputs(sqr) and outputs_after_inputs(mont)
    r_late = ", ".join(f'[r{i}] "=v"(r.v[{i}])' for i in range(8))  # outputs_after_inputs
    t_out = ", ".join(f'[t{i}] "=&v"(t[{i}])' for i in range(8))
    c_out = ", ".join(f'[c{i}] "=&s"(c{i})' for i in range(NCARRY))
    c3_out = ", ".join(f'[c{i}] "=&s"(c{i})' for i in range(3))
    return f"""// field_asm.h — GENERATED by tools/gen_field_asm.py; do not edit.
//
// Hand-scheduled gfx950 field arithmetic mod p = 2^256 - 2^32 - 977 for the
// device build of field.h.  Same contract as the C++ functions there:
// inputs < 2^256, outputs weakly reduced (< 2^256, congruent mod p).
// Instruction mix (after scheduling):
//   fe_mul: {st['fe_mul']}
//   fe_sqr: {st['fe_sqr']}
//   fe_add: {st['fe_add']}
//   fe_sub: {st['fe_sub']}
//   sc_mont: {st['sc_mont']}
// The program lists are verified against Python integers by
// tests/test_field_asm.py (interpreter in the generator), and end to end on
// the GPU by the bit-exact parity tests.
#pragma once
#include <stdint.h>

// r = a * b mod p (weak).  Temporaries: v{MUL_BASE}..v{MUL_BASE + MUL_NREGS - 1} (clobbered).
__device__ __forceinline__ void fe_mul_asm(fe &r, const fe &a, const fe &b) {{
  uint64_t {", ".join(f"c{i}" for i in range(NCARRY))};
  asm volatile(
{asm_body(mul)}
      : {r_late}, {c_out}
      : {a_in}, {b_in}
      : {clob}, "scc");
}}

// r = a^2 mod p (weak), Comba squaring.  Temporaries as fe_mul.
__device__ __forceinline__ void fe_sqr_asm(fe &r, const fe &a) {{
  uint64_t {", ".join(f"c{i}" for i in range(NCARRY))};
  asm volatile(
{asm_body(sqr)}
      : {r_late}, {c_out}
      : {a_in}
      : {clob}, "scc");
}}

// r = a + b mod p (weak)
__device__ __forceinline__ void fe_add_asm(fe &r, const fe &a, const fe &b) {{
  uint64_t c0, c1, c2;
  uint32_t k0, k1;
  asm volatile(
{asm_body(add)}
      : {r_out}, [k0] "=&v"(k0), [k1] "=&v"(k1), {c3_out}
      : {a_in}, {b_in}
      : "scc");
}}

// r = a - b mod p (weak)
__device__ __forceinline__ void fe_sub_asm(fe &r, const fe &a, const fe &b) {{
  uint64_t c0, c1, c2;
  uint32_t k0, k1;
  asm volatile(
{asm_body(sub)}
      : {r_out}, [k0] "=&v"(k0), [k1] "=&v"(k1), {c3_out}
      : {a_in}, {b_in}
      : "scc");
}}

// r = a * b * 2^-256 mod N (Montgomery), a < 2^256, b < N; r < N.
// Temporaries: v{MONT_BASE}..v{MONT_BASE + MONT_NREGS - 1} (clobbered).
__device__ __forceinline__ void sc_mont_asm(sc &r, const sc &a, const sc &b) {{
  uint64_t c0, c1, c2;
  asm volatile(
{asm_body(mont)}
      : {r_late}, {c3_out}
      : {a_in}, {b_in}, {n_in}, {nc_in}, [ninv] "v"({hex(NINV)}u)
      : {clob_m});
}}

// ---- zipped multiplies for latency-bound single-wave chains (gen_zip) ----
// Temporaries: v0..v{MUL_NREGS}*K - 1 (clobbered).
{"".join(zip_wrapper(k) for k in ZIP_COMBOS)}"""


def main():
    text = header()
    if "--check" in sys.argv:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        if cur != text:
            print(f"{OUT} is stale: run python tools/gen_field_asm.py", file=sys.stderr)
            sys.exit(1)
        return
    with open(OUT, "w") as f:
        f.write(text)
    for k in PROGRAMS:
        print(k, stats(build(k)))


if __name__ == "__main__":
    main()
