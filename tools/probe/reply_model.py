#!/usr/bin/env python3
"""Design check (CPU, tools only): a Python model of board_nd_records
(csrc/bgx_movegen.h) -- the 15 non-doubles rolls of a root from shared first
moves, rule mode and bar mode -- against the oracle's movegen on self-play and
random placements. It checks the algorithm (roll order, pass order, the
nd_first filter, the bar-mode duplicate rule), not the kernel; the kernel is
checked by tests/test_gpu_reply.py."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import oracle as orc  # noqa: E402
from test_gpu_parity import _fuzz_positions, _random_positions  # noqa: E402


def sort2(a, b):
    return (a | (b << 5)) if a <= b else (b | (a << 5))


def nd_key(s1, t1, h1, s2, t2, h2):
    r0, r1, a0, a1 = s1, s2, t1, t2
    if s2 != 31:
        if t1 == s2:
            r1, a0 = 31, 31
        elif t2 == s1:
            r0, a1 = 31, 31
    hh0 = t1 if h1 else 31
    hh1 = t2 if h2 else 31
    return sort2(r0, r1) | (sort2(a0, a1) << 10) | (sort2(hh0, hh1) << 20)


class Root:
    def __init__(self, b, p):
        self.p = p
        self.m = [int(x) for x in b[24 * p:24 * p + 24]]
        self.o = [int(x) for x in b[24 * (1 - p):24 * (1 - p) + 24]]
        self.bar, self.obar = int(b[48 + p]), int(b[48 + 1 - p])
        self.off, self.ooff = int(b[50 + p]), int(b[50 + 1 - p])
        self.block = sum(1 << i for i in range(24) if self.o[i] >= 2)
        self.blot = sum(1 << i for i in range(24) if self.o[i] == 1)
        self.occ = sum(1 << i for i in range(24) if self.m[i] >= 1)

    def ok(self, d):
        free = ~self.block & 0xFFFFFF
        return (free >> d) & ((1 << (24 - d)) - 1) if self.p == 0 else (free << d) & 0xFFFFFF

    def entry(self, d):
        return d - 1 if self.p == 0 else 24 - d

    def dest(self, s, d):
        t = self.entry(d) if s == 24 else (s + d if self.p == 0 else s - d)
        return 25 if t < 0 or t > 23 else t

    def rule(self):
        home = sum(self.m[18:24]) if self.p == 0 else sum(self.m[0:6])
        return self.bar == 0 and 15 - self.off - home >= 3

    def board(self, key):
        m, o = list(self.m), list(self.o)
        bar, obar, off = self.bar, self.obar, self.off
        for i in range(2):
            a, h = (key >> (10 + 5 * i)) & 31, (key >> (20 + 5 * i)) & 31
            if a == 25:
                off += 1
            elif a < 24:
                m[a] += 1
            if h < 24:
                o[h] -= 1
                obar += 1
        for i in range(2):
            r = (key >> (5 * i)) & 31
            if r == 24:
                bar -= 1
            elif r < 24:
                m[r] -= 1
        out = np.zeros(52, np.uint8)
        out[24 * self.p:24 * self.p + 24] = m
        out[24 * (1 - self.p):24 * (1 - self.p) + 24] = o
        out[48 + self.p], out[48 + 1 - self.p], out[50 + self.p], out[50 + 1 - self.p] = bar, obar, off, self.ooff
        return out


def bits(m):
    return [i for i in range(25) if (m >> i) & 1]


def popc(m):
    return bin(m).count("1")


def nd_first(R, occ0, pas, s1, t1, s2, t2, H, L):
    chain = s2 == t1
    if not chain and t2 != s1:
        return pas == 0
    if chain and ((R.blot >> t1) & 1):
        return True
    x = s1 if chain else s2
    iH = x + H if R.p == 0 else x - H
    iL = x + L if R.p == 0 else x - L
    bad = R.block | R.blot
    A, B = not ((bad >> iH) & 1), bool((occ0 >> iL) & 1)
    C, D = not ((bad >> iL) & 1), bool((occ0 >> iH) & 1)
    me = (0 if chain else 1) if pas == 0 else (2 if chain else 3)
    p0 = R.p == 0
    if me == 0:
        return True if p0 else not B
    if me == 1:
        return (not A) if p0 else True
    if me == 2:
        return (not A) and (not B) and (True if p0 else not D)
    return (not A) and (not B) and ((not C) if p0 else True)


def board_nd(R):
    """{(L, H): [keys]} or None (not covered)."""
    onbar = R.bar > 0
    rule = (not onbar) and R.rule()
    if not onbar and not rule:
        return None
    occ = R.occ
    opn = {d: not ((R.block >> R.entry(d)) & 1) for d in range(1, 7)}
    first = []   # lanes: (d, s1, t1, h1, base2)
    for d in range(6, 0, -1):
        if rule:
            for s1 in bits(occ & R.ok(d)):
                t1 = s1 + d if R.p == 0 else s1 - d
                last1 = (1 << s1) if R.m[s1] == 1 else 0
                first.append((d, s1, t1, bool((R.blot >> t1) & 1), (occ & ~last1) | (1 << t1)))
        elif opn[d]:
            t1 = R.entry(d)
            first.append((d, 24, t1, bool((R.blot >> t1) & 1), occ | (1 << t1)))
    if len(first) > 64:
        return None
    child_bar = R.bar >= 2
    out = {}
    for L in range(1, 6):
        for H in range(L + 1, 7):
            m2s = []
            for (d, s1, t1, h1, base2) in first:
                if d == H or d == L:
                    if child_bar:
                        m2 = (1 << 24) if opn[L if d == H else H] else 0
                    else:
                        m2 = base2 & (R.ok(L) if d == H else R.ok(H))
                else:
                    m2 = 0
                m2s.append(m2)
            two1 = any(f[0] == H and m2 for f, m2 in zip(first, m2s))
            two2 = any(f[0] == L and m2 for f, m2 in zip(first, m2s))
            nH = popc(occ & R.ok(H)) if rule else int(opn[H])
            keys = []
            if two1 or (nH != 1 and two2):
                K0 = None
                if not rule:
                    eH, eL = R.entry(H), R.entry(L)
                    hH = bool((R.blot >> eH) & 1)
                    if child_bar:
                        if opn[H] and opn[L]:
                            K0 = nd_key(24, eH, hH, 24, eL, bool((R.blot >> eL) & 1))
                    elif opn[H] and ((R.ok(L) >> eH) & 1):
                        t2 = eH + L if R.p == 0 else eH - L
                        b2 = R.blot & ~((1 << eH) if hH else 0)
                        K0 = nd_key(24, eH, hH, eH, t2, bool((b2 >> t2) & 1))
                for (d, s1, t1, h1, base2), m2 in zip(first, m2s):
                    if d != H and d != L:
                        continue
                    pas = 1 if d == L else 0
                    if rule and pas == 1:
                        rv = s1 - H if R.p == 0 else s1 + H
                        m2 &= (1 << t1) | ((1 << rv) if 0 <= rv < 24 else 0)
                    for s2 in bits(m2):
                        t2 = R.dest(s2, H if pas else L)
                        blot2 = R.blot & ~((1 << t1) if h1 else 0)
                        h2 = t2 < 24 and bool((blot2 >> t2) & 1)
                        key = nd_key(s1, t1, h1, s2, t2, h2)
                        keep = nd_first(R, occ, pas, s1, t1, s2, t2, H, L) if rule else not (pas == 1 and key == K0)
                        if keep:
                            keys.append(key)
            else:
                for (d, s1, t1, h1, base2) in first:
                    if d == H or (d == L and nH != 1):
                        keys.append(nd_key(s1, t1, h1, 31, 31, False))
            out[(L, H)] = keys
    return out


def main():
    pos = _fuzz_positions(77, 24) + _random_positions(5, 3000) + _random_positions(6, 3000)
    covered = bad = 0
    for b, p in pos:
        R = Root(b, p)
        res = board_nd(R)
        if res is None:
            continue
        covered += 1
        for (L, H), keys in res.items():
            n, want, _ = orc.movegen(b, p, L, H, cap=4096)
            got = np.array([R.board(k) for k in keys]).reshape(-1, 52)
            if len(got) != n or not np.array_equal(got, want[:n]):
                bad += 1
                if bad < 5:
                    print("mismatch", p, L, H, len(got), n, "bar", R.bar)
    print(f"positions {len(pos)}, covered {covered}, mismatching (root, roll) lists {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())


def board_nd_v2(R):
    """The flat-round form (board_nd_records2): counts per (lane, partner die),
    roll-major flat starts, 64-child rounds with marks + max-scan + carry.
    Same {(L, H): keys} as board_nd, or None."""
    onbar = R.bar > 0
    rule = (not onbar) and R.rule()
    if not onbar and not rule:
        return None
    occ = R.occ
    opn = {d: not ((R.block >> R.entry(d)) & 1) for d in range(1, 7)}
    lanes = []   # (die, s1, t1, h1, base2)
    nd = {}
    for d in range(6, 0, -1):
        src = bits(occ & R.ok(d)) if rule else ([24] if opn[d] else [])
        nd[d] = len(src)
        for s1 in src:
            if rule:
                t1 = s1 + d if R.p == 0 else s1 - d
                last1 = (1 << s1) if R.m[s1] == 1 else 0
                base2 = (occ & ~last1) | (1 << t1)
            else:
                t1 = R.entry(d)
                base2 = occ | (1 << t1)
            lanes.append((d, s1, t1, bool((R.blot >> t1) & 1), base2))
    if len(lanes) > 64:
        return None
    child_bar = R.bar >= 2
    m2tab, cu, cr = {}, {}, {}
    for li, (dl, s1, t1, h1, base2) in enumerate(lanes):
        for dB in range(1, 7):
            if dB == dl:
                continue
            m2 = ((1 << 24) if opn[dB] else 0) if child_bar else base2 & R.ok(dB)
            cu[li, dB] = popc(m2)
            if rule and dB > dl:
                rv = s1 - dB if R.p == 0 else s1 + dB
                m2 &= (1 << t1) | ((1 << rv) if 0 <= rv < 24 else 0)
            cr[li, dB] = popc(m2)
            m2tab[li, dB] = m2
    rolls = [(L, H) for L in range(1, 6) for H in range(L + 1, 7)]
    single, starts, total = {}, {}, 0
    for q, (L, H) in enumerate(rolls):
        two1 = any(lanes[i][0] == H and cu[i, L] > 0 for i in range(len(lanes)))
        two2 = any(lanes[i][0] == L and cu[i, H] > 0 for i in range(len(lanes)))
        nH = nd[H]
        two = two1 or (nH != 1 and two2)
        single[q] = not two
        for i, ln in enumerate(lanes):
            dl = ln[0]
            if two:
                c = cr[i, L] if dl == H else (cr[i, H] if dl == L else 0)
            else:
                c = 1 if (dl == H or (dl == L and nH != 1)) else 0
            if c:
                starts[i, q] = (total, c)
                total += c
    # rounds: each position gets its parent by the marks
    parent_at = {}
    for (i, q), (s, c) in starts.items():
        for k in range(c):
            parent_at[s + k] = (i, q, s)
    out = {rl: [] for rl in rolls}
    for r in range(total):
        i, q, s = parent_at[r]
        L, H = rolls[q]
        dl, s1, t1, h1, base2 = lanes[i]
        pp = 1 if dl == L else 0
        if single[q]:
            out[(L, H)].append(nd_key(s1, t1, h1, 31, 31, False))
            continue
        src2 = m2tab[i, H if pp else L]
        s2 = 24 if src2 >> 24 else bits(src2)[r - s]
        t2 = R.dest(s2, H if pp else L)
        blot2 = R.blot & ~((1 << t1) if h1 else 0)
        h2 = t2 < 24 and bool((blot2 >> t2) & 1)
        key = nd_key(s1, t1, h1, s2, t2, h2)
        if rule:
            keep = nd_first(R, occ, pp, s1, t1, s2, t2, H, L)
        else:
            K0 = None
            if pp == 1:
                eH, eL = R.entry(H), R.entry(L)
                hH = bool((R.blot >> eH) & 1)
                if child_bar:
                    if opn[H] and opn[L]:
                        K0 = nd_key(24, eH, hH, 24, eL, bool((R.blot >> eL) & 1))
                elif opn[H] and ((R.ok(L) >> eH) & 1):
                    t2c = eH + L if R.p == 0 else eH - L
                    b2 = R.blot & ~((1 << eH) if hH else 0)
                    K0 = nd_key(24, eH, hH, eH, t2c, bool((b2 >> t2c) & 1))
            keep = not (pp == 1 and key == K0)
        if keep:
            out[(L, H)].append(key)
    return out


def main_v2():
    pos = _fuzz_positions(77, 24) + _random_positions(5, 3000)
    bad = cov = 0
    for b, p in pos:
        R = Root(b, p)
        a, v = board_nd(R), board_nd_v2(R)
        if a is None:
            assert v is None
            continue
        cov += 1
        if a != v:
            bad += 1
    print(f"v2 vs v1: covered {cov}, differing roots {bad}")
    return 1 if bad else 0
