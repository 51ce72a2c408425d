"""Offline LDS bank-conflict model of lenet_train's hot LDS accesses (gfx950 rules).

Replays the exact per-lane byte addresses of each LDS instruction of the fused
train kernel (csrc/kernels/lenet_fused.hip) for every wave, applies the CDNA4
banking rules (MI355X_MICROARCH.md §LDS: lane groups per instruction width, bank
= (addr/4) mod 64 for b64/b128/tr_b16 reads, mod 32 otherwise) and reports the
extra LDS cycles per access site, i.e. what SQ_LDS_BANK_CONFLICT attributes to
each.  Used to choose layouts without a GPU run.

    python tools/lds_bank_model.py            # per-site report, split step (B <= 64, KS = 4)
    python tools/lds_bank_model.py --unsplit  # the one-workgroup-per-sample path (older sites)
    python tools/lds_bank_model.py --search   # search a dgrad K-slice order (kDgOrder)
"""
import os
import re
import sys
from collections import defaultdict

# ---- layout constants (mirror lenet_fused.hip)
LD_W2C, LD_F1 = 432, 328
LD_P1H, DG_OCP, LD_DC2, LD_DC1 = 24, 24, 72, 592
LD_P1 = 148  # P1 / I1 channel pitch (elements, lenet_fused.hip)
DC2H_RP = 16 * 24 + 32  # DC2H row pitch (elements)
P1H_RP = 12 * 24 + 32   # P1H row pitch (elements)
DG_CH = 77  # dgrad B image is chunk-major [chunk][16 rows][8]
S_W2C = 0
S_W2D = 21 * LD_W2C * 2
S_F1 = S_W2D + DG_CH * 16 * 16
S_X = 65536  # (I_END - I_W2C) * 2
S_P1 = S_X + 1600
S_I1 = S_P1 + 10 * LD_P1 * 2
S_P2 = S_I1 + (10 * LD_P1 + 15) // 16 * 16
S_I2 = S_P2 + 640
S_P1H = S_I2 + 320
S_DC2 = S_P1H + 12 * P1H_RP * 2
S_DC2H = S_DC2 + 32 * LD_DC2 * 2
S_DC1 = S_DC2H + 16 * DC2H_RP * 2

B128_GROUPS = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
               [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31],
               [32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59],
               [36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63]]
HALVES = [list(range(32)), list(range(32, 64))]


def extra_cycles(addrs, width, kind="read", active=None):
    """Extra LDS cycles of one wave-instruction (addrs: 64 byte addresses or None)."""
    if width == 16:
        groups, nb = (B128_GROUPS, 64) if kind == "read" else ([list(range(i, i + 8)) for i in range(0, 64, 8)], 32)
    elif width == 8:
        groups, nb = HALVES, (64 if kind == "read" else 32)
    else:
        groups, nb = HALVES, 32
    ndw = max(1, width // 4)
    extra = 0
    for g in groups:
        banks = defaultdict(set)
        for l in g:
            if active is not None and not active[l]:
                continue
            a = addrs[l]
            if a is None:
                continue
            for d in range(ndw):
                dw = a // 4 + d
                banks[dw % nb].add(dw)
        worst = max((len(v) for v in banks.values()), default=1)
        extra += worst - 1
    return extra


def lanes():
    for lane in range(64):
        yield lane, lane & 15, lane >> 4


def kernel_order(name):
    """A K-slice order table of the kernel (kDgOrder / kC2Order in lenet_images.h)."""
    src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc", "kernels",
                            "lenet_images.h")).read()
    body = re.search(name + r" o\{\{([0-9,\s]+)\}", src).group(1)
    return [int(v) for v in body.replace("\n", " ").split(",")]


def kernel_dg_order():
    return kernel_order("DgOrder")


def dgrad_offsets(order=None, rp=None):
    order = order or kernel_dg_order()
    rp = rp or DC2H_RP
    tab = {}
    for q in range(4):
        for ks in range(24):
            kg = order[min(4 * ks + q, 74)]
            tap, ocg = kg // 3, kg % 3
            tab[q, ks] = (tap // 5) * rp + (tap % 5) * DG_OCP + ocg * 8
    return tab


def conv2_offsets():
    order = kernel_order("C2Order")
    tab = {}
    for q in range(4):
        for ks in range(16):
            kg = order[min(4 * ks + q, 49)]
            tap = kg >> 1
            tab[q, ks] = (tap // 5) * P1H_RP + (tap % 5) * LD_P1H + (kg & 1) * 8
    return tab


def dgrad_A_step(tab, ks, rp):
    tot = 0
    for wave in range(8):
        addrs = []
        for lane, l16, kq in lanes():
            m = wave * 16 + l16
            addrs.append(S_DC2H + 2 * ((m // 12) * rp + (m % 12) * DG_OCP + tab[kq, ks]))
        tot += extra_cycles(addrs, 16)
    return tot


def site_dgrad_A(order=None, rp=None):
    rp = rp or DC2H_RP
    tab = dgrad_offsets(order, rp)
    return sum(dgrad_A_step(tab, ks, rp) for ks in range(19))


def search_dg_order(rp=DC2H_RP, iters=6000, seeds=6):
    """Local search (random swaps) for a K-slice order minimising the dgrad A conflicts."""
    import random
    best = None
    for seed in range(seeds):
        rng = random.Random(seed)
        order = list(range(75))
        rng.shuffle(order)

        def step_cost(o, ks):
            return dgrad_A_step(dgrad_offsets(o, rp), ks, rp)
        per = [step_cost(order, k) for k in range(19)]
        for _ in range(iters):
            i, j = rng.sample(range(75), 2)
            order[i], order[j] = order[j], order[i]
            touched = {i // 4, j // 4} | ({18} if 74 in (i, j) else set())
            new = {k: step_cost(order, k) for k in touched}
            if sum(new.values()) <= sum(per[k] for k in touched):
                for k, v in new.items():
                    per[k] = v
            else:
                order[i], order[j] = order[j], order[i]
        if best is None or sum(per) < best[0]:
            best = (sum(per), list(order))
    return best


def site_dgrad_B():
    tot = 0
    for wave in range(8):
        for ks in range(19):
            addrs = [S_W2D + 2 * (((4 * ks + kq) * 16 + l16) * 8) for lane, l16, kq in lanes()]
            tot += extra_cycles(addrs, 16)
    return tot


def site_conv2_A():
    tab = conv2_offsets()
    tot = 0
    for wave in range(8):
        mt = wave & 3
        for ks in range(13):
            addrs = []
            for lane, l16, kq in lanes():
                m = mt * 16 + l16
                p, q = m >> 2, m & 3
                oy, ox = 2 * (p >> 2) + (q >> 1), 2 * (p & 3) + (q & 1)
                addrs.append(S_P1H + 2 * (oy * P1H_RP + ox * LD_P1H + tab[kq, ks]))
            tot += extra_cycles(addrs, 16)
    return tot


def site_conv2_B():
    tot = 0
    for wave in range(8):
        nt = wave >> 2
        for ks in range(13):
            addrs = [S_W2C + 2 * (min(nt * 16 + l16, 20) * LD_W2C + 8 * kq + ks * 32) for lane, l16, kq in lanes()]
            tot += extra_cycles(addrs, 16)
    return tot


def site_conv1_gather():
    koff = [(k // 5) * 28 + (k % 5) if k < 25 else 0 for k in range(32)]
    tot = 0
    for wave in range(8):
        for it in range(5):
            mt = min(wave + 8 * it, 35)
            for j in range(8):
                addrs = []
                for lane, l16, kq in lanes():
                    m = mt * 16 + l16
                    p, q = m >> 2, m & 3
                    pb = (2 * (p // 12) + (q >> 1)) * 28 + 2 * (p % 12) + (q & 1)
                    addrs.append(S_X + 2 * (pb + koff[8 * kq + j]))
                tot += extra_cycles(addrs, 2)
    return tot


def site_conv1_epilogue():
    tot = 0
    for wave in range(8):
        for it in range(5):
            mt = wave + 8 * it
            if mt >= 36:
                continue
            act = [l16 < 10 for lane, l16, kq in lanes()]
            w = [mt * 4 + kq for lane, l16, kq in lanes()]
            p1 = [S_P1 + 2 * (l16 * LD_P1 + w[lane]) for lane, l16, kq in lanes()]
            i1 = [S_I1 + (l16 * LD_P1 + w[lane]) for lane, l16, kq in lanes()]
            p1h = [S_P1H + 2 * ((w[lane] // 12) * P1H_RP + (w[lane] % 12) * LD_P1H + l16)
                   for lane, l16, kq in lanes()]
            tot += extra_cycles(p1, 2, "write", act) + extra_cycles(i1, 1, "write", act) + \
                extra_cycles(p1h, 2, "write", act)
    return tot


def site_conv2_wgrad_gather():
    tot = 0
    for wave in range(8):
        kwb = []
        for jj in range(2):
            row = []
            for lane, l16, kq in lanes():
                k = min((wave + 8 * jj) * 16 + l16, 249)
                ic, r = k // 25, k % 25
                row.append(ic * LD_P1 + (r // 5) * 12 + r % 5)
            kwb.append(row)
        for ps in range(2):
            for jj in range(2):
                for j in range(8):
                    addrs = []
                    for lane, l16, kq in lanes():
                        ohr = ((ps * 32 + 8 * kq) >> 3) * 12
                        addrs.append(S_P1 + 2 * (kwb[jj][lane] + ohr + j))
                    tot += extra_cycles(addrs, 2)
    return tot


def site_conv1_wgrad():
    tot = 0
    for wave in range(8):
        kc1 = [(wave & 1) * 16 + l16 for lane, l16, kq in lanes()]
        koffc = [(k // 5) * 28 + (k % 5) if k < 25 else 0 for k in kc1]
        for i in range(5):
            ps = min((wave >> 1) + 4 * i, 17)
            dc1 = [S_DC1 + 2 * (l16 * LD_DC1 + ps * 32 + 8 * kq) for lane, l16, kq in lanes()]
            tot += extra_cycles(dc1, 16)
            for j in range(8):
                addrs = []
                for lane, l16, kq in lanes():
                    p0 = ps * 32 + 8 * kq
                    oh, ow0 = p0 // 24, p0 % 24
                    addrs.append(S_X + 2 * (oh * 28 + ow0 + koffc[lane] + j))
                tot += extra_cycles(addrs, 2)
    return tot


def site_stage5_writes():
    tot = 0
    for t in range(20):
        for pos in range(4):
            act = [lane < 16 for lane in range(64)]
            dc2, dc2h = [], []
            for lane in range(64):
                w = lane & 15
                oh, ow = 2 * (w >> 2) + (pos >> 1), 2 * (w & 3) + (pos & 1)
                dc2.append(S_DC2 + 2 * (t * LD_DC2 + oh * 8 + (ow & ~1)) if (pos & 1) == 0 else None)
                dc2h.append(S_DC2H + 2 * ((oh + 4) * DC2H_RP + (ow + 4) * DG_OCP + t))
            tot += extra_cycles(dc2, 2, "write", act) + extra_cycles(dc2h, 2, "write", act)
    return tot


def site_dgrad_store():
    tot = 0
    for wave in range(8):
        for r in range(4):
            act = [l16 < 10 for lane, l16, kq in lanes()]
            for d in (0, 24):  # two 32-bit pair writes per window
                addrs = []
                for lane, l16, kq in lanes():
                    mm = wave * 16 + 4 * kq + r
                    ih, iw = mm // 12, mm % 12
                    addrs.append(S_DC1 + 2 * (l16 * LD_DC1 + 2 * ih * 24 + 2 * iw + d))
                tot += extra_cycles(addrs, 4, "write", act)
    return tot


# ---------------------------------------------------------------- split step (KS = 4, B <= 64)
# The headline path: 4 workgroups per sample (part = 0..3), 16 waves each.  Sites per workgroup,
# averaged over the 4 parts (lenet_fused.hip stages 1-8, split branch).
DG_KS = 19
LD_DC2_ = LD_DC2
S_COFF = S_DC1 + 16 * LD_DC1 * 2
S_DOFF = S_COFF + 4 * 16 * 2
S_DZ1B = S_DOFF + 4 * 24 * 2
S_F = S_DZ1B + 64 * 2
S_W1C = S_F + 2816 * 4
S_LABEL = S_W1C + 16 * 32 * 2
S_DBG = S_LABEL + 16
S_C1T = S_DBG + 32 * 8
S_C1H = S_C1T + 1024 * 8
S_XC = S_C1H + 1024 * 8
XC_LD = 800
S_CONSTB = S_XC + 3 * XC_LD * 2
S_I2 = S_P2 + 640


def xrun(e):  # the aligned 4-pixel run X[e .. e+3] (lenet_fused.hip: X or a shifted copy)
    c = e & 3
    return (S_X if c == 0 else S_XC + 2 * (c - 1) * XC_LD) + 2 * (e - c)


def split_conv1_reads():  # (tried in round 4: aligned runs from shifted copies; slower, not kept)
    tot = 0
    for mt in range(36):
        A, B, C = [], [], []
        for lane, l16, kq in lanes():
            m = mt * 16 + l16
            p, q = m >> 2, m & 3
            pb = (2 * (p // 12) + (q >> 1)) * 28 + 2 * (p % 12) + (q & 1)
            e1, e2 = pb + 28 * kq, pb + 112 + (2 if kq == 1 else 0)
            A.append(xrun(e1))
            B.append(S_X + 2 * (e1 + 4))
            C.append(xrun(e2))
        tot += extra_cycles(A, 8) + extra_cycles(B, 2) + extra_cycles(C, 8)
    return tot


def split_conv1_gather():  # stage 1: 36 tiles, 8 ds_read_u16 each
    koff = [(k // 5) * 28 + (k % 5) if k < 25 else 0 for k in range(32)]
    tot = 0
    for mt in range(36):
        for j in range(8):
            addrs = []
            for lane, l16, kq in lanes():
                m = mt * 16 + l16
                p, q = m >> 2, m & 3
                pb = (2 * (p // 12) + (q >> 1)) * 28 + 2 * (p % 12) + (q & 1)
                # r1 = pb + 28 kq + {0..4}; r2 = pb + 112 + (kq == 1 ? 2 : 0) + {0..2}
                off = pb + 28 * kq + j if j < 5 else pb + 112 + (2 if kq == 1 else 0) + (j - 5)
                addrs.append(S_X + 2 * off)
            tot += extra_cycles(addrs, 2)
    return tot


def split_conv1_epilogue():
    tot = 0
    for mt in range(36):
        act = [l16 < 10 for lane, l16, kq in lanes()]
        w = [mt * 4 + kq for lane, l16, kq in lanes()]
        p1 = [S_P1 + 2 * (l16 * LD_P1 + w[lane]) for lane, l16, kq in lanes()]
        i1 = [S_I1 + (l16 * LD_P1 + w[lane]) for lane, l16, kq in lanes()]
        p1h = [S_P1H + 2 * ((w[lane] // 12) * P1H_RP + (w[lane] % 12) * LD_P1H + l16) for lane, l16, kq in lanes()]
        tot += extra_cycles(p1, 2, "write", act) + extra_cycles(i1, 1, "write", act) + \
            extra_cycles(p1h, 2, "write", act)
    return tot


def split_conv2_epilogue():  # stage 2: P2 / I2 writes
    tot = 0
    for wave in range(8):
        mt, nt = wave & 3, wave >> 2
        act = [nt * 16 + l16 < 20 for lane, l16, kq in lanes()]
        p2 = [S_P2 + 2 * ((nt * 16 + l16) * 16 + mt * 4 + kq) for lane, l16, kq in lanes()]
        i2 = [S_I2 + ((nt * 16 + l16) * 16 + mt * 4 + kq) for lane, l16, kq in lanes()]
        tot += extra_cycles(p2, 2, "write", act) + extra_cycles(i2, 1, "write", act)
    return tot


def split_fc1():  # stage 3: waves 0-3, 10 K-steps (A = P2 broadcast row)
    tot = 0
    for wave in range(4):
        for ks in range(10):
            pa = [S_P2 + 2 * (ks * 32 + 8 * kq) for lane, l16, kq in lanes()]
            fb = [S_F1 + 2 * (min(wave * 16 + l16, 50) * LD_F1 + 8 * kq + ks * 32) for lane, l16, kq in lanes()]
            tot += extra_cycles(pa, 16) + extra_cycles(fb, 16)
    return tot


def split_stage5_tr():  # dP2: transposed fc1 reads (ds_read_b64_tr_b16), 20 channel tiles
    tot = 0
    for t in range(20):
        for base in (0, 4, 32, 36):
            addrs = [S_F1 + 2 * (min(base + 8 * kq + (l16 >> 2), 50) * LD_F1 + 4 * (l16 & 3) + t * 16)
                     for lane, l16, kq in lanes()]
            tot += extra_cycles(addrs, 8)
    return tot


def split_stage5_writes():  # lane group kq writes window position kq (DC2H) / row kq < 2 (DC2)
    tot = 0
    for t in range(20):
        act = [(lane >> 4) < 2 for lane in range(64)]
        dc2, dc2h = [], []
        for lane, l16, kq in lanes():
            oh0, ow0 = 2 * (l16 >> 2), 2 * (l16 & 3)
            dc2.append(S_DC2 + 2 * (t * LD_DC2 + (oh0 + (kq & 1)) * 8 + ow0))
            dc2h.append(S_DC2H + 2 * ((oh0 + (kq >> 1) + 4) * DC2H_RP + (ow0 + (kq & 1) + 4) * DG_OCP + t))
        tot += extra_cycles(dc2, 4, "write", act) + extra_cycles(dc2h, 2, "write")
    return tot


def split_conv2_wgrad(part):  # stage 6, waves 12-15: one N-tile each
    tot = 0
    for w in range(4):
        kk = [min((4 * part + w) * 16 + l16, 249) for lane, l16, kq in lanes()]
        for j in list(range(8)) + list(range(48, 56)):
            addrs = [S_P1 + 2 * ((kk[lane] // 25) * LD_P1 + ((kk[lane] % 25) // 5) * 12 + (kk[lane] % 25) % 5 + kq * 12 + j)
                     for lane, l16, kq in lanes()]
            tot += extra_cycles(addrs, 2)
        for row0, col in ((0, 0), (16, 0), (0, 32), (16, 32)):
            addrs = [S_DC2 + 2 * ((row0 + l16) * LD_DC2 + col + 8 * kq) for lane, l16, kq in lanes()]
            tot += extra_cycles(addrs, 16)
    return tot


def split_dgrad(part):  # stage 6, waves 0-11: T3 tiles x P K-parts, <= 5 K-steps each
    tab = dgrad_offsets()
    T3 = 3 if part == 0 else 2
    P = 4 if T3 == 3 else 6
    tot = 0
    for wave in range(12):
        ts, pp = wave % T3, wave // T3
        ks0, ks1 = pp * DG_KS // P, (pp + 1) * DG_KS // P
        for u in range(5):
            ks = ks0 + u
            a_ = []
            b_ = []
            for lane, l16, kq in lanes():
                mw = (part + 4 * ts) * 16 + l16
                a_.append(S_DC2H + 2 * ((mw // 12) * DC2H_RP + (mw % 12) * DG_OCP + tab[kq, min(ks, DG_KS - 1)]))
                b_.append(S_W2D + 2 * ((((4 * ks + kq) * 16 + l16) * 8) if ks < ks1 else ((DG_CH - 1) * 16 + l16) * 8))
            tot += extra_cycles(a_, 16) + extra_cycles(b_, 16)
        for r in range(4):
            tot += extra_cycles([S_C1T + 4 * ((ts * P + pp) * 256 + r * 64 + lane) for lane in range(64)], 4, "write")
    return tot


def split_dgrad_reduce(part):  # stage 7: sum of the K parts + relu / pool1 backward into DC1
    T3 = 3 if part == 0 else 2
    P = 4 if T3 == 3 else 6
    tot = 0
    for wv in range(T3 * 4):
        tids = range(wv * 64, wv * 64 + 64)
        ts = [t >> 8 for t in tids]
        e = [t & 255 for t in tids]  # thread -> partial element (MFMA output layout)
        row = [4 * ((x >> 4) & 3) + (x >> 6) for x in e]
        ci = [x & 15 for x in e]
        act = [c < 10 for c in ci]
        for q in range(6):
            tot += extra_cycles([S_C1T + 4 * ((ts[i] * P + q) * 256 + e[i]) for i in range(64)], 4, "read", act)
        mm = [(part + 4 * ts[i]) * 16 + row[i] for i in range(64)]
        tot += extra_cycles([S_P1 + 2 * (ci[i] * LD_P1 + mm[i]) for i in range(64)], 2, "read", act)
        tot += extra_cycles([S_I1 + (ci[i] * LD_P1 + mm[i]) for i in range(64)], 1, "read", act)
        for d in (0, 24):
            tot += extra_cycles([S_DC1 + 2 * (ci[i] * LD_DC1 + 2 * (mm[i] // 12) * 24 + 2 * (mm[i] % 12) + d)
                                 for i in range(64)], 4, "write", act)
    return tot


def split_conv1_wgrad():  # stage 8, waves 0-11: 3 K-steps each (DC1 A fragment + X runs)
    tot = 0
    for wave in range(12):
        for i in range(3):
            ps = min((wave >> 1) + 6 * i, 17)
            tot += extra_cycles([S_DC1 + 2 * (l16 * LD_DC1 + ps * 32 + 8 * kq) for lane, l16, kq in lanes()], 16)
            for half in range(2):
                addrs = []
                for lane, l16, kq in lanes():
                    kc1 = (wave & 1) * 16 + l16
                    p0 = ps * 32 + 8 * kq
                    oh, ow0 = p0 // 24, p0 % 24
                    if kc1 < 25:
                        ee = oh * 28 + ow0 + (kc1 // 5) * 28 + kc1 % 5
                        c = ee & 3
                        addrs.append(xrun(ee) + 8 * half)
                    else:
                        addrs.append(S_CONSTB + 2 * (8 if kc1 == 25 else 0) + 8 * half)
                tot += extra_cycles(addrs, 8)
    return tot


def _avg_parts(fn):
    return lambda: round(sum(fn(p) for p in range(4)) / 4)


SPLIT_SITES = [("conv1 gathers (u16)", split_conv1_gather), ("conv1 epilogue writes", split_conv1_epilogue),
               ("conv2 A (b128)", site_conv2_A), ("conv2 B (b128)", site_conv2_B),
               ("conv2 epilogue writes", split_conv2_epilogue), ("fc1 A / B (b128)", split_fc1),
               ("dP2 transposed reads", split_stage5_tr), ("stage5 DC2/DC2H writes", split_stage5_writes),
               ("conv2 wgrad (waves 12-15)", _avg_parts(split_conv2_wgrad)),
               ("dgrad A / B + partial writes", _avg_parts(split_dgrad)),
               ("dgrad reduce + DC1 scatter", _avg_parts(split_dgrad_reduce)),
               ("conv1 wgrad DC1 + X runs", split_conv1_wgrad)]

SITES = [("dgrad A (b128)", site_dgrad_A), ("dgrad B (b128)", site_dgrad_B), ("conv2 A (b128)", site_conv2_A),
         ("conv2 B (b128)", site_conv2_B), ("conv1 gathers (u16)", site_conv1_gather),
         ("conv1 epilogue writes", site_conv1_epilogue), ("conv2 wgrad gathers (u16)", site_conv2_wgrad_gather),
         ("conv1 wgrad A b128 + gathers", site_conv1_wgrad), ("stage5 DC2/DC2H writes", site_stage5_writes),
         ("dgrad DC1 scatter", site_dgrad_store)]

if __name__ == "__main__":
    if "--search" in sys.argv:
        cost, order = search_dg_order()
        print(f"dgrad A extra cycles {cost} with order {order}")
        sys.exit(0)
    total = 0
    if "--unsplit" not in sys.argv:  # default: the split step (B <= 64)
        SITES = SPLIT_SITES
        print("split step (KS = 4), per workgroup, averaged over the 4 parts")
    for name, fn in SITES:
        v = fn()
        total += v
        print(f"{name:32s} {v:6d} extra LDS cycles / sample / workgroup")
    print(f"{'total (modelled sites)':32s} {total:6d}")
