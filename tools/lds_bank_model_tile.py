"""Offline LDS bank-conflict model of lenet_tile (csrc/kernels/lenet_tile.hip), the large-batch
step: replays the per-lane byte addresses of each hot LDS instruction for one 4-sample tile and
applies the gfx950 banking rules (tools/lds_bank_model.py: extra_cycles).  Reports the extra LDS
cycles per tile and site, i.e. what SQ_LDS_BANK_CONFLICT attributes to each.

    python tools/lds_bank_model_tile.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lds_bank_model import (DG_CH, DG_OCP, LD_F1, LD_P1H, LD_W2C, P1H_RP, conv2_offsets,  # noqa: E402
                            extra_cycles, kernel_dg_order, lanes)

TS, X_LD = 4, 804
XCP = TS * X_LD + 32
P1H_SZ = 12 * P1H_RP
DC2_LD = 80
DC2_SZ = 20 * DC2_LD + 24
DCH_SZ = 64 * DG_OCP + 120
I1_LD = 148
I1_SZ = 10 * I1_LD
DY1_LD = 584
DY1_SZ = 10 * DY1_LD
DG_KS = 19
# static weight images (LDS offset 0), dynamic carve after them (W_BYTES = 65536: bank-aligned)
S_W2C, S_W2D, S_F1 = 0, 21 * LD_W2C * 2, 21 * LD_W2C * 2 + DG_CH * 16 * 16
W = 65536
F_END = (4 * 20 + 4 * 52 + 4 * 64 + 4 + 2 * 4 + 3) // 4 * 4
D_PAR = W + 16 * 32 * 2
D_COFF = D_PAR + 592 * 4
D_DGT = D_COFF + 64 * 2
D_ONES = D_DGT + 4 * 20 * 4
D_ZERO = D_ONES + 192 * 2
D_X = D_ZERO + 192 * 2
D_P1H = D_X + (2 * XCP * 2 + 15) // 16 * 16
D_I1 = D_P1H + TS * P1H_SZ * 2
D_P2 = D_I1 + TS * I1_SZ
D_I2 = D_P2 + TS * 320 * 2
D_F = D_I2 + TS * 320
D_DZ1B = D_F + F_END * 4
D_DC2 = D_DZ1B + TS * 64 * 2
D_DCH = D_DC2 + TS * DC2_SZ * 2


def DY1(s):
    return (D_P1H if s < 2 else D_DC2) + (s & 1) * DY1_SZ * 2


def conv1():
    rd = wr = 0
    for wave in range(16):
        wsmp, wq = wave >> 2, wave & 3
        for k in range(9):
            xs = wsmp * X_LD + wq * 168 + (k // 3) * 56 + 8 * (k % 3)
            a = {n: [] for n in ("r0", "r1", "e4", "r2", "e2")}
            for lane, l16, kq in lanes():
                q1 = l16 & 3
                xl = (q1 >> 1) * 28 + 2 * (l16 >> 2) + (q1 & 1)
                o1 = xl + 28 * kq
                o2 = xl + 112 + (2 if kq == 1 else 0)
                xr1 = (o1 & 1) * XCP + (o1 & ~1)
                xr2 = (o2 & 1) * XCP + (o2 & ~1)
                a["r0"].append(D_X + 2 * (xr1 + xs))
                a["r1"].append(D_X + 2 * (xr1 + xs) + 4)
                a["e4"].append(D_X + 2 * (o1 + 4 + xs))
                a["r2"].append(D_X + 2 * (xr2 + xs))
                a["e2"].append(D_X + 2 * (o2 + 2 + xs))
            rd += sum(extra_cycles(v, 4 if n[0] == "r" else 2) for n, v in a.items())
            mt3, mtr = 3 * wq + k // 3, k % 3
            act = [l16 < 10 for lane, l16, kq in lanes()]
            p1h = [D_P1H + 2 * (wsmp * P1H_SZ + mt3 * P1H_RP + 4 * mtr * LD_P1H + kq * LD_P1H + min(l16, 9))
                   for lane, l16, kq in lanes()]
            i1 = [D_I1 + wsmp * I1_SZ + 4 * (3 * mt3 + mtr) + min(l16, 9) * I1_LD + kq for lane, l16, kq in lanes()]
            wr += extra_cycles(p1h, 2, "write", act) + extra_cycles(i1, 1, "write", act)
    return {"conv1 X reads": rd, "conv1 P1H / I1 writes": wr}


def conv2():
    tab = conv2_offsets()
    ra = rb = wr = 0
    for wave in range(16):
        s, mt = wave >> 2, wave & 3
        for ks in range(13):
            A, B0, B1 = [], [], []
            for lane, l16, kq in lanes():
                m = mt * 16 + l16
                p, q = m >> 2, m & 3
                oy, ox = 2 * (p >> 2) + (q >> 1), 2 * (p & 3) + (q & 1)
                A.append(D_P1H + 2 * (s * P1H_SZ + oy * P1H_RP + ox * LD_P1H + tab[kq, ks]))
                B0.append(S_W2C + 2 * (min(l16, 20) * LD_W2C + 8 * kq + ks * 32))
                B1.append(S_W2C + 2 * (min(16 + l16, 20) * LD_W2C + 8 * kq + ks * 32))
            ra += extra_cycles(A, 16)
            rb += extra_cycles(B0, 16) + extra_cycles(B1, 16)
        for nt in range(2):
            act = [nt * 16 + l16 < 20 for lane, l16, kq in lanes()]
            p2 = [D_P2 + 2 * (s * 320 + (nt * 16 + l16) * 16 + mt * 4 + kq) for lane, l16, kq in lanes()]
            i2 = [D_I2 + (s * 320 + (nt * 16 + l16) * 16 + mt * 4 + kq) for lane, l16, kq in lanes()]
            wr += extra_cycles(p2, 2, "write", act) + extra_cycles(i2, 1, "write", act)
    return {"conv2 A": ra, "conv2 B": rb, "conv2 P2 / I2 writes": wr}


def wgrad2():
    ra = rb = 0
    for wave in range(16):
        ntap = 2 if wave < 10 else 1
        taps = [min(wave + 16 * t, 24) for t in range(ntap)]
        bias = [False, wave == 9]
        for j in range(2 * TS):
            ss, ps = j >> 1, j & 1
            a0 = [D_DC2 + 2 * (min(l16, 19) * DC2_LD + 8 * kq + ss * DC2_SZ + ps * 32) for lane, l16, kq in lanes()]
            a1 = [D_DC2 + 2 * (min(16 + l16, 19) * DC2_LD + 8 * kq + ss * DC2_SZ + ps * 32) for lane, l16, kq in lanes()]
            ra += extra_cycles(a0, 16) + extra_cycles(a1, 16)
            for t in range(ntap):
                if bias[t]:
                    continue
                kh, kw = taps[t] // 5, taps[t] % 5
                for extra in (0, 4 * LD_P1H):
                    addrs = [D_P1H + 2 * ((kq + kh) * P1H_RP + ((l16 >> 2) + kw) * LD_P1H + 4 * (l16 & 3)
                                          + ss * P1H_SZ + 4 * ps * P1H_RP + extra) for lane, l16, kq in lanes()]
                    rb += extra_cycles(addrs, 8)
    return {"conv2 wgrad A (dL/dconv2)": ra, "conv2 wgrad B (tr16 pool1)": rb}


def dgrad():
    order = kernel_dg_order()
    ra = rb = ri = wr = 0
    for wave in range(16):
        ntl = 3 if wave < 4 else 2
        for i in range(ntl):
            RT = wave + 16 * i
            ss = RT // 9
            info = []
            tl = RT - 9 * ss  # 4 x 4 pixel block tl (lenet_tile.hip dgrad)
            for lane, l16, kq in lanes():
                info.append(((tl // 3) * 4 + (l16 >> 2), (tl % 3) * 4 + (l16 & 3)))
            for ks in range(DG_KS):
                A = []
                for lane, l16, kq in lanes():
                    kgd = order[min(4 * ks + kq, 74)]
                    tap, ocg = kgd // 3, kgd % 3
                    ty, tx = tap // 5, tap % 5
                    y, x = info[lane]
                    ok = 0 <= y + ty - 4 < 8 and 0 <= x + tx - 4 < 8
                    rel = (ty * 8 + tx) * DG_OCP + ocg * 8
                    A.append(D_DCH + 2 * (ss * DCH_SZ + ((y - 4) * 8 + (x - 4)) * DG_OCP + rel) if ok else D_ZERO)
                ra += extra_cycles(A, 16)
                if i == 0:
                    rb += extra_cycles([S_W2D + 2 * ((kq * 16 + l16) * 8 + ks * 512) for lane, l16, kq in lanes()], 16)
            p0 = [((tl // 3) * 4 + kq) * 12 + (tl % 3) * 4 for lane, l16, kq in lanes()]
            ri += extra_cycles([D_I1 + ss * I1_SZ + min(l16, 9) * I1_LD + p0[lane] for lane, l16, kq in lanes()], 4)
            act = [l16 < 10 for lane, l16, kq in lanes()]
            for dy in range(2):
                addrs = []
                for lane, l16, kq in lanes():
                    py, px0 = p0[lane] // 12, p0[lane] % 12
                    addrs.append(DY1(ss) + 2 * (min(l16, 9) * DY1_LD + 2 * py * 24 + 2 * px0 + dy * 24))
                wr += extra_cycles(addrs, 16, "write", act)
    return {"dgrad A (DCH)": ra, "dgrad B (W2D)": rb, "dgrad I1 reads": ri, "dgrad DY1 writes": wr}


def wgrad1():
    ra = rb = 0
    for wave in range(16):
        ss, rbase = wave >> 2, 36 * ((wave >> 1) & 1)
        for j in range(9):
            A, B = [], [[], [], [], []]
            for lane, l16, kq in lanes():
                kcol = (wave & 1) * 16 + l16
                kc = min(kcol, 24)
                kh, kw = kc // 5, kc % 5
                r = rbase + kq + 4 * j
                oh, ow0 = r // 3, 8 * (r % 3)
                A.append(DY1(ss) + 2 * (min(l16, 9) * DY1_LD + 8 * r))
                if kcol < 25:
                    xb = D_X + 2 * ((kw & 1) * XCP + ss * X_LD + kh * 28 + (kw & ~1) + oh * 28 + ow0)
                else:
                    xb = D_ONES if kcol == 25 else D_ZERO
                for d in range(4):
                    B[d].append(xb + 4 * d)
            ra += extra_cycles(A, 16)
            rb += sum(extra_cycles(b, 4) for b in B)
    return {"conv1 wgrad A (dL/dconv1)": ra, "conv1 wgrad B (X runs)": rb}


def stage5_writes():
    wr = 0
    for wave in range(16):
        for tt in range(2):
            t = wave + 16 * tt
            if t >= 20:
                continue
            for dy in range(2):
                addrs = [D_DC2 + 2 * (kq * DC2_SZ + t * DC2_LD + (2 * (l16 >> 2) + dy) * 8 + 2 * (l16 & 3))
                         for lane, l16, kq in lanes()]
                wr += extra_cycles(addrs, 4, "write")
            for pos in range(4):
                addrs = [D_DCH + 2 * (kq * DCH_SZ + ((2 * (l16 >> 2) + (pos >> 1)) * 8 + 2 * (l16 & 3) + (pos & 1)) * DG_OCP + t)
                         for lane, l16, kq in lanes()]
                wr += extra_cycles(addrs, 2, "write")
    return {"stage5 DC2 / DCH writes": wr}


def dp2():
    tr = 0
    for wave in range(16):
        for tt in range(2 if wave < 4 else 1):
            t = wave + 16 * tt
            for base in (0, 4, 32, 36):
                addrs = [S_F1 + 2 * (min(base + 8 * kq + (l16 >> 2), 50) * LD_F1 + 4 * (l16 & 3) + t * 16)
                         for lane, l16, kq in lanes()]
                tr += extra_cycles(addrs, 8)
    return {"dP2 transposed fc1 reads": tr}


if __name__ == "__main__":
    total = 0
    for fn in (conv1, conv2, dp2, stage5_writes, wgrad2, dgrad, wgrad1):
        for name, v in fn().items():
            total += v
            print(f"{name:32s} {v:7d} extra LDS cycles / tile")
    print(f"{'total (modelled sites)':32s} {total:7d}")
