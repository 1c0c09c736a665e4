"""LDS bank-conflict model for the conv kernels' fragment reads and staging stores (host-only).

Per wave instruction, lanes are serviced in fixed groups (MI355X LDS table: ds_read_b128 4 x 16
lanes over 64 banks, ds_read_b64 / ds_read_b64_tr_b16 2 x 32 lanes over 64 banks, ds_write_b128
8 x 8 lanes over 32 banks); a group costs as many LDS cycles as the most distinct dwords on one
bank. Prints cycles vs the conflict-free ideal for conv2 forward's A (image) and B (weight)
fragment reads and the W2 staging stores, with and without the odd-8-row weight swizzle
(csrc/kernels/mnist.hip c2f_wrow).

    python tools/debug/lds_banks.py
"""
G128 = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27], [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
G128 += [[lane + 32 for lane in g] for g in G128]
C2F_W, C2F_PLANE, C2F_WLD = 24, 18 * 24, 48


def cycles(addrs, kind):
    """addrs: byte address per lane (None = inactive); returns (cycles, conflict-free cycles)."""
    if kind == "r128":
        groups, nd, nb = G128, 4, 64
    elif kind == "tr64":
        groups, nd, nb = [list(range(0, 32)), list(range(32, 64))], 2, 64
    elif kind == "w128":
        groups, nd, nb = [list(range(i, i + 8)) for i in range(0, 64, 8)], 4, 32
    else:
        raise ValueError(kind)
    tot = 0
    for g in groups:
        banks = {}
        for lane in g:
            if addrs[lane] is None:
                continue
            for d in range(nd):
                dw = addrs[lane] // 4 + d
                banks.setdefault(dw % nb, set()).add(dw)
        tot += max((len(v) for v in banks.values()), default=1)
    return tot, len(groups)


def wrow(r, swizzle):
    """plain: r * 48; swizzled: groups of 8 rows 384 apart, rows 32 apart, odd groups +16."""
    if not swizzle:
        return r * C2F_WLD
    return (r >> 3) * 384 + (r & 7) * 32 + ((r >> 3) & 1) * 16


def conv2_fwd_a():
    tot = ideal = 0
    for w in range(8):
        for j in range(2):
            for tap in range(25):
                kh, kw = divmod(tap, 5)
                toff = (kh * C2F_W + kw) * 8
                out = []
                for lane in range(64):
                    g, m, px = lane >> 4, (w + 8 * j) * 16 + (lane & 15), 0
                    if m < 196:
                        pp, win = m >> 2, m & 3
                        px = (2 * (pp // 7) + (win >> 1)) * C2F_W + 2 * (pp % 7) + (win & 1)
                    out.append(((g * C2F_PLANE + px) * 8 + toff) * 2)
                c, n = cycles(out, "r128")
                tot, ideal = tot + c, ideal + n
    return tot, ideal


def conv2_fwd_b(swizzle):
    tot = ideal = 0
    for _w in range(8):
        for tap in range(25):
            for half in range(2):
                for second in range(2):
                    out = []
                    for lane in range(64):
                        g, q, p4 = lane >> 4, (lane & 15) >> 2, lane & 3
                        out.append((wrow(tap * 32 + 8 * g + q + 4 * second, swizzle) + 4 * p4 + 16 * half) * 2)
                    c, n = cycles(out, "tr64")
                    tot, ideal = tot + c, ideal + n
    return tot, ideal


def w2_store(swizzle):
    tot = ideal = 0
    for w in range(4):
        for j in range(13):
            out = []
            for lane in range(64):
                i = w * 64 + lane + 256 * j
                out.append((wrow(i >> 2, swizzle) + (i & 3) * 8) * 2 if i < 3200 else None)
            c, n = cycles(out, "w128")
            tot, ideal = tot + c, ideal + n
    return tot, ideal


if __name__ == "__main__":
    print("conv2 fwd A reads (8 waves): %d LDS cycles, ideal %d" % conv2_fwd_a())
    for sw in (False, True):
        print("conv2 fwd B reads, swizzle=%s: %d, ideal %d" % ((sw,) + conv2_fwd_b(sw)))
        print("W2 staging stores, swizzle=%s: %d, ideal %d" % ((sw,) + w2_store(sw)))


# ---- conv2 dgrad (conv2_dgrad_lds): image [8 chunks][224 px] x 16 B, weights [800][72]
C2D_COLS, C2D_PLANE, C2D_WLD = 20, 224, 72


def conv2_dgrad(wld=C2D_WLD):
    ta = tb = ia = ib = 0
    for w in range(8):
        mt0, kq = w & 3, w >> 2
        for tap in (range(13, 25) if kq else range(13)):
            kh, kw = divmod(tap, 5)
            for sk in range(2):
                coff = -(kh * C2D_COLS + kw) * 8 + sk * 4 * C2D_PLANE * 8
                for j in range(2):
                    out = []
                    for lane in range(64):
                        g, iw = lane >> 4, lane & 15
                        base = ((mt0 + 4 * j + 4) * C2D_COLS + iw + 4) * 8 + g * C2D_PLANE * 8
                        out.append((base + coff) * 2)
                    c, n = cycles(out, "r128")
                    ta, ia = ta + c, ia + n
                for half in range(2):
                    out = []
                    for lane in range(64):
                        g = lane >> 4
                        out.append(((lane & 15) * wld + 8 * g + tap * 32 * wld + sk * 32 + half * 16 * wld) * 2)
                    c, n = cycles(out, "r128")
                    tb, ib = tb + c, ib + n
    return ta, ia, tb, ib


if __name__ == "__main__":
    print("conv2 dgrad A reads: %d, ideal %d; B reads: %d, ideal %d" % conv2_dgrad())
    for wld in (64, 68, 72, 76, 80, 88):
        print("  dgrad weight pitch", wld, "-> B %d (ideal %d)" % conv2_dgrad(wld)[2:])


# ---- conv2 wgrad (conv2_wgrad_lds): image [18][18] x CS ch, dz2 rows [224][DS]; both via tr reads
def conv2_wgrad(cs=40, ds=72):
    PW = 18
    ta = tb = ia = ib = 0
    for w in range(8):
        h, n = w >> 2, w & 3
        for s in range(7):
            for second in range(2):  # frag_tr16 = two ds_read_b64_tr_b16 (rows +0 / +4)
                out = []
                for lane in range(64):
                    g, q, p4 = lane >> 4, (lane & 15) >> 2, lane & 3
                    out.append((((32 * s + 8 * g + q + 4 * second) * ds) + 16 * n + 4 * p4) * 2)
                c, m = cycles(out, "tr64")
                tb, ib = tb + c, ib + m
            for tap in range(7):
                toff = (tap // 5) * PW + tap % 5
                for u in range(2):
                    out = []
                    for lane in range(64):
                        g, q, p4 = lane >> 4, (lane & 15) >> 2, lane & 3
                        k = 32 * s + 8 * g + q + 4 * u
                        pos = (k // 14) * PW + (k % 14) if k < 196 else 0
                        out.append(((pos + toff) * cs + 16 * h + 4 * p4) * 2)
                    c, m = cycles(out, "tr64")
                    ta, ia = ta + c, ia + m
    return ta, ia, tb, ib


if __name__ == "__main__":
    print("conv2 wgrad (per image, 7 taps): A %d (ideal %d), B %d (ideal %d)" % conv2_wgrad())
    for cs in (32, 36, 40, 44, 48):
        for ds in (64, 68, 72, 80):
            r = conv2_wgrad(cs, ds)
            print("  cs", cs, "ds", ds, "-> A %d B %d (ideal %d / %d)" % (r[0], r[2], r[1], r[3]))
