#!/usr/bin/env python3
"""numpy emulation of k_conv3m's data path (csrc/conv3m.hip) against a direct circular 3x3 conv:
the halo LDS-DMA placement (slot 16 i + l/4, physical piece l % 4 reading logical piece
(l % 4) ^ sw(col)), the fragment-ordered weight copy of tcx_pack_conv_weight_h2_frag staged per tap
pair in the ring, the per-lane A addresses aq[q] (+ row-block immediates, ^16 for lo), the per-lane
B gather address bq, and v_mfma_f32_16x16x32_f16 (A[i][k] from lane i + 16 (k // 8), B[k][j] from
lane j + 16 (k // 8), D[4 (l >> 4) + r][l & 15]).  hi / lo pieces carry independent random integers
so a mix-up of pieces, taps, chunks or lanes changes the result.  Also checks the A-read bank rule of
the ds_read_b128 lane groups (MI355X_MICROARCH.md §LDS) for every pair type and row block.
"""
import numpy as np

GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
          list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
GROUPS += [[l + 32 for l in g] for g in GROUPS]


def sw(col):
    return (col >> 2) & 1


def run(W, H, Cin, Cout=96, seed=0):
    rng = np.random.default_rng(seed)
    TP, W2 = 256, W + 2
    NPX = (TP // W + 2) * W2
    NI = (NPX + 15) // 16
    cpt = Cin // 16
    npair = 9 * cpt // 2
    # h2 record values: xh/xl [H][W][Cin], weights wh/wl [Cout][Cin][3][3]
    xh = rng.integers(-3, 4, (H, W, Cin)).astype(np.float64)
    xl = rng.integers(-3, 4, (H, W, Cin)).astype(np.float64)
    wh = rng.integers(-3, 4, (Cout, Cin, 3, 3)).astype(np.float64)
    wl = rng.integers(-3, 4, (Cout, Cin, 3, 3)).astype(np.float64)

    def conv(a, w):
        out = np.zeros((H, W, Cout))
        for dy in range(3):
            for dx in range(3):
                src = np.roll(np.roll(a, 1 - dy, 0), 1 - dx, 1)  # src[y][x] = a[y+dy-1][x+dx-1]
                out += np.einsum("yxc,oc->yxo", src, w[:, :, dy, dx])
        return out
    ref = conv(xh, wl) + conv(xl, wh) + conv(xh, wh)

    # fragment-ordered weights: wf[c][n][hl][lane][8]  (one n block of 96)
    nch = 9 * cpt
    wf = np.zeros((nch, 3, 2, 64, 8))
    for c in range(nch):
        j, t = divmod(c, 9)
        dy, dx = divmod(t, 3)
        for n in range(3):
            for lane in range(64):
                row = 32 * n + (lane & 31)
                ci = j * 16 + 8 * (lane >> 5) + np.arange(8)
                wf[c, n, 0, lane] = wh[row, ci, dy, dx]
                wf[c, n, 1, lane] = wl[row, ci, dy, dx]
    ring_of_pair = lambda k: wf[2 * k: 2 * k + 2].reshape(-1)  # 12 KB = 6144 halves, byte b -> half b // 2

    out = np.zeros((H * W, Cout))
    r0_of_tile = lambda m0: (m0 % (H * W)) // W
    for m0 in range(0, H * W, TP):
        r0 = r0_of_tile(m0)

        def halo_image(j):
            """LDS image of chunk j: [NI*16 slots][4 pieces][8] as the DMA fills it"""
            img = np.zeros((NI * 16, 4, 8))
            for i in range(NI):
                for lane in range(64):
                    sl = 16 * i + lane // 4
                    hr, hc = divmod(sl, W2)
                    hcs = hc
                    if sl >= NPX:
                        hr, hc = divmod(NPX - 1, W2)
                    y = (r0 + hr - 1) % H
                    x = (hc - 1) % W
                    logical = (lane & 3) ^ sw(hcs)
                    g, hl = divmod(logical, 2)
                    ch = j * 16 + 8 * g + np.arange(8)
                    img[sl, lane & 3] = (xh if hl == 0 else xl)[y, x, ch]
            return img.reshape(-1)  # halves; byte b -> half b // 2

        for wv in range(4):
            acc = np.zeros((4, 6, 64, 4))
            aq = np.zeros((9, 64), dtype=np.int64)
            for lane in range(64):
                li, g, th = lane & 15, (lane >> 4) & 1, lane >> 5
                mloc = wv * 64 + li
                rr, cc = divmod(mloc, W)
                for q in range(9):
                    c = 2 * q + th
                    hb = 1 if c >= 9 else 0
                    t = c - 9 * hb
                    dy, dx = divmod(t, 3)
                    aq[q, lane] = hb * (NI * 1024) + ((rr + dy) * W2 + cc + dx) * 64 + 16 * ((2 * g) ^ sw(cc + dx))

            def rbo(rb):
                return rb * 16 * 64 if W == 64 else ((rb >> 1) * W2 * 64 + (rb & 1) * 16 * 64 if W == 32 else rb * W2 * 64)
            bq = np.array([(l >> 5) * 6144 + ((l >> 4) & 1) * 512 + (l & 15) * 16 for l in range(64)])
            for pp in range(cpt // 2):
                lds = np.concatenate([halo_image(2 * pp), halo_image(2 * pp + 1)])
                for q in range(9):
                    k = 9 * pp + q
                    ring = ring_of_pair(k)
                    # bank check of the A reads
                    for rb in range(4):
                        for lo in (0, 1):
                            addr = (aq[q] ^ (16 * lo)) + rbo(rb)
                            for grp in GROUPS:
                                qs = [(int(addr[l]) // 16) % 16 for l in grp]
                                assert len(set(qs)) == 16, (W, q, rb, lo, qs)
                    for rb in range(4):
                        A = {}
                        for lo in (0, 1):
                            addr = (aq[q] ^ (16 * lo)) + rbo(rb)
                            A[lo] = np.stack([lds[a // 2: a // 2 + 8] for a in addr])  # [64][8]
                        for nb in range(6):
                            B = {}
                            for hl in (0, 1):
                                off = bq + (nb >> 1) * 2048 + (nb & 1) * 256 + hl * 1024
                                B[hl] = np.stack([ring[o // 2: o // 2 + 8] for o in off])
                            for (ai, bi) in ((0, 1), (1, 0), (0, 0)):  # hi.lo, lo.hi, hi.hi
                                Am = np.zeros((16, 32))
                                Bm = np.zeros((32, 16))
                                for l in range(64):
                                    Am[l & 15, 8 * (l >> 4): 8 * (l >> 4) + 8] = A[ai][l]
                                    Bm[8 * (l >> 4): 8 * (l >> 4) + 8, l & 15] = B[bi][l]
                                D = Am @ Bm
                                for l in range(64):
                                    acc[rb, nb, l] += D[4 * (l >> 4): 4 * (l >> 4) + 4, l & 15]
            for rb in range(4):
                for nb in range(6):
                    for l in range(64):
                        for r in range(4):
                            pix = m0 + 64 * wv + 16 * rb + 4 * (l >> 4) + r
                            out[pix, 16 * nb + (l & 15)] = acc[rb, nb, l, r]
    err = np.abs(out - ref.reshape(H * W, Cout)).max()
    print(f"W={W} H={H} Cin={Cin}: max |emulated - direct| = {err}")
    assert err == 0


if __name__ == "__main__":
    run(16, 16, 32)
    run(32, 8, 32)
    run(64, 4, 64)
    print("ok")
