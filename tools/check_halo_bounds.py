"""CPU-side bounds check of the halo conv's global accesses (conv_halo.hip), for every launch
shape of the bench configs (and small ragged shapes).

The kernel reads and writes global memory only through raw-buffer instructions whose descriptor
covers 2 GB from a wave-uniform base (dma::rsrc / dma::brsrc, num_records 0x7FFFFFF0): a lane is
either "out of range" (voffset = dma::OOB = 0x80000000: the load returns 0, the store is dropped)
or addresses base + voffset with NO check against the tensor's extent.  So an illegal address can
only come from an in-range voffset that lands outside the tensor.  This restates, lane by lane,
the address arithmetic of the shipped kernel (issue_prep / issue_piece: the halo patch pieces,
16 LDS rows x 4 pieces of 16 B per instruction; the weight pieces; r_off / load_route of the
fused BN backward; the epilogue stores) and checks, for every in-range lane, that
  * its 16 bytes lie inside the tensor it addresses (pixel index < n*h*w, channels inside the
    view row: off + c + 8 <= ld for bf16),
  * its voffset is < 0x7FFFFFF0 (else the access would be silently dropped), and
  * out-of-range lanes carry OOB (never a wrapped small offset).
Only the boundary tiles are enumerated (first / last tile row and column of the first and last
image): the offsets are affine in the tile position, so the extremes are there.

    python tools/check_halo_bounds.py        (exit status 1 on a violation)

Round-6 finding: the round-5 variant library that faulted (liblines.so,
gpurun_out/r05p_ab.txt) is not in the tree; every access pattern of the SHIPPED kernel is inside
its tensor by this check.
"""
import itertools
import sys

import numpy as np

TH, TW, NWAVE, KT = 16, 32, 8, 9
PW = TW + 2
OOB = 0x80000000
NREC = 0x7FFFFFF0


def pair_perm(nn):
    # igemm_common.h pair_perm: row nn of a 32-column pair holds GEMM column pair_perm(nn)
    # (a permutation inside each 32-column pair; its exact form does not matter for bounds as
    # long as it stays inside the pair)
    return nn


def check_launch(name, n, h, w, cin, N, ld_in, off_in, ld_out, off_out, es=2, epi=1, bnb=None, route=None,
                 line=64):
    """One halo launch: input view (n, h, w, ld_in, off_in) with cin channels, N output columns
    written into (ld_out, off_out).  bnb = (c0, c1, r_ld, r_off); route = pool_ld.  line: bytes
    of a pixel row one patch instruction reads per 32-channel chunk (64: the shipped 16 rows x
    4 pieces; 128: the full-line 8 rows x 8 pieces shape the round-5 variant tried, which reads the
    chunk's line-mate as well).  Returns a list of violations."""
    cc = 64 // es                       # channels per chunk (64-byte LDS rows)
    pe = 16 // es                       # channels per 16-byte piece
    bn = 32 if route else (64 if N % 64 == 0 else 32)
    nch = cin // cc
    nblk = N // bn
    prows = (TH + 2) * PW
    ppc = (prows + 15) // 16
    npi = (ppc + NWAVE - 1) // NWAVE
    bpc = KT * bn // 16
    nbi = (bpc + NWAVE - 1) // NWAVE
    tiles_x, tiles_y = (w + TW - 1) // TW, (h + TH - 1) // TH
    K = KT * cin
    bad = []
    lane = np.arange(64)
    lpr = line // 16                    # lanes (16-byte pieces) per patch row in one instruction
    lrow, lpc = lane // lpr, lane % lpr
    rpi = 64 // lpr                     # patch rows per instruction
    npi = (prows + rpi - 1) // rpi // NWAVE + 1
    xs = sorted({0, tiles_x - 1})
    ys = sorted({0, tiles_y - 1})
    imgs = sorted({0, n - 1})
    in_elems = n * h * w * ld_in
    for img, ty, tx in itertools.product(imgs, ys, xs):
        y0, x0 = ty * TH, tx * TW
        for ch in sorted({0, nch - 1}):
            c = ch * cc
            # patch pieces: the patch origin may be pixel -1 (pbase before the tensor); each lane's
            # voffset is relative to it
            po = (img * h + y0 - 1) * w + x0 - 1
            for wave in range(NWAVE):
                for i in range(npi):
                    row = (wave * npi + i) * rpi + lrow
                    piece = lpc ^ (((row >> 2) & 1) << 1) if lpr == 4 else lpc
                    py, px = row // PW, row % PW
                    yy = np.where(row < prows, y0 + py - 1, -(1 << 29))
                    xx = x0 + px - 1
                    ok = (yy >= 0) & (yy < h) & (xx >= 0) & (xx < w)
                    voff = ((py * w + px) * ld_in + piece * pe) * es
                    if np.any(voff[ok] >= NREC):
                        bad.append((name, "patch voffset >= num_records"))
                    pix = po + py * w + px  # absolute pixel of an in-range lane
                    e0 = pix * ld_in + off_in + c + piece * pe
                    okb = (pix >= 0) & (pix < n * h * w) & (off_in + c + piece * pe + pe <= ld_in) & (e0 + pe <= in_elems)
                    if np.any(ok & ~okb):
                        bad.append((name, f"patch piece outside the input (img {img}, tile {ty},{tx}, chunk {ch})"))
            # weight pieces (per column block)
            for nb in sorted({0, nblk - 1}):
                n0 = nb * bn
                for wave in range(NWAVE):
                    for i in range(nbi):
                        row = (wave * nbi + i) * 16 + (lane >> 2)
                        piece = (lane & 3) ^ (((row >> 2) & 1) << 1)
                        tap, nn = row // bn, row % bn
                        ok = row < KT * bn
                        e0 = n0 * K + c + pair_perm(nn) * K + tap * cin + piece * pe
                        if np.any(ok & ((e0 < 0) | (e0 + pe > N * K))):
                            bad.append((name, "weight piece outside the weights"))
        # stores / r / route of the epilogue, per column block and wave
        for nb in sorted({0, nblk - 1}):
            n0 = nb * bn
            for wave in range(NWAVE):
                oh0 = y0 + wave * 2
                for f in range(4):
                    rr, col = f // 2, (f % 2) * 16 + (lane & 15)
                    g = lane >> 4
                    ok = (oh0 + rr < h) & (x0 + col < w)
                    pix = (img * h + oh0 + rr) * w + x0 + col
                    for q in range(bn // 32):
                        cl = 32 * q + 8 * g
                        if bnb is None:
                            e0 = pix * ld_out + off_out + n0 + cl
                            okb = (pix < n * h * w) & (off_out + n0 + cl + 8 <= ld_out)
                            if np.any(ok & ~okb):
                                bad.append((name, "store outside the output"))
                            voff = ((rr * w + col) * ld_out + cl) * es
                            if np.any(voff[ok] >= NREC):
                                bad.append((name, "store voffset >= num_records"))
                        else:
                            c0, c1, r_ld, r_off = bnb
                            cabs = n0 + cl
                            rok = ok & (cabs >= c0) & (cabs < c1)
                            e0 = pix * r_ld + r_off + cabs - c0
                            okb = (pix < n * h * w) & (r_off + cabs - c0 + 8 <= r_ld)
                            if np.any(rok & ~okb):
                                bad.append((name, "r load outside r"))
                            voff = ((rr * w + col) * r_ld + (cabs - c0)) * es
                            if np.any(voff[rok] >= NREC):
                                bad.append((name, "r voffset >= num_records"))
                            # dz [M][c1-c0] (fused columns) / g into the out view (the others)
                            zok = pix < n * h * w
                            if np.any(rok & ~zok) or np.any(ok & ~rok & ~((pix < n * h * w) & (off_out + cabs + 8 <= ld_out))):
                                bad.append((name, "dz / g store outside its tensor"))
                        if route:
                            pl = route
                            pb = ((img * (h // 2) + (oh0 // 2)) * (w // 2) + x0 // 2)
                            pix2 = pb + (f % 2) * 8 + ((lane & 15) >> 1)
                            okr = (oh0 < h) & (x0 + col < w)
                            if np.any(okr & ((pix2 >= n * (h // 2) * (w // 2)) | (n0 + cl + 8 > pl))):
                                bad.append((name, "route load outside the pooled gradient"))
    return bad


def bench_launches():
    """(name, args) of the halo launches of the bench configs (1080p padded to 1088, 4K) and of
    ragged small frames (partial tiles in both directions)."""
    L = []
    for (H, W, n) in ((1088, 1920, 32), (2160, 3840, 8), (34, 70, 2), (20, 40, 2)):
        lv = lambda k: (H >> k, W >> k)  # noqa: E731
        for name, k, cin, cout in (("enc1b", 0, 32, 32), ("enc2b", 1, 64, 64), ("enc3a", 2, 64, 128),
                                   ("enc3b", 2, 128, 128), ("enc4a", 3, 128, 256), ("enc4b", 3, 256, 256),
                                   ("crossa", 4, 256, 512), ("crossb", 4, 512, 512), ("dec6", 3, 768, 512),
                                   ("dec7", 2, 384, 256), ("dec8", 1, 192, 128)):
            h, w = lv(k)
            if h < 1 or w < 1 or h % 2 or w % 2:
                continue
            L.append((f"{name} fwd {n}x{h}x{w}", (n, h, w, cin, cout, cin, 0, cout, 0)))
            L.append((f"{name} dgrad {n}x{h}x{w}", (n, h, w, cout, cin, cout, 0, cin, 0)))
            # decoder dgrads with the up columns fused (parity sums), r read from the concat view
            if name.startswith("dec"):
                up = cout  # the up member of the concat: its last cout channels
                L.append((f"{name} dgrad_bn {n}x{h}x{w}", (n, h, w, cout, cin, cout, 0, cin, 0),
                          dict(epi=2, bnb=(cin - up, cin, cin, cin - up))))
                # the deferred skip columns with the pool route: dz [.., cin - up] with pooled rows
                L.append((f"{name} dgrad_bn+route {n}x{h}x{w}", (n, h, w, cout, cin - up, cout, 0, cin - up, 0),
                          dict(epi=2, bnb=(0, cin - up, cin - up, 0), route=cin - up)))
        h, w = H, W
        # dec9: the [conv1 32 | up9 64] concat as two sources (fwd), its up columns' fused dgrad
        L.append((f"dec9 fwd(up) {n}x{h}x{w}", (n, h, w, 64, 64, 64, 0, 64, 0)))
        L.append((f"dec9 dgrad_bn(up) {n}x{h}x{w}", (n, h, w, 64, 64, 64, 0, 64, 0), dict(epi=2, bnb=(0, 64, 64, 0))))
        L.append((f"dec9 dgrad_bn+route {n}x{h}x{w}", (n, h, w, 64, 32, 64, 0, 32, 0),
                  dict(epi=2, bnb=(0, 32, 32, 0), route=32)))
    return L


def run(line=64):
    bad, n = [], 0
    for item in bench_launches():
        name, a = item[0], item[1]
        kw = item[2] if len(item) > 2 else {}
        nn, h, w, cin, N, ld_in, off_in, ld_out, off_out = a
        bad += check_launch(name, nn, h, w, cin, N, ld_in, off_in, ld_out, off_out, line=line, **kw)
        n += 1
    return bad, n


def main():
    bad, n = run()
    for b in bad[:20]:
        print("VIOLATION", *b)
    print(f"{n} launches checked, {len(bad)} violations")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
