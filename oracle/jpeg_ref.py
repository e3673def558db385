"""numpy restatement of the pixel half of the JPEG input pipeline (TEST INFRASTRUCTURE ONLY).

Checks vit.rs_amd/csrc/jpeg.hip.  Only tests/ may import this module; the product path never
does.  The reference (Rust ViT.rs) has no image decoder -- its forward takes a prepared input
array (/root/reference/train_vit.rs:188, encoder call :196) -- so the algorithms restated here are
the published IJG libjpeg ones that libjpeg-turbo implements (the library Pillow links; Pillow is
the pin: tests/test_jpeg_cpu.py requires this restatement to reproduce Pillow's decode of the same
files bit for bit):

* jpeg_idct_islow (libjpeg 6b jidctint.c): dequantise, 1-D passes over columns then rows with
  CONST_BITS = 13, PASS1_BITS = 2, descale by rounding shifts, +128 and the range-limit table
  (x & 1023 wrap-around) -- int32 arithmetic;
* "fancy" chroma upsampling (jdsample.c h2v1_fancy_upsample / h2v2_fancy_upsample): triangle
  filters, 3/4 nearer + 1/4 further sample with alternating rounding biases, edge rows replicated,
  plain replication when the component is <= 2 samples wide;
* YCbCr -> RGB (jdcolor.c build_ycc_rgb_table, SCALEBITS = 16);
then the pipeline's own crop / flip / bilinear resize in 1/256-pixel fixed point (jpeg.hip tap()).
"""
import numpy as np

CB, P1 = 13, 2
F0298, F0390, F0541, F0765, F0899, F1175 = 2446, 3196, 4433, 6270, 7373, 9633
F1501, F1847, F1961, F2053, F2562, F3072 = 12299, 15137, 16069, 16819, 20995, 25172
FIX_R, FIX_B, FIX_GR, FIX_GB = 91881, 116130, 46802, 22554
GRAY, YCC444, YCC422, YCC420 = 0, 1, 2, 3


def _descale(x, n):
    return (x + (1 << (n - 1))) >> n


def _idct8(x, sh):
    """x [..., 8] int64 -> [..., 8] (one libjpeg islow 1-D pass, values kept in int32 range)."""
    i = [x[..., k] for k in range(8)]
    z1 = (i[2] + i[6]) * F0541
    t2 = z1 + i[6] * (-F1847)
    t3 = z1 + i[2] * F0765
    t0 = (i[0] + i[4]) << CB
    t1 = (i[0] - i[4]) << CB
    t10, t13, t11, t12 = t0 + t3, t0 - t3, t1 + t2, t1 - t2
    o0, o1, o2, o3 = i[7], i[5], i[3], i[1]
    z1, z2, z3, z4 = o0 + o3, o1 + o2, o0 + o2, o1 + o3
    z5 = (z3 + z4) * F1175
    o0, o1, o2, o3 = o0 * F0298, o1 * F2053, o2 * F3072, o3 * F1501
    z1, z2, z3, z4 = z1 * -F0899, z2 * -F2562, z3 * -F1961 + z5, z4 * -F0390 + z5
    o0, o1, o2, o3 = o0 + z1 + z3, o1 + z2 + z4, o2 + z2 + z3, o3 + z1 + z4
    out = [t10 + o3, t11 + o2, t12 + o1, t13 + o0, t13 - o0, t12 - o1, t11 - o2, t10 - o3]
    return np.stack([_descale(v, sh) for v in out], -1)


def _range_limit(x):
    v = x & 1023
    return np.where(v < 128, v + 128, np.where(v < 512, 255, np.where(v < 896, 0, v - 896))).astype(np.uint8)


def idct_blocks(coef, qt):
    """coef [n][64] int16 (natural order), qt [64] -> [n][8][8] uint8."""
    d = coef.astype(np.int64).reshape(-1, 8, 8) * np.asarray(qt, np.int64).reshape(8, 8)
    ws = _idct8(d.transpose(0, 2, 1), CB - P1).transpose(0, 2, 1)   # columns
    return _range_limit(_idct8(ws, CB + P1 + 3))                       # rows


def parse_info(info):
    info = np.asarray(info)
    w, h, kind, nc = (int(v) for v in info[:4])
    comp = info[4:16].reshape(3, 4)
    qt = info[16:16 + 192].reshape(3, 64)
    return w, h, kind, nc, comp, qt


def planes(coef, info):
    """All component planes (uint8 [bh*8][bw*8]) of one image from its coefficients."""
    w, h, kind, nc, comp, qt = parse_info(info)
    out, o = [], 0
    for c in range(nc):
        bw, bh = int(comp[c, 0]), int(comp[c, 1])
        blk = idct_blocks(coef[o:o + bw * bh], qt[c])
        o += bw * bh
        out.append(blk.reshape(bh, bw, 8, 8).transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8))
    return out


def _up_h2v1(p, cw):
    p = p.astype(np.int64)[:, :cw]
    if cw <= 2:
        return np.repeat(p, 2, axis=1)
    left = np.concatenate([p[:, :1], p[:, :-1]], 1)
    right = np.concatenate([p[:, 1:], p[:, -1:]], 1)
    even = (3 * p + left + 1) >> 2
    odd = (3 * p + right + 2) >> 2
    even[:, 0] = p[:, 0]
    odd[:, -1] = p[:, -1]
    return np.stack([even, odd], -1).reshape(p.shape[0], 2 * cw)


def _up_h2v2(p, cw, ch):
    p = p.astype(np.int64)[:ch, :cw]
    if cw <= 2:
        return np.repeat(np.repeat(p, 2, axis=0), 2, axis=1)
    above = np.concatenate([p[:1], p[:-1]], 0)
    below = np.concatenate([p[1:], p[-1:]], 0)
    rows = []
    for nb in (above, below):
        cs = 3 * p + nb
        left = np.concatenate([cs[:, :1], cs[:, :-1]], 1)
        right = np.concatenate([cs[:, 1:], cs[:, -1:]], 1)
        even = (3 * cs + left + 8) >> 4
        odd = (3 * cs + right + 7) >> 4
        even[:, 0] = (4 * cs[:, 0] + 8) >> 4
        odd[:, -1] = (4 * cs[:, -1] + 7) >> 4
        rows.append(np.stack([even, odd], -1).reshape(ch, 2 * cw))
    return np.stack(rows, 1).reshape(2 * ch, 2 * cw)


def rgb_image(coef, info):
    """Full-resolution RGB uint8 [h][w][3] of one image (the libjpeg-turbo output)."""
    w, h, kind, nc, comp, qt = parse_info(info)
    pl = planes(coef, info)
    y = pl[0][:h, :w].astype(np.int64)
    if kind == GRAY:
        return np.repeat(y[..., None].astype(np.uint8), 3, -1)
    ch = []
    for c in (1, 2):
        cw_, chh = int(comp[c, 2]), int(comp[c, 3])
        if kind == YCC444:
            u = pl[c].astype(np.int64)
        elif kind == YCC422:
            u = _up_h2v1(pl[c][:chh], cw_)
        else:
            u = _up_h2v2(pl[c], cw_, chh)
        ch.append(u[:h, :w] - 128)
    cb, cr = ch
    r = y + ((FIX_R * cr + 32768) >> 16)
    g = y + ((-FIX_GB * cb + 32768 - FIX_GR * cr) >> 16)
    b = y + ((FIX_B * cb + 32768) >> 16)
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)


def _taps(n, b0, bl, length):
    o = np.arange(n, dtype=np.int64)
    s = (2 * o + 1) * bl * 128 // n - 128 + 256 * b0
    i = s >> 8
    f = s & 255
    return np.clip(i, 0, length - 1), np.clip(i + 1, 0, length - 1), f


def resize(rgb, box, img):
    """Crop box (x0, y0, w, h, flip) of rgb [H][W][3], bilinear to [img][img][3] uint8."""
    H, W, _ = rgb.shape
    x0, y0, bw, bh, flip = (int(v) for v in box)
    xi0, xi1, fx = _taps(img, x0, bw, W)
    yi0, yi1, fy = _taps(img, y0, bh, H)
    if flip:
        xi0, xi1, fx = xi0[::-1], xi1[::-1], fx[::-1]
    v = rgb.astype(np.int64)
    fx = fx[None, :, None]
    fy = fy[:, None, None]
    a = v[yi0][:, xi0]
    b = v[yi0][:, xi1]
    c = v[yi1][:, xi0]
    e = v[yi1][:, xi1]
    out = (a * (256 - fx) * (256 - fy) + b * fx * (256 - fy) + c * (256 - fx) * fy + e * fx * fy + 32768) >> 16
    return out.astype(np.uint8)


def normalise(u8, mean, std):
    """[B][img][img][3] uint8 -> fp32 [B][3][img][img]: (x / 255 - mean[c]) / std[c] in fp32."""
    x = u8.astype(np.float32) / np.float32(255.0)
    x = (x - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return np.ascontiguousarray(x.transpose(0, 3, 1, 2))
