"""numpy restatement of the MXFP8 block quantization used by the fp8 mode (test infrastructure).

Build-defined numerics (the reference has no low-precision path; BASELINE.json config 5 names
fp8 weights/activations): OCP fp8 e4m3fn values with one E8M0 scale per 32 consecutive
k-elements of a row.  Per block: X = ceil(log2(amax / 448)) (so amax / 2^X <= 448, the e4m3
maximum), scale byte X + 127 clamped to [0, 254] (127 for an all-zero block), elements
x / 2^X rounded to nearest even.  Scales are stored in the lane-native layout of
vit.rs_amd/csrc/gemm_fp8.hip: [K/64][Rpad/32][64] bytes, byte h*32 + r of row group g at step s =
scale of row 32g + r, block 2s + h; Rpad = rows rounded up to 256, padding rows carry 0.
"""
import numpy as np


def e4m3_round(y):
    """Nearest e4m3fn value (round half to even) of float64 y with |y| <= 448."""
    y = np.asarray(y, np.float64)
    a = np.abs(y)
    e = np.floor(np.log2(np.where(a > 0, a, 1.0)))
    e = np.maximum(e, -6.0)               # below 2^-6 the subnormal quantum 2^-9
    q = np.exp2(e - 3.0)
    return np.copysign(np.rint(a / q) * q, y)


def e4m3_encode(v):
    """e4m3fn bytes of exactly representable float64 values v."""
    v = np.asarray(v, np.float64)
    sign = np.signbit(v).astype(np.uint8) << 7
    a = np.abs(v)
    e = np.floor(np.log2(np.where(a > 0, a, 1.0)))
    normal = a >= 2.0 ** -6
    exp_f = np.where(normal, e + 7, 0).astype(np.int64)
    mant = np.where(normal, np.rint((a / np.exp2(e) - 1.0) * 8), np.rint(a / 2.0 ** -9)).astype(np.int64)
    return (sign | (exp_f << 3).astype(np.uint8) | mant.astype(np.uint8)).astype(np.uint8)


def e4m3_decode(b):
    b = np.asarray(b, np.uint8).astype(np.int64)
    s, e, m = b >> 7, (b >> 3) & 15, b & 7
    v = np.where(e == 0, m * 2.0 ** -9, (1.0 + m / 8.0) * np.exp2(e - 7.0))
    v = np.where((e == 15) & (m == 7), np.nan, v)
    return np.where(s == 1, -v, v)


def scale_bytes(amax):
    """E8M0 byte of X = ceil(log2(amax / 448)) + 127 from the fp32 bits of amax (as the GPU)."""
    amax = np.asarray(amax, np.float32)
    u = amax.view(np.uint32).astype(np.int64)
    ex, mant = (u >> 23) & 0xFF, u & 0x7FFFFF
    s = np.clip(ex - 8 + (mant > 0x600000), 0, 254)
    return np.where(amax > 0, s, 127).astype(np.uint8)


def rows_padded(r):
    return (r + 255) // 256 * 256


def quantize(x):
    """x [R][K] (float32 values) -> (q [R][K] e4m3 bytes, block scale bytes [R][K/32])."""
    x = np.asarray(x, np.float32)
    R, K = x.shape
    assert K % 64 == 0
    blocks = x.reshape(R, K // 32, 32)
    sb = scale_bytes(np.abs(blocks).max(-1))
    inv = np.exp2(127.0 - sb.astype(np.float64))[..., None]
    q = e4m3_encode(e4m3_round(blocks.astype(np.float64) * inv)).reshape(R, K)
    return q, sb


def to_lane_native(sb):
    """block scales [R][K/32] -> the lane-native [K/64][Rpad/32][64] bytes."""
    R, nb = sb.shape
    Rp = rows_padded(R)
    full = np.zeros((Rp, nb), np.uint8)
    full[:R] = sb
    # [rg][r][s][h] -> [s][rg][h][r]
    t = full.reshape(Rp // 32, 32, nb // 2, 2).transpose(2, 0, 3, 1)
    return np.ascontiguousarray(t).reshape(-1)


def from_lane_native(sl, R, K):
    Rp = rows_padded(R)
    t = np.asarray(sl, np.uint8).reshape(K // 64, Rp // 32, 2, 32).transpose(1, 3, 0, 2)
    return np.ascontiguousarray(t).reshape(Rp, K // 32)[:R]


def dequantize(q, sb):
    """q [R][K] bytes, block scales [R][K/32] -> float64 values."""
    R, K = q.shape
    return (e4m3_decode(q).reshape(R, K // 32, 32) * np.exp2(sb.astype(np.float64) - 127.0)[..., None]).reshape(R, K)
