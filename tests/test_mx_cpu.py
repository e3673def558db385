"""CPU checks of the numpy MX quantizer (tests/mx.py) that pins the fp8 path's numerics."""
import numpy as np

import mx


def test_e4m3_codec_roundtrip():
    codes = np.arange(256, dtype=np.uint8)
    vals = mx.e4m3_decode(codes)
    ok = ~np.isnan(vals)
    assert ok.sum() == 254
    back = mx.e4m3_encode(vals[ok])
    # +0 / -0 both decode to 0; every other code round-trips
    assert np.array_equal(back[vals[ok] != 0], codes[ok][vals[ok] != 0])
    assert np.array_equal(mx.e4m3_round(vals[ok]), vals[ok])
    assert mx.e4m3_decode(np.uint8(0x7E)) == 448.0


def test_rne_ties_and_scale_rule():
    assert mx.e4m3_round(np.array([1.0625]))[0] == 1.0       # tie -> even mantissa
    assert mx.e4m3_round(np.array([1.1875]))[0] == 1.25
    assert mx.scale_bytes(np.array([448.0], np.float32))[0] == 127
    assert mx.scale_bytes(np.array([449.0], np.float32))[0] == 128
    assert mx.scale_bytes(np.array([1.0], np.float32))[0] == 119
    assert mx.scale_bytes(np.array([0.0], np.float32))[0] == 127


def test_quantize_bounds_and_layout():
    rng = np.random.default_rng(0)
    x = (rng.normal(size=(300, 192)) * np.exp(rng.normal(size=(300, 1)) * 3)).astype(np.float32)
    q, sb = mx.quantize(x)
    dq = mx.dequantize(q, sb)
    blocks = np.abs(x.reshape(300, 6, 32)).max(-1)
    # every block's scaled maximum lies in (224, 448]: no overflow, at most one binade of headroom
    smax = blocks / np.exp2(sb.astype(np.float64) - 127)
    assert (smax <= 448).all() and (smax > 224).all()
    # relative error of e4m3 with RNE: <= 2^-4 for normal values
    big = np.abs(x) > np.repeat(blocks, 32, axis=1) * 2.0 ** -6
    assert (np.abs(dq - x)[big] <= np.abs(x)[big] * 2.0 ** -4 + 1e-30).all()
    sl = mx.to_lane_native(sb)
    assert sl.size == mx.rows_padded(300) * 192 // 32
    assert np.array_equal(mx.from_lane_native(sl, 300, 192), sb)
