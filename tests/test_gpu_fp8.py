"""GPU checks of the MXFP8 path (quantizer + fp8 GEMM engine) through the C ABI.

- quantize_mx_*: bit-exact against the numpy restatement (tests/mx.py): every fp8 value and every
  E8M0 scale byte, bf16 and fp32 inputs, ragged row counts;
- gemm_fp8_fused: against float64 numpy on the DEQUANTIZED operands the GPU quantizer produced, so
  only fp32 accumulation order / output rounding differ (products of e4m3 values are exact in
  fp32): 1e-4 max-normalised for fp32 outputs, 1e-2 for bf16 outputs (bf16 rounding 2^-9), every
  fused epilogue of the trainer.
"""
import numpy as np
import pytest

import mx
from conftest import rel_err

pytestmark = pytest.mark.gpu


def D(vit, a, dtype=np.float32):
    return vit.DeviceArray.from_numpy(np.ascontiguousarray(a, dtype=dtype))


def Z(vit, n, dtype=np.float32):
    return vit.DeviceArray.zeros(n, dtype)


def quant_gpu(v, x, src="bf16"):
    """x float32 [R][K] -> (device q, device scales, numpy q, numpy block scales [R][K/32])."""
    R, K = x.shape
    q = Z(v, R * K, np.uint8)
    sl = Z(v, int(v.lib().mx_scale_size(R, K)), np.uint8)
    if src == "bf16":
        v.call("quantize_mx_bf16_ex", q, sl, D(v, v.bf16_bits(x), np.uint16), R, K, K, K)
    else:
        v.call("quantize_mx_f32_ex", q, sl, D(v, x), R, K, K, K)
    return q, sl, q.numpy().reshape(R, K), mx.from_lane_native(sl.numpy(), R, K)


@pytest.mark.parametrize("R,K,src", [(1, 64, "f32"), (33, 128, "bf16"), (300, 192, "f32"), (257, 1280, "bf16"),
                                     (1000, 640, "f32")])
def test_quantize_mx_bit_exact(gpu, R, K, src):
    v = gpu
    rng = np.random.default_rng(R + K)
    # per-row magnitudes over many binades, exact zeros, and one all-zero block
    x = (rng.normal(size=(R, K)) * np.exp2(rng.integers(-20, 20, size=(R, 1)))).astype(np.float32)
    x[0, :32] = 0.0
    x[rng.random(size=x.shape) < 0.01] = 0.0
    if src == "bf16":
        x = v.bf16_to_f32(v.bf16_bits(x)).reshape(R, K)
    _, sl, q_gpu, sb_gpu = quant_gpu(v, x, src)
    q_ref, sb_ref = mx.quantize(x)
    assert np.array_equal(sb_gpu, sb_ref)
    # values (signed zeros compare equal); no NaN codes
    dq_gpu, dq_ref = mx.e4m3_decode(q_gpu), mx.e4m3_decode(q_ref)
    assert not np.isnan(dq_gpu).any()
    assert np.array_equal(dq_gpu, dq_ref)
    # padding rows of the scale array carry 0
    full = mx.from_lane_native(sl.numpy(), mx.rows_padded(R), K)
    assert (full[R:] == 0).all()


def _gelu64(x):
    s = np.sqrt(2.0 / np.pi)
    return 0.5 * x * (1.0 + np.tanh(s * (x + 0.044715 * x ** 3)))


def _gelu_grad64(x):
    s = np.sqrt(2.0 / np.pi)
    a = s * (x + 0.044715 * x ** 3)
    th = np.tanh(a)
    return 0.5 * (1 + th) + 0.5 * x * (1 - th * th) * s * (1 + 3 * 0.044715 * x * x)


@pytest.mark.parametrize("M,N,K", [(16384, 8448, 64), (16424, 8452, 64), (16424, 8452, 128), (5000, 1284, 64)])
def test_gemm_fp8_streaming_short_k_matches_one_tile(gpu, M, N, K):
    """The persistent fp8 engine (production variant 7) against the one-tile engine (variant 2) at the
    shortest K (one or two 64-deep steps) with more than 512 tiles (three or more tiles per workgroup)
    and ragged M / N: K = 64 must take the one-tile engine (the streaming ring fetches two steps
    ahead), K = 128 streams; the outputs are bit-identical either way."""
    v = gpu
    L = v.lib()
    rng = np.random.default_rng(M + N + K)
    a = rng.normal(size=(M, K)).astype(np.float32)
    w = (rng.normal(size=(N, K)) * 0.05).astype(np.float32)
    qa, sa, _, _ = quant_gpu(v, a, "bf16")
    qw, sw, _, _ = quant_gpu(v, w, "f32")
    bias = D(v, rng.normal(size=N).astype(np.float32))
    res = D(v, rng.normal(size=(M, N)).astype(np.float32))
    outs = {}
    try:
        for var in (2, 7):
            L.gemm_bf16_set_variant(var)
            o = []
            for epi in (0, 3, 5, 8):
                c = Z(v, M * N, np.float32 if epi in (0, 5) else np.uint16)
                c2 = Z(v, M * N, np.uint16) if epi == 8 else None
                v.call("gemm_fp8_fused", c, c2, N, res if epi == 5 else None, N if epi == 5 else 0, qa, sa, K,
                       qw, sw, K, bias if epi != 3 else None, None, M, N, K, epi)
                o.append(c.numpy())
                if c2 is not None:
                    o.append(c2.numpy())
            outs[var] = o
    finally:
        L.gemm_bf16_set_variant(0)
    for x, y in zip(outs[2], outs[7]):
        assert np.array_equal(x, y)
    assert np.abs(outs[7][0]).max() > 0


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 520, 128), (1576, 768, 192), (2056, 1280, 1280),
                                   (777, 3840, 320)])
def test_gemm_fp8_epilogues(gpu, M, N, K):
    v = gpu
    rng = np.random.default_rng(M * 3 + N + K)
    a = rng.normal(size=(M, K)).astype(np.float32)
    w = (rng.normal(size=(N, K)) * 0.05).astype(np.float32)
    qa, sa, qa_np, sba = quant_gpu(v, a, "bf16")
    qw, sw, qw_np, sbw = quant_gpu(v, w, "f32")
    ar, wr = mx.dequantize(qa_np, sba), mx.dequantize(qw_np, sbw)
    bias = rng.normal(size=N).astype(np.float32)
    acc = ar @ wr.T
    pre = acc + bias
    # 0: fp32 store + bias
    c0 = Z(v, M * N)
    v.call("gemm_fp8_fused", c0, None, N, None, 0, qa, sa, K, qw, sw, K, D(v, bias), None, M, N, K, 0)
    assert rel_err(c0.numpy().reshape(M, N), pre) < 1e-4
    # 3: bf16 store, no bias
    c1 = Z(v, M * N, np.uint16)
    v.call("gemm_fp8_fused", c1, None, N, None, 0, qa, sa, K, qw, sw, K, None, None, M, N, K, 3)
    assert rel_err(v.bf16_to_f32(c1.numpy()).reshape(M, N), acc) < 1e-2
    # 4: GELU pair
    c2, c3 = Z(v, M * N, np.uint16), Z(v, M * N, np.uint16)
    v.call("gemm_fp8_fused", c2, c3, N, None, 0, qa, sa, K, qw, sw, K, D(v, bias), None, M, N, K, 4)
    assert rel_err(v.bf16_to_f32(c2.numpy()).reshape(M, N), pre) < 1e-2
    assert rel_err(v.bf16_to_f32(c3.numpy()).reshape(M, N), _gelu64(pre)) < 1e-2
    # 5: fp32 residual
    res = rng.normal(size=(M, N)).astype(np.float32)
    c4 = Z(v, M * N)
    v.call("gemm_fp8_fused", c4, None, N, D(v, res), N, qa, sa, K, qw, sw, K, D(v, bias), None, M, N, K, 5)
    assert rel_err(c4.numpy().reshape(M, N), pre + res) < 1e-4
    # 6: DGELU x aux + fused column sums
    x = rng.normal(size=(M, N)).astype(np.float32)
    xb = v.bf16_bits(x)
    xr = v.bf16_to_f32(xb).reshape(M, N).astype(np.float64)
    c5, cs = Z(v, M * N, np.uint16), D(v, np.ones(N, np.float32))
    v.call("gemm_fp8_fused", c5, None, N, D(v, xb, np.uint16), N, qa, sa, K, qw, sw, K, None, cs, M, N, K, 6)
    want = acc * _gelu_grad64(xr)
    assert rel_err(v.bf16_to_f32(c5.numpy()).reshape(M, N), want) < 1e-2
    assert rel_err(cs.numpy(), 1.0 + want.sum(0)) < 1e-3
    # 8: gelu' / gelu pair (the trainer's fc forward); 9: product with a stored gelu' + column sums
    c6, c7 = Z(v, M * N, np.uint16), Z(v, M * N, np.uint16)
    v.call("gemm_fp8_fused", c6, c7, N, None, 0, qa, sa, K, qw, sw, K, D(v, bias), None, M, N, K, 8)
    assert rel_err(v.bf16_to_f32(c6.numpy()).reshape(M, N), _gelu_grad64(pre)) < 1e-2
    assert np.array_equal(c7.numpy(), c3.numpy())
    c8, cs2 = Z(v, M * N, np.uint16), D(v, np.ones(N, np.float32))
    v.call("gemm_fp8_fused", c8, None, N, D(v, xb, np.uint16), N, qa, sa, K, qw, sw, K, None, cs2, M, N, K, 9)
    want = acc * xr
    assert rel_err(v.bf16_to_f32(c8.numpy()).reshape(M, N), want) < 1e-2
    assert rel_err(cs2.numpy(), 1.0 + want.sum(0)) < 1e-3


def test_gemm_fp8_quantization_error_vs_bf16(gpu):
    """Model-level expectation for the fp8 mode: an MXFP8 product of N(0,1) operands against the
    exact product.  e4m3 rounds each element with a relative error uniform in +-2^-4 / mantissa
    (RMS ~2.6 %); two quantized operands give ~3.7 % RMS on the product (measured 3.75 %)."""
    v = gpu
    rng = np.random.default_rng(5)
    M, N, K = 512, 512, 1280
    a = rng.normal(size=(M, K)).astype(np.float32)
    w = rng.normal(size=(N, K)).astype(np.float32)
    qa, sa, _, _ = quant_gpu(v, a, "f32")
    qw, sw, _, _ = quant_gpu(v, w, "f32")
    c = Z(v, M * N)
    v.call("gemm_fp8_fused", c, None, N, None, 0, qa, sa, K, qw, sw, K, None, None, M, N, K, 0)
    exact = a.astype(np.float64) @ w.astype(np.float64).T
    err = np.abs(c.numpy().reshape(M, N) - exact)
    assert err.max() / np.abs(exact).max() < 1e-1
    assert np.sqrt((err ** 2).mean() / (exact ** 2).mean()) < 4.5e-2


@pytest.mark.parametrize("M,N,K", [(300, 512, 128), (1576, 3072, 192), (777, 3840, 320)])
def test_gemm_fp8_fused_mx_output(gpu, M, N, K):
    """The MX copy a GELU / GELU' epilogue writes next to its bf16 output (the trainer's fp8 mode
    feeds it to the next GEMM instead of re-quantizing) is byte-identical to quantize_mx_bf16_ex of
    that bf16 output: every e4m3 byte and the whole lane-native scale array (padding rows 0)."""
    v = gpu
    rng = np.random.default_rng(M + N + K)
    a = rng.normal(size=(M, K)).astype(np.float32)
    w = (rng.normal(size=(N, K)) * 0.05).astype(np.float32)
    qa, sa, _, _ = quant_gpu(v, a, "bf16")
    qw, sw, _, _ = quant_gpu(v, w, "f32")
    bias = D(v, rng.normal(size=N).astype(np.float32))
    nsc = int(v.lib().mx_scale_size(M, N))
    xb = D(v, v.bf16_bits(rng.normal(size=(M, N)).astype(np.float32)), np.uint16)
    for epi in (4, 6, 8, 9):
        c, c2 = Z(v, M * N, np.uint16), Z(v, M * N, np.uint16)
        fq, fs = Z(v, M * N, np.uint8), Z(v, nsc, np.uint8)
        if epi in (4, 8):
            v.call("gemm_fp8_fused_mx", c, c2, N, None, 0, qa, sa, K, qw, sw, K, bias, None, M, N, K, epi, fq, fs)
            out = c2
        else:
            v.call("gemm_fp8_fused_mx", c, None, N, xb, N, qa, sa, K, qw, sw, K, None, None, M, N, K, epi, fq, fs)
            out = c
        rq, rs = Z(v, M * N, np.uint8), Z(v, nsc, np.uint8)
        v.call("quantize_mx_bf16_ex", rq, rs, out, M, N, N, N)
        assert np.array_equal(fs.numpy(), rs.numpy()), f"epi {epi}: scale bytes differ"
        assert np.array_equal(fq.numpy(), rq.numpy()), f"epi {epi}: e4m3 bytes differ"
        # the bf16 outputs are unchanged by the extra output
        c0, c02 = Z(v, M * N, np.uint16), Z(v, M * N, np.uint16)
        if epi in (4, 8):
            v.call("gemm_fp8_fused", c0, c02, N, None, 0, qa, sa, K, qw, sw, K, bias, None, M, N, K, epi)
            assert np.array_equal(c02.numpy(), c2.numpy())
        else:
            v.call("gemm_fp8_fused", c0, None, N, xb, N, qa, sa, K, qw, sw, K, None, None, M, N, K, epi)
        assert np.array_equal(c0.numpy(), c.numpy())


@pytest.mark.parametrize("M,N,K", [(320, 512, 128), (1088, 3072, 192), (256, 1280, 320)])
def test_gemm_fp8_fused_mx_cols_output(gpu, M, N, K):
    """The column-wise MX copy the GELU-pair (fc fwd) and product (fcproj dgrad) epilogues write
    for the weight gradient, at a token offset inside a longer token axis, is byte-identical to
    quantize_mx_cols_bf16_ex of the bf16 output (M % 128 == 64 exercises the edge-tile path);
    bytes outside its token range are untouched; and omitting the MX-copied bf16 output (the
    trainer's fp8 mode) leaves every other output unchanged."""
    v = gpu
    rng = np.random.default_rng(M + 3 * N + K)
    a = rng.normal(size=(M, K)).astype(np.float32)
    w = (rng.normal(size=(N, K)) * 0.05).astype(np.float32)
    qa, sa, _, _ = quant_gpu(v, a, "bf16")
    qw, sw, _, _ = quant_gpu(v, w, "f32")
    bias = D(v, rng.normal(size=N).astype(np.float32))
    xb = D(v, v.bf16_bits(rng.normal(size=(M, N)).astype(np.float32)), np.uint16)
    off, ld = 128, 128 + M + 64
    nsr, nsc = int(v.lib().mx_scale_size(M, N)), int(v.lib().mx_scale_size(N, ld))

    def run(epi, keep):
        c, c2 = Z(v, M * N, np.uint16), Z(v, M * N, np.uint16)
        fq, fs = Z(v, M * N, np.uint8), Z(v, nsr, np.uint8)
        cq = D(v, np.full(N * ld, 0x5A, np.uint8), np.uint8)
        cs = D(v, np.full(nsc, 0x5A, np.uint8), np.uint8)
        if epi == 8:
            v.call("gemm_fp8_fused_mxc", c, c2 if keep else None, N, None, 0, qa, sa, K, qw, sw, K, bias, None,
                   M, N, K, epi, fq, fs, cq, cs, ld, off)
        else:
            v.call("gemm_fp8_fused_mxc", c if keep else None, None, N, xb, N, qa, sa, K, qw, sw, K, None, None,
                   M, N, K, epi, fq, fs, cq, cs, ld, off)
        return c, c2, fq, fs, cq, cs

    for epi in (8, 9):
        c, c2, fq, fs, cq, cs = run(epi, True)
        out = c2 if epi == 8 else c
        rq, rs = Z(v, N * M, np.uint8), Z(v, int(v.lib().mx_scale_size(N, M)), np.uint8)
        v.call("quantize_mx_cols_bf16_ex", rq, rs, out, M, N, N)
        got = cq.numpy().reshape(N, ld)
        assert np.array_equal(got[:, off:off + M], rq.numpy().reshape(N, M)), f"epi {epi}: e4m3 bytes differ"
        assert (got[:, :off] == 0x5A).all() and (got[:, off + M:] == 0x5A).all()
        blk = mx.from_lane_native(cs.numpy(), N, ld)
        assert np.array_equal(blk[:, off // 32:(off + M) // 32], mx.from_lane_native(rs.numpy(), N, M)), \
            f"epi {epi}: scale bytes differ"
        c_, c2_, fq_, fs_, cq_, cs_ = run(epi, False)
        for x, y in ((fq, fq_), (fs, fs_), (cq, cq_), (cs, cs_)):
            assert np.array_equal(x.numpy(), y.numpy())
        if epi == 8:  # the GELU' output is still stored; the GELU output was not
            assert np.array_equal(c.numpy(), c_.numpy())
            assert not c2_.numpy().any()


@pytest.mark.parametrize("R,C", [(1, 64), (100, 128), (197, 768), (4001, 320), (50432 // 8, 1280)])
def test_quantize_mx_cols_bit_exact(gpu, R, C):
    """Column-wise MX (the fp8 weight gradients' operands: blocks of 32 consecutive tokens) equals
    the row quantizer's restatement applied to the zero-padded transpose, byte for byte, including
    the padding tokens (zero bytes) and the padding rows' zero scales."""
    v = gpu
    rng = np.random.default_rng(R * 7 + C)
    x = (rng.normal(size=(R, C)) * np.exp2(rng.integers(-12, 12, size=(1, C)))).astype(np.float32)
    x[rng.random(size=x.shape) < 0.01] = 0.0
    xb = v.bf16_bits(x)
    xr = v.bf16_to_f32(xb).reshape(R, C)
    kp = int(v.lib().mx_cols_padded(R))
    assert kp == (R + 63) // 64 * 64
    nsc = int(v.lib().mx_scale_size(C, kp))
    q = D(v, np.full(C * kp, 0x5A, np.uint8), np.uint8)   # poison: every byte must be written
    sl = D(v, np.full(nsc, 0x5A, np.uint8), np.uint8)
    v.call("quantize_mx_cols_bf16_ex", q, sl, D(v, xb, np.uint16), R, C, C)
    t = np.zeros((C, kp), np.float32)
    t[:, :R] = xr.T
    q_ref, sb_ref = mx.quantize(t)
    assert np.array_equal(sl.numpy(), mx.to_lane_native(sb_ref))
    assert np.array_equal(q.numpy().reshape(C, kp), q_ref)


@pytest.mark.parametrize("R,C,parts", [(100, 128, 1), (197, 768, 1), (4001, 320, 1), (2 * 257 * 16, 1280, 2),
                                        (3 * 1024 + 70, 192, 3), (1000, 2304, 2), (300, 3840, 1)])
def test_quantize_mx_rowcol_bit_exact(gpu, R, C, parts):
    """The fused row+column quantizer (the fp8 trainer's ln1 / atty / ln2 / dres / dqkv) equals the
    two separate quantizers byte for byte: the row form of each micro-batch slice against
    quantize_mx_bf16_ex, the column form assembled from `parts` slices (token offsets multiples of
    64, the last one carrying the padding tokens) against one quantize_mx_cols_bf16_ex over all R."""
    v = gpu
    rng = np.random.default_rng(R + C + parts)
    x = (rng.normal(size=(R, C)) * np.exp2(rng.integers(-12, 12, size=(1, C)))).astype(np.float32)
    x[rng.random(size=x.shape) < 0.01] = 0.0
    xb = v.bf16_bits(x)
    xd = D(v, xb, np.uint16)
    kp = int(v.lib().mx_cols_padded(R))
    nsc = int(v.lib().mx_scale_size(C, kp))
    qc_ref, sc_ref = Z(v, C * kp, np.uint8), Z(v, nsc, np.uint8)
    v.call("quantize_mx_cols_bf16_ex", qc_ref, sc_ref, xd, R, C, C)
    qc = D(v, np.full(C * kp, 0x5A, np.uint8), np.uint8)
    sc = D(v, np.full(nsc, 0x5A, np.uint8), np.uint8)
    step = ((R + parts - 1) // parts + 63) // 64 * 64 if parts > 1 else R
    bounds = [min(i * step, R) for i in range(parts)] + [R]
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        n = hi - lo
        if n <= 0:
            continue
        ntok = kp - lo if hi == R else n
        nsr = int(v.lib().mx_scale_size(n, C))
        qr = D(v, np.full(n * C, 0x5A, np.uint8), np.uint8)
        sr = D(v, np.full(nsr, 0x5A, np.uint8), np.uint8)
        xs = D(v, xb.reshape(R, C)[lo:hi].copy(), np.uint16)
        v.call("quantize_mx_rowcol_bf16_ex", qr, sr, qc, sc, xs, n, C, C, kp, lo, ntok)
        qr_ref, sr_ref = Z(v, n * C, np.uint8), Z(v, nsr, np.uint8)
        v.call("quantize_mx_bf16_ex", qr_ref, sr_ref, xs, n, C, C, C)
        assert np.array_equal(sr.numpy(), sr_ref.numpy()), f"row scales differ at slice {lo}"
        assert np.array_equal(qr.numpy(), qr_ref.numpy()), f"row bytes differ at slice {lo}"
    assert np.array_equal(sc.numpy(), sc_ref.numpy()), "column scales differ"
    assert np.array_equal(qc.numpy(), qc_ref.numpy()), "column bytes differ"


@pytest.mark.parametrize("R,C,parts", [(100, 256, 1), (197, 768, 1), (2 * 257 * 16, 1280, 2), (1000, 1024, 2),
                                        (3 * 1024 + 70, 512, 3), (300, 2048, 1), (4001, 1536, 1), (64 * 257, 1280, 1),
                                        (128 * 257, 768, 2)])
def test_layernorm_forward_mx_bit_exact(gpu, R, C, parts):
    """LayerNorm straight into the MX forms (the fp8 trainer's ln1 / ln2) equals the unfused pair it
    replaces byte for byte: layernorm_forward_bf16 (its mean / rstd bit for bit too) and then
    quantize_mx_rowcol_bf16_ex of the bf16 output, per micro-batch slice (row form, row scales incl.
    the padding rows' zero scales), the column form assembled from `parts` slices (padding tokens
    of the last) against the same assembled by the unfused pair.  Inputs: rows of widely varying
    scale and offset, some constant rows (rstd = 1/sqrt(eps)), weights with zeros (zero blocks:
    scale byte 127).  16 448 rows (520 tiles: more than the 512 slots) and 32 896 in two slices take
    the leftover-row path (the last partial round's rows one per wave, their column form from a
    follow-up quantize of their bf16 rows)."""
    v = gpu
    rng = np.random.default_rng(R + C + 5 * parts)
    x = (rng.normal(size=(R, C)) * np.exp2(rng.integers(-6, 6, size=(R, 1))) + rng.normal(size=(R, 1)) * 3).astype(np.float32)
    x[rng.integers(0, R, size=3)] = 1.5
    w = rng.normal(size=C).astype(np.float32)
    w[rng.integers(0, C, size=C // 16)] = 0.0
    w[:32] = 0.0
    b = (rng.normal(size=C) * 0.1).astype(np.float32)
    b[:32] = 0.0
    kp = int(v.lib().mx_cols_padded(R))
    nsc = int(v.lib().mx_scale_size(C, kp))
    qc_ref, sc_ref = Z(v, C * kp, np.uint8), Z(v, nsc, np.uint8)
    qc = D(v, np.full(C * kp, 0x5A, np.uint8), np.uint8)
    sc = D(v, np.full(nsc, 0x5A, np.uint8), np.uint8)
    wd, bd = D(v, w), D(v, b)
    step = ((R + parts - 1) // parts + 63) // 64 * 64 if parts > 1 else R
    bounds = [min(i * step, R) for i in range(parts)] + [R]
    v.kernel_hits_reset()
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        n = hi - lo
        if n <= 0:
            continue
        ntok = kp - lo if hi == R else n
        nsr = int(v.lib().mx_scale_size(n, C))
        xs = D(v, x[lo:hi].copy())
        ln_bf, mu_ref, rs_ref = Z(v, n * C, np.uint16), Z(v, n), Z(v, n)
        v.call("layernorm_forward_bf16", ln_bf, mu_ref, rs_ref, xs, wd, bd, 1, n, C)
        qr_ref, sr_ref = Z(v, n * C, np.uint8), Z(v, nsr, np.uint8)
        v.call("quantize_mx_rowcol_bf16_ex", qr_ref, sr_ref, qc_ref, sc_ref, ln_bf, n, C, C, kp, lo, ntok)
        qr = D(v, np.full(n * C, 0x5A, np.uint8), np.uint8)
        sr = D(v, np.full(nsr, 0x5A, np.uint8), np.uint8)
        mu = D(v, np.full(n, np.nan, np.float32))
        rs = D(v, np.full(n, np.nan, np.float32))
        v.call("layernorm_forward_mx", qr, sr, qc, sc, mu, rs, xs, wd, bd, n, C, kp, lo, ntok)
        assert np.array_equal(mu.numpy(), mu_ref.numpy()) and np.array_equal(rs.numpy(), rs_ref.numpy()), lo
        assert np.array_equal(sr.numpy(), sr_ref.numpy()), f"row scales differ at slice {lo}"
        assert np.array_equal(qr.numpy(), qr_ref.numpy()), f"row bytes differ at slice {lo}"
    assert np.array_equal(sc.numpy(), sc_ref.numpy()), "column scales differ"
    assert np.array_equal(qc.numpy(), qc_ref.numpy()), "column bytes differ"
    assert v.kernel_hits()[v.HIT_LN_MX] == sum(1 for lo, hi in zip(bounds[:-1], bounds[1:]) if hi > lo)


@pytest.mark.parametrize("R,C,parts,dsum", [(100, 256, 1, True), (197, 768, 1, False), (2 * 257 * 16, 1280, 2, True),
                                             (1000, 1024, 2, True), (3 * 1024 + 70, 512, 3, True), (4001, 1280, 1, False),
                                             (64 * 257, 1280, 1, True), (128 * 257, 768, 2, True)])
def test_layernorm_backward_mx_bit_exact(gpu, R, C, parts, dsum):
    """The residual-gradient LayerNorm backward with both MX forms of its bf16 plane (the fp8 trainer's
    dres2 / dres3) against the unfused pair it replaces: layernorm_backward_stream (the trainer's
    ln_bwd_vec_k) then quantize_mx_rowcol_bf16_ex of its bf16 output.  The bf16 and lo8 planes, the
    row form (with the padding rows' zero scales) and the column form assembled over `parts`
    micro-batch slices are equal byte for byte; dW / db / dres column sums group their rows
    differently (fixed order), so they agree to fp32 rounding (1e-5 of the column's magnitude).  The
    ViT-H/14 micro-batch (16 448 rows: 520 tiles, more than one round on 256 CUs) and 32 896 rows in two
    slices take the leftover-row path (the last partial round's rows spread over all workgroups, their
    column form from the follow-up quantize)."""
    v = gpu
    rng = np.random.default_rng(R + 3 * C + parts)
    x = (rng.normal(size=(R, C)) * 2 + rng.normal(size=(R, 1))).astype(np.float32)
    mu = x.mean(1).astype(np.float32)
    rs = (1.0 / np.sqrt(x.var(1) + 1e-5)).astype(np.float32)
    w = rng.normal(size=C).astype(np.float32)
    dyb = v.bf16_bits((rng.normal(size=(R, C)) * np.exp2(rng.integers(-6, 6, size=(R, 1)))).astype(np.float32))
    hib = v.bf16_bits(rng.normal(size=(R, C)).astype(np.float32))
    lo = rng.integers(0, 256, size=(R, C), dtype=np.uint8)
    kp = int(v.lib().mx_cols_padded(R))
    nsc = int(v.lib().mx_scale_size(C, kp))
    qc_ref, sc_ref = Z(v, C * kp, np.uint8), Z(v, nsc, np.uint8)
    qc = D(v, np.full(C * kp, 0x5A, np.uint8), np.uint8)
    sc = D(v, np.full(nsc, 0x5A, np.uint8), np.uint8)
    sums_ref = [Z(v, C), Z(v, C), Z(v, C)]
    sums = [Z(v, C), Z(v, C), Z(v, C)]
    step = ((R + parts - 1) // parts + 63) // 64 * 64 if parts > 1 else R
    bounds = [min(i * step, R) for i in range(parts)] + [R]
    wd = D(v, w)
    v.kernel_hits_reset()
    nlaunch = 0
    for lo_, hi_ in zip(bounds[:-1], bounds[1:]):
        n = hi_ - lo_
        if n <= 0:
            continue
        nlaunch += 1
        ntok = kp - lo_ if hi_ == R else n
        args = (D(v, hib[lo_:hi_].copy(), np.uint16), D(v, lo[lo_:hi_].copy(), np.uint8))
        com = (D(v, dyb[lo_:hi_].copy(), np.uint16), D(v, x[lo_:hi_].copy()), wd, D(v, mu[lo_:hi_].copy()),
               D(v, rs[lo_:hi_].copy()), n, C)
        ho_ref, lo_ref = Z(v, n * C, np.uint16), Z(v, n * C, np.uint8)
        v.call("layernorm_backward_stream", ho_ref, lo_ref, *args, sums_ref[0], sums_ref[1],
               sums_ref[2] if dsum else None, *com)
        nsr = int(v.lib().mx_scale_size(n, C))
        qr_ref, sr_ref = Z(v, n * C, np.uint8), Z(v, nsr, np.uint8)
        v.call("quantize_mx_rowcol_bf16_ex", qr_ref, sr_ref, qc_ref, sc_ref, ho_ref, n, C, C, kp, lo_, ntok)
        ho, lo8 = D(v, np.full(n * C, 0x5A5A, np.uint16), np.uint16), D(v, np.full(n * C, 0x5A, np.uint8), np.uint8)
        qr = D(v, np.full(n * C, 0x5A, np.uint8), np.uint8)
        sr = D(v, np.full(nsr, 0x5A, np.uint8), np.uint8)
        v.call("layernorm_backward_stream_mx", ho, lo8, *args, sums[0], sums[1], sums[2] if dsum else None, *com,
               qr, sr, qc, sc, kp, lo_, ntok)
        assert np.array_equal(ho.numpy(), ho_ref.numpy()), f"bf16 plane differs at slice {lo_}"
        assert np.array_equal(lo8.numpy(), lo_ref.numpy()), f"lo8 plane differs at slice {lo_}"
        assert np.array_equal(sr.numpy(), sr_ref.numpy()), f"row scales differ at slice {lo_}"
        assert np.array_equal(qr.numpy(), qr_ref.numpy()), f"row bytes differ at slice {lo_}"
    assert np.array_equal(sc.numpy(), sc_ref.numpy()), "column scales differ"
    assert np.array_equal(qc.numpy(), qc_ref.numpy()), "column bytes differ"
    for k in range(3 if dsum else 2):
        a, b = sums[k].numpy(), sums_ref[k].numpy()
        assert np.max(np.abs(a - b)) <= 1e-5 * max(np.max(np.abs(b)), 1e-30), k
    assert v.kernel_hits()[v.HIT_LNB_MX] == nlaunch


@pytest.mark.parametrize("OC,Cin,R", [(256, 256, 64), (768, 320, 1000), (1280, 5120, 4112), (512, 768, 6000)])
def test_gemm_fp8_wgrad_splitk(gpu, OC, Cin, R):
    """The fp8 weight gradient dW += dout^T . inp (epi 2) on column-quantized operands: one split
    accumulating in place (the small shapes) or K-split fp32 slabs + the fixed-order reduce (2 and 5
    splits) equal float64 numpy on the dequantized operands to 1e-4, and two launches give
    bit-identical results (no atomics)."""
    v = gpu
    rng = np.random.default_rng(OC + Cin + R)
    dout = rng.normal(size=(R, OC)).astype(np.float32)
    inp = rng.normal(size=(R, Cin)).astype(np.float32)
    kp = int(v.lib().mx_cols_padded(R))

    def colq(x):
        C = x.shape[1]
        q = Z(v, C * kp, np.uint8)
        sl = Z(v, int(v.lib().mx_scale_size(C, kp)), np.uint8)
        v.call("quantize_mx_cols_bf16_ex", q, sl, D(v, v.bf16_bits(x), np.uint16), R, C, C)
        return q, sl, mx.dequantize(q.numpy().reshape(C, kp), mx.from_lane_native(sl.numpy(), C, kp))

    qa, sa, ar = colq(dout)
    qb, sb, br = colq(inp)
    dw0 = rng.normal(size=(OC, Cin)).astype(np.float32)
    want = dw0 + ar @ br.T
    outs = []
    for _ in range(2):
        dw = D(v, dw0)
        v.call("gemm_fp8_fused", dw, None, Cin, None, 0, qa, sa, kp, qb, sb, kp, None, None, OC, Cin, kp, 2)
        outs.append(dw.numpy())
    assert rel_err(outs[0].reshape(OC, Cin), want) < 1e-4
    assert np.array_equal(outs[0], outs[1])
