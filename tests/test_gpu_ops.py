"""GPU parity of every C-ABI op against the CPU oracle (same seeded inputs), through the C ABI.

fp32 ops: <= 1e-4 relative to the oracle's fp32 result (max-normalised), the parity bar of
BASELINE.json.  bf16 ops: compared with the fp64 oracle run on the bf16-ROUNDED inputs, so only
accumulation order / output rounding differ; tolerance 1e-2 (bf16 output rounding is 2^-9).
"""
import os

import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu


def D(vit, a, dtype=np.float32):
    return vit.DeviceArray.from_numpy(np.ascontiguousarray(a, dtype=dtype))


def Z(vit, n, dtype=np.float32):
    return vit.DeviceArray.zeros(n, dtype)


# ------------------------------------------------------------------ fp32 reference ops
def test_kats_on_gpu(gpu):
    v = gpu
    out = Z(v, 10)
    v.call("residual_forward", out, D(v, np.ones(10)), D(v, np.full(10, 2.0)), 10)
    assert np.array_equal(out.numpy(), np.full(10, 3.0, np.float32))
    B, T, C, OC = 2, 3, 4, 5
    out = Z(v, B * T * OC)
    v.call("matmul_forward", out, D(v, np.ones(B * T * C)), D(v, np.full(OC * C, 2.0)),
           D(v, np.full(OC, 3.0)), B, T, C, OC)
    assert np.array_equal(out.numpy(), np.full(B * T * OC, 11.0, np.float32))
    B, T, C, NH = 2, 3, 4, 2
    out, pre, att = Z(v, B * T * C), Z(v, B * T * NH * T), Z(v, B * T * NH * T)
    v.call("attention_forward", out, pre, att, D(v, np.ones(B * T * 3 * C)), B, T, C, NH)
    assert np.allclose(out.numpy(), 1.0, atol=1e-6)
    out, m, r = Z(v, 24), Z(v, 6), Z(v, 6)
    v.call("layernorm_forward", out, m, r, D(v, np.ones(24)), D(v, np.full(4, 2.0)), D(v, np.full(4, 3.0)), 2, 3, 4)
    assert np.allclose(out.numpy(), 3.0) and np.allclose(m.numpy(), 1.0)
    assert np.allclose(r.numpy(), 1 / np.sqrt(np.float32(1e-5)), rtol=1e-5)
    g = Z(v, 10)
    v.call("gelu_forward", g, D(v, np.ones(10)), 10)
    assert np.allclose(g.numpy(), 0.841192, atol=2e-6)
    p = Z(v, 24)
    v.call("softmax_forward", p, D(v, np.ones(24)), 2, 3, 4)
    assert np.allclose(p.numpy(), 0.25)


@pytest.mark.parametrize("B,T,C,OC", [(2, 3, 4, 5), (3, 17, 32, 96), (2, 197, 192, 576), (1, 50, 100, 37)])
def test_matmul_fp32(gpu, oracle32, B, T, C, OC):
    v, o = gpu, oracle32
    rng = np.random.default_rng(B * 1000 + T)
    inp, w, b = o.arr(rng.normal(size=B * T * C)), o.arr(rng.normal(size=OC * C) * 0.1), o.arr(rng.normal(size=OC))
    dout = o.arr(rng.normal(size=B * T * OC))
    ref = o.arr(np.zeros(B * T * OC))
    o.call("matmul_forward", ref, inp, w, b, B, T, C, OC)
    out = Z(v, B * T * OC)
    v.call("matmul_forward", out, D(v, inp), D(v, w), D(v, b), B, T, C, OC)
    assert rel_err(out.numpy(), ref) < 1e-5
    # backward accumulates (+=) into pre-filled buffers
    pre_i, pre_w, pre_b = rng.normal(size=B * T * C), rng.normal(size=OC * C), rng.normal(size=OC)
    ri, rw, rb = o.arr(pre_i), o.arr(pre_w), o.arr(pre_b)
    o.call("matmul_backward", ri, rw, rb, dout, inp, w, B, T, C, OC)
    gi, gw, gb = D(v, pre_i), D(v, pre_w), D(v, pre_b)
    v.call("matmul_backward", gi, gw, gb, D(v, dout), D(v, inp), D(v, w), B, T, C, OC)
    assert rel_err(gi.numpy(), ri) < 1e-5
    assert rel_err(gw.numpy(), rw) < 1e-5
    assert rel_err(gb.numpy(), rb) < 1e-5


def test_matmul_fp32_null_bias_and_dinp(gpu, oracle32):
    v, o = gpu, oracle32
    rng = np.random.default_rng(9)
    B, T, C, OC = 2, 5, 8, 6
    inp, w = o.arr(rng.normal(size=B * T * C)), o.arr(rng.normal(size=OC * C))
    ref = o.arr(np.zeros(B * T * OC))
    o.call("matmul_forward", ref, inp, w, None, B, T, C, OC)
    out = Z(v, B * T * OC)
    v.call("matmul_forward", out, D(v, inp), D(v, w), None, B, T, C, OC)
    assert rel_err(out.numpy(), ref) < 1e-6
    dout = o.arr(rng.normal(size=B * T * OC))
    rw = o.arr(np.zeros(OC * C))
    o.call("matmul_backward", None, rw, None, dout, inp, w, B, T, C, OC)
    gw = Z(v, OC * C)
    v.call("matmul_backward", None, gw, None, D(v, dout), D(v, inp), D(v, w), B, T, C, OC)
    assert rel_err(gw.numpy(), rw) < 1e-6


@pytest.mark.parametrize("B,T,C,NH", [(2, 3, 4, 2), (2, 17, 32, 2), (2, 197, 192, 3), (1, 1, 64, 1), (1, 300, 64, 4)])
def test_attention_fp32(gpu, oracle32, B, T, C, NH):
    v, o = gpu, oracle32
    rng = np.random.default_rng(T)
    inp = o.arr(rng.normal(size=B * T * 3 * C))
    n = B * T * NH * T
    out, pre, att = o.arr(np.zeros(B * T * C)), o.arr(np.zeros(n)), o.arr(np.zeros(n))
    o.call("attention_forward", out, pre, att, inp, B, T, C, NH)
    gout, gpre, gatt = Z(v, B * T * C), Z(v, n), Z(v, n)
    gi = D(v, inp)
    v.call("attention_forward", gout, gpre, gatt, gi, B, T, C, NH)
    assert rel_err(gout.numpy(), out) < 1e-5
    assert rel_err(gpre.numpy(), pre) < 1e-5
    assert rel_err(gatt.numpy(), att) < 1e-5
    dout = o.arr(rng.normal(size=B * T * C))
    pre_d = rng.normal(size=B * T * 3 * C)
    dinp, dpre, datt = o.arr(pre_d), o.arr(np.zeros(n)), o.arr(np.zeros(n))
    o.call("attention_backward", dinp, dpre, datt, dout, inp, att, B, T, C, NH)
    gd, gdp, gda = D(v, pre_d), Z(v, n), Z(v, n)
    v.call("attention_backward", gd, gdp, gda, D(v, dout), gi, gatt, B, T, C, NH)
    assert rel_err(gd.numpy(), dinp) < 1e-4
    assert rel_err(gdp.numpy(), dpre) < 1e-4
    assert rel_err(gda.numpy(), datt) < 1e-5
    # NULL scratch (internal workspace) gives the same input gradient
    gd2 = D(v, pre_d)
    v.call("attention_backward", gd2, None, None, D(v, dout), gi, gatt, B, T, C, NH)
    assert rel_err(gd2.numpy(), dinp) < 1e-4


@pytest.mark.parametrize("rows,C", [(6, 4), (394, 192), (100, 768), (7, 1000)])
def test_layernorm_fp32(gpu, oracle32, rows, C):
    v, o = gpu, oracle32
    rng = np.random.default_rng(C)
    x, w, b = o.arr(rng.normal(size=rows * C) * 3 + 1), o.arr(rng.normal(size=C)), o.arr(rng.normal(size=C))
    out, m, r = o.arr(np.zeros(rows * C)), o.arr(np.zeros(rows)), o.arr(np.zeros(rows))
    o.call("layernorm_forward", out, m, r, x, w, b, rows, 1, C)
    go, gm, gr = Z(v, rows * C), Z(v, rows), Z(v, rows)
    v.call("layernorm_forward", go, gm, gr, D(v, x), D(v, w), D(v, b), rows, 1, C)
    assert rel_err(go.numpy(), out) < 1e-5 and rel_err(gm.numpy(), m) < 1e-5 and rel_err(gr.numpy(), r) < 1e-5
    dy = o.arr(rng.normal(size=rows * C))
    p0 = rng.normal(size=rows * C)
    di, dw, db = o.arr(p0), o.arr(np.ones(C)), o.arr(np.zeros(C))
    o.call("layernorm_backward", di, dw, db, dy, x, w, m, r, rows, 1, C)
    gdi, gdw, gdb = D(v, p0), D(v, np.ones(C)), Z(v, C)
    v.call("layernorm_backward", gdi, gdw, gdb, D(v, dy), D(v, x), D(v, w), gm, gr, rows, 1, C)
    assert rel_err(gdi.numpy(), di) < 1e-4 and rel_err(gdw.numpy(), dw) < 1e-5 and rel_err(gdb.numpy(), db) < 1e-5


def test_elementwise_fp32(gpu, oracle32):
    v, o = gpu, oracle32
    rng = np.random.default_rng(11)
    n = 100003
    x, y, g = o.arr(rng.normal(size=n) * 3), o.arr(rng.normal(size=n)), o.arr(rng.normal(size=n))
    ref = o.arr(np.zeros(n))
    o.call("gelu_forward", ref, x, n)
    out = Z(v, n)
    v.call("gelu_forward", out, D(v, x), n)
    assert rel_err(out.numpy(), ref) < 1e-6
    p0 = rng.normal(size=n)
    ref = o.arr(p0)
    o.call("gelu_backward", ref, x, g, n)
    out = D(v, p0)
    v.call("gelu_backward", out, D(v, x), D(v, g), n)
    assert rel_err(out.numpy(), ref) < 1e-5
    a1, a2 = o.arr(p0), o.arr(-p0)
    o.call("residual_backward", a1, a2, g, n)
    b1, b2 = D(v, p0), D(v, -p0)
    v.call("residual_backward", b1, b2, D(v, g), n)
    assert np.array_equal(b1.numpy(), a1) and np.array_equal(b2.numpy(), a2)
    ref = o.arr(np.zeros(n))
    o.call("residual_forward", ref, x, y, n)
    out = Z(v, n)
    v.call("residual_forward", out, D(v, x), D(v, y), n)
    assert np.array_equal(out.numpy(), ref)
    pp = o.arr(p0)
    o.sgd_step(pp, g, 0.01)
    gp = D(v, p0)
    v.call("sgd_step", gp, D(v, g), n, 0.01)
    assert np.array_equal(gp.numpy(), pp)


@pytest.mark.parametrize("rows,V", [(5, 10), (256, 1000), (3, 4)])
def test_softmax_ce_fp32(gpu, oracle32, rows, V):
    v, o = gpu, oracle32
    rng = np.random.default_rng(V)
    logits = o.arr(rng.normal(size=rows * V) * 4)
    tgt = rng.integers(0, V, size=rows).astype(np.int32)
    probs, losses = o.arr(np.zeros(rows * V)), o.arr(np.zeros(rows))
    o.call("softmax_forward", probs, logits, rows, 1, V)
    o.call("crossentropy_forward", losses, probs, tgt, rows, 1, V)
    gp, gl = Z(v, rows * V), Z(v, rows)
    gt = D(v, tgt, np.int32)
    v.call("softmax_forward", gp, D(v, logits), rows, 1, V)
    v.call("crossentropy_forward", gl, gp, gt, rows, 1, V)
    assert rel_err(gp.numpy(), probs) < 1e-5 and rel_err(gl.numpy(), losses) < 1e-5
    dl = o.arr(np.full(rows, 1.0 / rows))
    p0 = rng.normal(size=rows * V)
    ref = o.arr(p0)
    o.call("crossentropy_softmax_backward", ref, dl, probs, tgt, rows, 1, V)
    out = D(v, p0)
    v.call("crossentropy_softmax_backward", out, D(v, dl), gp, gt, rows, 1, V)
    assert rel_err(out.numpy(), ref) < 1e-6


@pytest.mark.parametrize("B,IMG,P,C", [(2, 32, 8, 32), (3, 48, 16, 64), (2, 224, 16, 192)])
def test_patch_embed_fp32(gpu, oracle32, B, IMG, P, C):
    v, o = gpu, oracle32
    rng = np.random.default_rng(IMG)
    NP, K = (IMG // P) ** 2, 3 * P * P
    T = NP + 1
    px = o.arr(rng.normal(size=B * 3 * IMG * IMG))
    w, b, cls, wpe = (o.arr(rng.normal(size=s) * 0.05) for s in (C * K, C, C, T * C))
    enc = o.arr(np.zeros(B * T * C))
    o.call("patch_embed_forward", enc, px, w, b, cls, wpe, B, IMG, P, C)
    genc = Z(v, B * T * C)
    gpx = D(v, px)
    v.call("patch_embed_forward", genc, gpx, D(v, w), D(v, b), D(v, cls), D(v, wpe), B, IMG, P, C)
    assert rel_err(genc.numpy(), enc) < 1e-5
    denc = o.arr(rng.normal(size=B * T * C))
    dw, db, dc, dp = (o.arr(np.zeros(s)) for s in (C * K, C, C, T * C))
    o.call("patch_embed_backward", dw, db, dc, dp, denc, px, B, IMG, P, C)
    gdw, gdb, gdc, gdp = (Z(v, s) for s in (C * K, C, C, T * C))
    v.call("patch_embed_backward", gdw, gdb, gdc, gdp, D(v, denc), gpx, B, IMG, P, C)
    for g, r in ((gdw, dw), (gdb, db), (gdc, dc), (gdp, dp)):
        assert rel_err(g.numpy(), r) < 1e-5


# ------------------------------------------------------------------ bf16 MFMA GEMM layouts
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (300, 200, 72), (1576, 576, 192), (50432 // 8, 768, 768), (64, 1000, 16)])
def test_matmul_bf16(gpu, oracle64, M, N, K):
    """forward (K-contig x K-contig), dgrad (K x N-contig) and split-K wgrad (M x N-contig)."""
    v = gpu
    rng = np.random.default_rng(M + N + K)
    x = rng.normal(size=(M, K)).astype(np.float32)
    w = (rng.normal(size=(N, K)) * 0.05).astype(np.float32)
    b = rng.normal(size=N).astype(np.float32)
    dy = rng.normal(size=(M, N)).astype(np.float32)
    xb, wb, dyb = v.bf16_bits(x), v.bf16_bits(w), v.bf16_bits(dy)
    xr, wr, dyr = (v.bf16_to_f32(a).astype(np.float64).reshape(s) for a, s in ((xb, (M, K)), (wb, (N, K)), (dyb, (M, N))))
    out = Z(v, M * N, np.uint16)
    v.call("matmul_forward_bf16", out, D(v, xb, np.uint16), D(v, wb, np.uint16), D(v, b), 1, M, K, N)
    ref = xr @ wr.T + b
    assert rel_err(v.bf16_to_f32(out.numpy()).reshape(M, N), ref) < 1e-2
    p_in, p_w, p_b = rng.normal(size=M * K), rng.normal(size=N * K), rng.normal(size=N)
    gi, gw, gb = D(v, p_in), D(v, p_w), D(v, p_b)
    v.call("matmul_backward_bf16", gi, gw, gb, D(v, dyb, np.uint16), D(v, xb, np.uint16), D(v, wb, np.uint16), 1, M, K, N)
    assert rel_err(gi.numpy().reshape(M, K), p_in.reshape(M, K) + dyr @ wr) < 2e-3
    assert rel_err(gw.numpy().reshape(N, K), p_w.reshape(N, K) + dyr.T @ xr) < 2e-3
    assert rel_err(gb.numpy(), p_b + dyr.sum(0)) < 2e-3


# ------------------------------------------------------------------ fused bf16 attention
@pytest.mark.parametrize("B,T,NH,HS,path", [
    (2, 197, 3, 64, "mfma"), (1, 1, 1, 64, "mfma"), (2, 17, 2, 64, "mfma"), (1, 64, 2, 64, "mfma"),
    (1, 256, 1, 64, "mfma"), (3, 33, 4, 64, "mfma"), (1, 300, 1, 64, "mfma"),
    # the other head sizes on the MFMA kernels: ViT-H/14 (hs 80, T 257), hs 32 / 96 / 128
    (2, 257, 2, 80, "mfma"), (1, 1, 1, 80, "mfma"), (2, 50, 3, 32, "mfma"), (1, 70, 2, 96, "mfma"),
    (1, 70, 1, 128, "mfma"), (1, 288, 1, 128, "mfma"),
    # past the LDS range (T > 320): the generic VALU kernels
    (1, 330, 1, 64, "auto"), (1, 400, 2, 32, "auto"),
    # the generic kernels forced on shapes the MFMA kernels also take (same outputs)
    (2, 257, 2, 80, "generic"), (1, 70, 2, 96, "generic"),
    # the backward variants (VIT_ATTN_BWD): paired roles, and the non-persistent one-pass kernel
    # on shapes the persistent one-pass kernel takes by default (B*NH > CUs: several items per WG)
    (2, 197, 3, 64, "pair"), (3, 33, 4, 64, "pair"), (1, 70, 1, 128, "pair"), (2, 257, 2, 80, "pair"),
    (2, 197, 3, 64, "one"), (3, 33, 4, 64, "one"),
    (24, 197, 12, 64, "mfma"), (30, 77, 12, 32, "mfma"), (30, 100, 12, 64, "mfma"), (50, 40, 8, 64, "mfma")])
def test_attention_fused_bf16(gpu, oracle64, monkeypatch, B, T, NH, HS, path):
    """bf16 attention (fused MFMA kernels for head sizes 32/64/80/96/128 while the head's images fit
    the LDS, generic VALU kernels past that) vs the fp64 oracle of the reference loops on the same
    bf16-rounded inputs."""
    if path == "generic":
        monkeypatch.setenv("VIT_ATTN_GENERIC", "1")
    if path in ("pair", "one"):
        monkeypatch.setenv("VIT_ATTN_BWD", path)
    v, o = gpu, oracle64
    C = HS * NH
    kind = v.lib().vit_attention_kernel_kind(T, C, NH)
    assert kind == {"mfma": 1, "pair": 1, "one": 1, "generic": 2}.get(path, 2), (path, kind)
    rng = np.random.default_rng(T * 7 + NH)
    qkv = rng.normal(size=B * T * 3 * C).astype(np.float32)
    qb = v.bf16_bits(qkv)
    qr = v.bf16_to_f32(qb).astype(np.float64)
    n = B * T * NH * T
    out, pre, att = np.zeros(B * T * C), np.zeros(n), np.zeros(n)
    o.call("attention_forward", out, pre, att, qr, B, T, C, NH)
    gq = D(v, qb, np.uint16)
    gout, glse = Z(v, B * T * C, np.uint16), Z(v, B * NH * T)
    v.call("attention_forward_fused_bf16", gout, glse, gq, B, T, C, NH)
    o_gpu = v.bf16_to_f32(gout.numpy())
    assert rel_err(o_gpu, out) < 1e-2
    # lse (log2 domain) = log2(sum exp(score)) per (b,h,t)
    s = pre.reshape(B, T, NH, T).transpose(0, 2, 1, 3)
    lse_ref = np.log2(np.exp(s).sum(-1))
    assert np.abs(glse.numpy().reshape(B, NH, T) - lse_ref).max() < 1e-2
    # backward vs the oracle run on the same bf16-rounded inputs (the O fed to delta is the GPU's)
    dy = rng.normal(size=B * T * C).astype(np.float32)
    dyb = v.bf16_bits(dy)
    dyr = v.bf16_to_f32(dyb).astype(np.float64)
    dinp = np.zeros(B * T * 3 * C)
    o.call("attention_backward", dinp, np.zeros(n), np.zeros(n), dyr, qr, att, B, T, C, NH)
    gd = Z(v, B * T * 3 * C, np.uint16)
    v.call("attention_backward_fused_bf16", gd, D(v, dyb, np.uint16), gq, gout, glse, B, T, C, NH)
    g = v.bf16_to_f32(gd.numpy()).reshape(B, T, 3, C)
    r = dinp.reshape(B, T, 3, C)
    for k, name in enumerate("qkv"):
        assert rel_err(g[:, :, k], r[:, :, k]) < 3e-2, name


@pytest.mark.parametrize("B,T,NH,HS", [(2, 197, 3, 64), (24, 197, 12, 64), (30, 100, 12, 64), (3, 257, 16, 80),
                                       (2, 129, 4, 64), (2, 161, 2, 80), (2, 65, 2, 32)])
def test_attention_backward_variants(gpu, oracle64, monkeypatch, B, T, NH, HS):
    """Every backward kernel (VIT_ATTN_BWD: persistent one-pass default, one workgroup per item,
    paired roles) on the same inputs: each within the bf16 gate of the fp64 oracle, the variants
    within bf16 rounding of each other, and each deterministic (two launches bitwise equal).
    T = 32k + 1 (ViT-H/14: head size 80, T = 257; and 129 / 161 / 65 at head sizes 64 / 80 / 32): the
    one-pass kernel over the first T-1 keys and all T queries with the last key on its VALU side
    path (its dS per query joins dQ as a rank-1 term, its dK / dV rows summed by one thread per
    output); VIT_ATTN_BWD=pair keeps the paired-role kernel."""
    v, o = gpu, oracle64
    C = HS * NH
    rng = np.random.default_rng(T * 7 + NH)  # the seed of test_attention_fused_bf16
    qkv = rng.normal(size=B * T * 3 * C).astype(np.float32)
    qb = v.bf16_bits(qkv)
    qr = v.bf16_to_f32(qb).astype(np.float64)
    n = B * T * NH * T
    out, pre, att = np.zeros(B * T * C), np.zeros(n), np.zeros(n)
    o.call("attention_forward", out, pre, att, qr, B, T, C, NH)
    gq = D(v, qb, np.uint16)
    gout, glse = Z(v, B * T * C, np.uint16), Z(v, B * NH * T)
    v.call("attention_forward_fused_bf16", gout, glse, gq, B, T, C, NH)
    dyb = v.bf16_bits(rng.normal(size=B * T * C).astype(np.float32))
    dinp = np.zeros(B * T * 3 * C)
    o.call("attention_backward", dinp, np.zeros(n), np.zeros(n), v.bf16_to_f32(dyb).astype(np.float64), qr, att,
           B, T, C, NH)
    r = dinp.reshape(B, T, 3, C)
    res = {}
    for variant in ["persistent", "one", "pair"]:
        monkeypatch.setenv("VIT_ATTN_BWD", variant)
        outs = []
        for _ in range(2):
            gd = Z(v, B * T * 3 * C, np.uint16)
            v.call("attention_backward_fused_bf16", gd, D(v, dyb, np.uint16), gq, gout, glse, B, T, C, NH)
            outs.append(gd.numpy())
        assert np.array_equal(outs[0], outs[1]), (variant, "nondeterministic")
        res[variant] = v.bf16_to_f32(outs[0]).reshape(B, T, 3, C)
        errs = [rel_err(res[variant][:, :, k], r[:, :, k]) for k in range(3)]
        print("\n", variant, " ".join(f"{e:.4f}" for e in errs))
        assert max(errs) < 3e-2, (variant, errs)
    for variant in ["one", "pair"]:
        assert rel_err(res[variant], res["persistent"]) < 2e-2, variant
    # the fused qkv-bias gradient (trainer form): column sums of dqkv, accumulated (+=)
    for variant in ["persistent", "one", "pair"]:
        monkeypatch.setenv("VIT_ATTN_BWD", variant)
        db = D(v, np.ones(3 * C, np.float32))
        v.call("attention_backward_fused_bf16_ex", Z(v, B * T * 3 * C, np.uint16), D(v, dyb, np.uint16), gq, gout,
               glse, B, T, C, NH, db)
        assert rel_err(db.numpy() - 1.0, dinp.reshape(B * T, 3 * C).sum(0)) < 3e-2, variant


def test_error_channel(gpu):
    """Unsupported shapes set the sticky error instead of launching (no silent fallback)."""
    v = gpu
    out = Z(v, 64, np.uint16)
    with pytest.raises(v.VitError):
        v.call("attention_forward_fused_bf16", out, Z(v, 64), Z(v, 3 * 81, np.uint16), 1, 1, 81, 1)


# ------------------------------------------------------------------ generic bf16 GEMM engine
# The engines the trainer launches (2 = 256x256 one workgroup per CU, with the split-K weight gradients
# on 256x128; 7 = persistent streaming 256x256; 11 = 7 with the two-group ping-pong 192x256 engine).  The variants that measured
# slower (4 = 256x128 everywhere, 5 = its software-pipelined form, 9 = one wave per SIMD, 10 = split
# tail) run only with VIT_TEST_EXPERIMENTAL=1 against a `make EXPERIMENTAL=1` library.
EXPERIMENTAL = os.environ.get("VIT_TEST_EXPERIMENTAL") == "1"
ENGINES = [2, 7, 11] + ([4, 5, 9, 10] if EXPERIMENTAL else [])


@pytest.fixture(params=ENGINES)
def engine(request, gpu):
    """Run a test under each GEMM engine of ENGINES, then restore the default."""
    gpu.lib().gemm_bf16_set_variant(request.param)
    yield request.param
    gpu.lib().gemm_bf16_set_variant(0)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (304, 520, 128), (776, 1000, 192), (512, 264, 640),
                                   (1000, 136, 96)])
@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 0), (0, 1)])
def test_gemm_bf16_layouts(gpu, engine, M, N, K, ak, bk):
    """Every operand layout through the GEMM engines (LDS-DMA 256x128 / 256x256, and the 128x128
    kernel for shapes they do not take), ragged M/N."""
    v = gpu
    rng = np.random.default_rng(M * 7 + N * 3 + K + 10 * ak + bk)
    a = rng.normal(size=(M, K)).astype(np.float32)
    b = rng.normal(size=(K, N)).astype(np.float32)
    ab, bb = v.bf16_bits(a), v.bf16_bits(b)
    ar, br = v.bf16_to_f32(ab).reshape(M, K).astype(np.float64), v.bf16_to_f32(bb).reshape(K, N).astype(np.float64)
    A = D(v, ab.reshape(M, K) if ak else ab.reshape(M, K).T.copy(), np.uint16)
    Bm = D(v, bb.reshape(K, N).T.copy() if bk else bb.reshape(K, N), np.uint16)
    bias = rng.normal(size=N).astype(np.float32)
    ref = ar @ br
    for epi in (0, 2, 3):
        out = Z(v, M * N, np.uint16 if epi == 3 else np.float32)
        dbias = Z(v, M) if (epi == 2 and not ak) else None
        v.call("gemm_bf16_ex", out, N, A, K if ak else M, ak, Bm, K if bk else N, bk,
               D(v, bias) if epi != 2 else None, dbias, M, N, K, epi, 0)
        got = out.numpy().reshape(M, N)
        if epi == 3:
            got = v.bf16_to_f32(got)
        want = ref + (bias if epi != 2 else 0)
        assert rel_err(got, want) < (1e-2 if epi == 3 else 2e-3), epi
        if dbias is not None:
            assert rel_err(dbias.numpy(), ar.sum(1)) < 2e-3


@pytest.mark.parametrize("gm", [0, 1, 3, 8, 14])
@pytest.mark.parametrize("M,N,K", [(6304, 3072, 768), (1576, 768, 3072), (776, 1000, 128)])
def test_gemm_bf16_tile_order_bit_identical(gpu, M, N, K, gm):
    """The persistent engine's tile order (row-major, or groups of gm row panels walked column by
    column, partial last group included) only moves tiles between CUs and rounds: every output is
    bit-identical to the one-tile engine (variant 2)."""
    v = gpu
    L = v.lib()
    rng = np.random.default_rng(M + 5 * N + K + gm)
    ab = v.bf16_bits(rng.uniform(-1, 1, size=(M, K)).astype(np.float32))
    wb = v.bf16_bits((rng.uniform(-1, 1, size=(N, K)) * 0.1).astype(np.float32))
    A, W = D(v, ab, np.uint16), D(v, wb, np.uint16)
    bias = D(v, rng.normal(size=N).astype(np.float32))
    res = D(v, rng.normal(size=(M, N)).astype(np.float32))
    outs = {}
    try:
        for var, flags in ((2, 0), (7, (gm + 1) << 16)):
            L.gemm_bf16_set_variant(var)
            L.gemm_bf16_set_debug(flags)
            o = []
            for epi in (3, 5):
                c = Z(v, M * N, np.float32 if epi == 5 else np.uint16)
                v.call("gemm_bf16_fused", c, None, N, res if epi == 5 else None, N, A, K, 1, W, K, 1, bias,
                       None, M, N, K, epi)
                o.append(c.numpy())
            outs[var] = o
    finally:
        L.gemm_bf16_set_debug(0)
        L.gemm_bf16_set_variant(0)
    for x, y in zip(outs[2], outs[7]):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("pair", [(2, 7), (7, 11)] + ([(4, 5), (2, 9)] if EXPERIMENTAL else []))
@pytest.mark.parametrize("M,N,K", [(6304, 3072, 768), (1576, 768, 3072), (520, 384, 256), (776, 1000, 128),
                                   (50432, 768, 768), (25216, 3072, 768), (25216, 768, 3072), (25216, 768, 2304)])
def test_gemm_bf16_pipelined_bit_identical(gpu, M, N, K, pair):
    """Engine variants that reorder only the schedule, not the arithmetic: the software-pipelined
    256x128 main loop (variant 5, g4::gemm_kernel_pipe) against the 256x128 engine (4), and the
    persistent streaming 256x256 engine (7, g2::gemm_kernel_s: tiles walked per CU, the next tile's
    first K-steps fetched under the epilogue, 32-row staging) against the one-tile 256x256 engine
    (2), and the one-wave-per-SIMD persistent engine (9, g5::gemm_kernel_w4: 128 x 128 per wave, one
    barrier per 32-deep K-step) against it too.  Same MFMAs in the same K order per accumulator and the same epilogue arithmetic: every
    fused epilogue of the trainer (bf16 store, GELU pair, fp32 residual, x aux + column sums)
    bit-identical, at the trainer's K (768, 3072), its M (50 432 = 197 full 256-row tiles: several
    tiles per CU) and ragged M / N."""
    v0, v1 = pair
    if (v0, v1) == (2, 7) and M >= 25216 and K > 768:
        pytest.skip("covered by the (2, 7) shapes above")
    v = gpu
    L = v.lib()
    rng = np.random.default_rng(M + 3 * N + K)
    ab = v.bf16_bits(rng.uniform(-1, 1, size=(M, K)).astype(np.float32))
    wb = v.bf16_bits((rng.uniform(-1, 1, size=(N, K)) * 0.1).astype(np.float32))
    A, W = D(v, ab, np.uint16), D(v, wb, np.uint16)
    bias = D(v, rng.normal(size=N).astype(np.float32))
    res = D(v, rng.normal(size=(M, N)).astype(np.float32))
    aux = D(v, v.bf16_bits(rng.normal(size=(M, N)).astype(np.float32)), np.uint16)
    outs = {}
    pp_hits = 0
    try:
        for var in (v0, v1):
            L.gemm_bf16_set_variant(var)
            L.gemm_bf16_set_debug(512 if var == 11 else 0)  # variant 11 on every shape it can take
            v.kernel_hits_reset()
            o = {}
            for epi in (3, 5, 8, 9):
                c = Z(v, M * N, np.float32 if epi == 5 else np.uint16)
                c2 = Z(v, M * N, np.uint16) if epi == 8 else None
                cs = D(v, np.zeros(N, np.float32)) if epi == 9 else None
                v.call("gemm_bf16_fused", c, c2, N, res if epi == 5 else (aux if epi == 9 else None), N,
                       A, K, 1, W, K, 1, bias if epi in (3, 5, 8) else None, cs, M, N, K, epi)
                o[epi] = [c.numpy()] + ([c2.numpy()] if c2 is not None else []) + ([cs.numpy()] if cs is not None else [])
            outs[var] = o
            if var == 11:
                pp_hits = int(v.kernel_hits()[v.HIT_GEMM_PP])
    finally:
        L.gemm_bf16_set_debug(0)
        L.gemm_bf16_set_variant(0)
    for epi in outs[v0]:
        for k, (x, y) in enumerate(zip(outs[v0][epi], outs[v1][epi])):
            if v1 == 11 and epi == 9 and k == 1:
                # the ping-pong engine sums columns per 96 output rows (128 elsewhere): the fp32 sums
                # differ in association only
                assert np.abs(x - y).max() <= 1e-5 * np.abs(x).max(), epi
            else:
                assert np.array_equal(x, y), epi
    assert np.abs(outs[v1][5][0]).max() > 0
    if v1 == 11:  # the engine ran where it applies (N % 256 == 0, M >= 256, K >= 256)
        assert pp_hits == (4 if (N % 256 == 0 and M >= 256 and K >= 256) else 0), pp_hits


@pytest.mark.parametrize("M,N,K", [(50432, 768, 768), (50432, 768, 3072), (25216, 768, 3072), (25216, 768, 2304),
                                   (2056, 768, 320), (1000, 520, 128)])
@pytest.mark.skipif(not EXPERIMENTAL, reason="variant 10 is built with make EXPERIMENTAL=1 only")
def test_gemm_bf16_tail_split(gpu, M, N, K):
    """Variant 10: the persistent engine with the last, partly filled round's tiles split along K
    (fp32 partial tiles + gemm_tail_fix_k) against variant 7 on the same inputs, at the trainer's
    N = 768 shapes (591 / 297 tiles: a tail of 79 / 41 tiles on 256 CUs) and ragged ones: the bias,
    fp32-residual and bf16-store epilogues agree to fp32 summation order (the bf16 store to one bf16
    ulp) over the whole output, and two launches are bitwise equal (fixed part order).  (The
    full-round tiles are not separately asserted bitwise.)"""
    v = gpu
    L = v.lib()
    rng = np.random.default_rng(M + 5 * N + K)
    ab = v.bf16_bits(rng.uniform(-1, 1, size=(M, K)).astype(np.float32))
    wb = v.bf16_bits((rng.uniform(-1, 1, size=(N, K)) * 0.1).astype(np.float32))
    A, W = D(v, ab, np.uint16), D(v, wb, np.uint16)
    bias = D(v, rng.normal(size=N).astype(np.float32))
    res = D(v, rng.normal(size=(M, N)).astype(np.float32))
    outs = {}
    try:
        for var in (7, 10, 10):
            L.gemm_bf16_set_variant(var)
            o = []
            for epi in (0, 3, 5):
                c = Z(v, M * N, np.uint16 if epi == 3 else np.float32)
                v.call("gemm_bf16_fused", c, None, N, res if epi == 5 else None, N, A, K, 1, W, K, 1, bias,
                       None, M, N, K, epi)
                o.append(c.numpy())
            outs.setdefault(var, []).append(o)
    finally:
        L.gemm_bf16_set_variant(0)
    ref, got, again = outs[7][0], outs[10][0], outs[10][1]
    for e, (x, y, z) in enumerate(zip(ref, got, again)):
        assert np.array_equal(y, z), e
        if x.dtype == np.uint16:
            xf, yf = v.bf16_to_f32(x), v.bf16_to_f32(y)
            assert np.abs(xf - yf).max() <= 2 ** -7 * np.abs(xf).max(), e
        else:
            assert np.abs(x - y).max() <= 1e-5 * np.abs(x).max(), e
    assert np.abs(ref[2]).max() > 0


def _gelu64(x):
    s = np.sqrt(2.0 / np.pi)
    return 0.5 * x * (1.0 + np.tanh(s * (x + 0.044715 * x ** 3)))


def _gelu_grad64(x):  # D4-corrected derivative (sech^2 of the tanh argument)
    s = np.sqrt(2.0 / np.pi)
    a = s * (x + 0.044715 * x ** 3)
    th = np.tanh(a)
    return 0.5 * (1 + th) + 0.5 * x * (1 - th * th) * s * (1 + 3 * 0.044715 * x * x)


@pytest.mark.parametrize("M,N,K", [(1576, 768, 192), (520, 384, 256), (6304, 3072, 192), (8192, 2304, 96)])
def test_gemm_bf16_fused_epilogues(gpu, engine, M, N, K):
    """The trainer's fused epilogues against float64 numpy: bias+GELU pair (fc forward),
    bias+fp32 residual (proj / fcproj forward), GELU' x aux with the fused column sum
    (fcproj dgrad -> fc bias gradient)."""
    v = gpu
    rng = np.random.default_rng(M + N + K)
    a = rng.uniform(-1, 1, size=(M, K)).astype(np.float32)
    w = (rng.uniform(-1, 1, size=(N, K)) * 0.1).astype(np.float32)
    ab, wb = v.bf16_bits(a), v.bf16_bits(w)
    ar = v.bf16_to_f32(ab).reshape(M, K).astype(np.float64)
    wr = v.bf16_to_f32(wb).reshape(N, K).astype(np.float64)
    bias = rng.normal(size=N).astype(np.float32)
    A, W = D(v, ab, np.uint16), D(v, wb, np.uint16)
    pre = ar @ wr.T + bias
    # 4: C = pre (bf16), C2 = gelu(pre) (bf16)
    c1, c2 = Z(v, M * N, np.uint16), Z(v, M * N, np.uint16)
    v.call("gemm_bf16_fused", c1, c2, N, None, 0, A, K, 1, W, K, 1, D(v, bias), None, M, N, K, 4)
    assert rel_err(v.bf16_to_f32(c1.numpy()).reshape(M, N), pre) < 1e-2
    assert rel_err(v.bf16_to_f32(c2.numpy()).reshape(M, N), _gelu64(pre)) < 1e-2
    # 5: C_f32 = acc + bias + aux_f32
    res = rng.normal(size=(M, N)).astype(np.float32)
    c3 = Z(v, M * N)
    v.call("gemm_bf16_fused", c3, None, N, D(v, res), N, A, K, 1, W, K, 1, D(v, bias), None, M, N, K, 5)
    assert rel_err(c3.numpy().reshape(M, N), pre + res) < 2e-3
    # 6: C_bf16 = (acc) * gelu'(aux_bf16); colsum += column sums of C (dgrad layout: W is [K][N])
    wkn = (rng.uniform(-1, 1, size=(K, N)) * 0.1).astype(np.float32)
    wkb = v.bf16_bits(wkn)
    wkr = v.bf16_to_f32(wkb).reshape(K, N).astype(np.float64)
    x = rng.normal(size=(M, N)).astype(np.float32)
    xb = v.bf16_bits(x)
    xr = v.bf16_to_f32(xb).reshape(M, N).astype(np.float64)
    c4, cs = Z(v, M * N, np.uint16), D(v, np.ones(N, np.float32))
    v.call("gemm_bf16_fused", c4, None, N, D(v, xb, np.uint16), N, A, K, 1, D(v, wkb, np.uint16), N, 0,
           None, cs, M, N, K, 6)
    want = (ar @ wkr) * _gelu_grad64(xr)
    assert rel_err(v.bf16_to_f32(c4.numpy()).reshape(M, N), want) < 1e-2
    assert rel_err(cs.numpy(), 1.0 + want.sum(0)) < 1e-2
    # 8: C = gelu'(pre), C2 = gelu(pre) (the trainer's fc forward); 9: C = acc * aux (its fcproj
    # dgrad, aux = the stored gelu') with the column sums
    c5, c6 = Z(v, M * N, np.uint16), Z(v, M * N, np.uint16)
    v.call("gemm_bf16_fused", c5, c6, N, None, 0, A, K, 1, W, K, 1, D(v, bias), None, M, N, K, 8)
    assert rel_err(v.bf16_to_f32(c5.numpy()).reshape(M, N), _gelu_grad64(pre)) < 1e-2
    assert np.array_equal(c6.numpy(), c2.numpy())  # same engine: the epi-4 GELU output, bit for bit
    c7, cs2 = Z(v, M * N, np.uint16), D(v, np.ones(N, np.float32))
    v.call("gemm_bf16_fused", c7, None, N, D(v, xb, np.uint16), N, A, K, 1, D(v, wkb, np.uint16), N, 0,
           None, cs2, M, N, K, 9)
    want = (ar @ wkr) * xr
    assert rel_err(v.bf16_to_f32(c7.numpy()).reshape(M, N), want) < 1e-2
    assert rel_err(cs2.numpy(), 1.0 + want.sum(0)) < 1e-2


# ------------------------------------------------------------------ bf16 op-level family
@pytest.mark.parametrize("rows,C", [(394, 192), (100, 768), (7, 1000)])
def test_layernorm_backward_bf16(gpu, oracle64, rows, C):
    """layernorm_backward_bf16 (train_vit.rs:603, bf16 LN-output gradient as the dgrad GEMMs write
    it) vs the fp64 oracle on the same bf16-rounded dout: += semantics on all three outputs."""
    v, o = gpu, oracle64
    rng = np.random.default_rng(C + 1)
    x, w, b = rng.normal(size=rows * C) * 3 + 1, rng.normal(size=C), rng.normal(size=C)
    out, m, r = np.zeros(rows * C), np.zeros(rows), np.zeros(rows)
    o.call("layernorm_forward", out, m, r, x, w, b, rows, 1, C)
    dyb = v.bf16_bits(rng.normal(size=rows * C).astype(np.float32))
    dyr = v.bf16_to_f32(dyb).astype(np.float64)
    p0 = rng.normal(size=rows * C)
    di, dw, db = p0.copy(), np.ones(C), np.zeros(C)
    o.call("layernorm_backward", di, dw, db, dyr, x, w, m, r, rows, 1, C)
    gdi, gdw, gdb = D(v, p0), D(v, np.ones(C)), Z(v, C)
    v.call("layernorm_backward_bf16", gdi, gdw, gdb, D(v, dyb, np.uint16), D(v, x), D(v, w), D(v, m), D(v, r),
           rows, 1, C)
    assert rel_err(gdi.numpy(), di) < 1e-4 and rel_err(gdw.numpy(), dw) < 1e-5 and rel_err(gdb.numpy(), db) < 1e-5


def test_gelu_bf16_pair(gpu, oracle64):
    """gelu_forward_bf16 / gelu_backward_bf16 (train_vit.rs:482, :639 with D4) vs the fp64 oracle
    on bf16-rounded inputs: forward within bf16 output rounding, backward (+= fp32) 1e-5."""
    v, o = gpu, oracle64
    rng = np.random.default_rng(12)
    n = 100003
    xb = v.bf16_bits((rng.normal(size=n) * 3).astype(np.float32))
    gb = v.bf16_bits(rng.normal(size=n).astype(np.float32))
    xr, gr = v.bf16_to_f32(xb).astype(np.float64), v.bf16_to_f32(gb).astype(np.float64)
    ref = np.zeros(n)
    o.call("gelu_forward", ref, xr, n)
    out = Z(v, n, np.uint16)
    v.call("gelu_forward_bf16", out, D(v, xb, np.uint16), n)
    assert rel_err(v.bf16_to_f32(out.numpy()), ref) < 4e-3
    p0 = rng.normal(size=n)
    dref = p0.copy()
    o.call("gelu_backward", dref, xr, gr, n)
    dout = D(v, p0)
    v.call("gelu_backward_bf16", dout, D(v, xb, np.uint16), D(v, gb, np.uint16), n)
    assert rel_err(dout.numpy(), dref) < 1e-5


def test_attention_forward_null_scores(gpu, oracle32):
    """attention_forward with preatt / att NULL (nullable in fused use): same output,
    nothing else written."""
    v, o = gpu, oracle32
    B, T, C, NH = 2, 17, 32, 2
    rng = np.random.default_rng(3)
    x = o.arr(rng.normal(size=B * T * 3 * C))
    n = B * T * NH * T
    ref, pre, att = o.arr(np.zeros(B * T * C)), o.arr(np.zeros(n)), o.arr(np.zeros(n))
    o.call("attention_forward", ref, pre, att, x, B, T, C, NH)
    out = Z(v, B * T * C)
    v.call("attention_forward", out, None, None, D(v, x), B, T, C, NH)
    assert rel_err(out.numpy(), ref) < 1e-5
    gatt = Z(v, n)
    v.call("attention_forward", out, None, gatt, D(v, x), B, T, C, NH)
    assert rel_err(gatt.numpy(), att) < 1e-5


def test_trainer_rejects_out_of_range_labels(gpu):
    v = gpu
    cfg = v.data.CONFIGS["test"]
    m = v.ViT.build(cfg, 2, v.VIT_FP32, params=v.data.init_params(cfg, "parity", seed=1))
    px, lab = v.data.synthetic_batch(cfg, 2, seed=2)
    lab[1] = cfg.num_classes
    with pytest.raises(v.VitError, match="outside"):
        m.set_batch(px, lab)
    m.close()
