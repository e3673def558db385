"""Trainer-level parity of the kernel set the benchmark times.

The model-level parity tests elsewhere run at B <= 8 (or B=1 at full ViT-B/16 width), where M = B*T
is too small for the production GEMM engines: every GEMM there takes the 128x128 fallback.  Here a
ViT with ViT-B/16's geometry per layer-op *shape class* runs at a batch where every GEMM of the bf16
step takes the engines bench.py times:

    C=256, NH=4 (head size 64, T=197 at 224^2/16), L=2, 1000 classes, B=128:
    B*T = 25,216 = 394 x 64 -> every K % 64 == 0 and every M, N >= 256; the weight gradients reduce
    over K = 25,216 (split-K slabs); 512 (b, h) attention items > 256 CUs.

The bf16 step runs exactly as bench.py runs it (stream concurrency on, two micro-batch streams) and
with one micro-batch (the persistent attention backward then walks two items per workgroup); the
launch counters (vit_kernel_hits) prove which kernels ran: the 256x256 LDS-DMA GEMM with the bf16
store (3), fp32-residual (5), GELU/GELU' pair (8) and x-aux + bias colsum (9) epilogues, the 256x128
split-K slab weight gradients + slab reduce, the fused MFMA attention forward and the persistent
one-pass backward, and NO 128x128 fallback.  All against the fp32 CPU oracle (oracle/oracle.c, the
reference loops of /root/reference/train_vit.rs:188-373) on the same seeded inputs, per tensor
(tests/parity.py: logits, loss, all 20 gradient tensors).
"""
import numpy as np
import pytest

import parity

pytestmark = pytest.mark.gpu

B = 128


def _cfg(v):
    return v.data.VitCfg("prod_l2", img=224, patch=16, channels=256, num_layers=2, num_heads=4, num_classes=1000)


@pytest.fixture(scope="module")
def ref(gpu, oracle32):
    import oracle_ctypes as oc
    v = gpu
    cfg = _cfg(v)
    params = v.data.init_params(cfg, "parity", seed=3)
    px, lab = v.data.synthetic_batch(cfg, B, seed=5)
    c = oc.VitConfig(cfg.img, cfg.patch, cfg.in_ch, cfg.channels, cfg.num_layers, cfg.num_heads, cfg.num_classes)
    m = oc.RefViT(oracle32, c, B)
    p = oracle32.arr(params)
    loss = m.forward(p, px, lab)
    g = np.zeros_like(p)
    m.backward(p, g)
    out = dict(cfg=cfg, params=params, px=px, lab=lab, loss=loss, logits=m.logits(), grads=g)
    del m
    return out


def _run(v, ref, prec, nmb):
    m = v.ViT.build(ref["cfg"], B, prec, params=ref["params"])
    m.set_concurrency(True)
    m.set_option("microbatch", nmb)
    m.set_batch(ref["px"], ref["lab"])
    m.sync()
    v.kernel_hits_reset()
    m.zero_grad()
    loss = m.forward()
    m.backward()
    g = m.grads()
    hits = v.kernel_hits()
    logits = m.logits()
    m.close()
    return loss, logits, g, hits


def _gate(ref, loss, logits, g, gate, label):
    pairs = parity.tensors(ref["cfg"], logits, g, ref["logits"], ref["grads"])
    bad, rep = parity.check(pairs, gate)
    lrel = abs(loss - ref["loss"]) / abs(ref["loss"])
    print(f"\n{label}: loss {lrel:.2e}, {parity.summary(rep)}")
    assert lrel <= gate["loss"], (label, lrel)
    assert not bad, (label, bad)
    return rep


@pytest.mark.parametrize("nmb", [2, 1])
def test_production_bf16_step_vs_oracle(gpu, ref, nmb):
    v = gpu
    loss, logits, g, hits = _run(v, ref, v.VIT_BF16, nmb)
    _gate(ref, loss, logits, g, parity.BF16, f"bf16 nmb={nmb}")
    L = ref["cfg"].num_layers
    G2, G4 = v.HIT_GEMM_256x256, v.HIT_GEMM_256x128
    assert hits[v.HIT_GEMM_128:v.HIT_GEMM_128 + 16].sum() == 0, "128x128 fallback ran"
    assert hits[G2 + 3] >= 4 * L * nmb          # qkv fwd + fc / proj / qkv dgrads (bf16 store)
    assert hits[G2 + 5] == 2 * L * nmb          # proj / fcproj fwd (+ bias + fp32 residual)
    assert hits[G2 + 8] == L * nmb              # fc fwd (gelu' / gelu pair)
    assert hits[G2 + 9] == L * nmb              # fcproj dgrad (x stored gelu', fc-bias colsum)
    assert hits[G4 + 7] >= 4 * L                # split-K weight gradients into slabs
    # every split-K launch reduces its slabs once (the head's fp32 GEMMs included); no atomics
    assert hits[v.HIT_SPLITK_REDUCE] == hits[G4 + 7] + hits[G2 + 7] + hits[v.HIT_GEMM_F32 + 7]
    assert hits[v.HIT_ATTN_FWD_MFMA] == L * nmb
    assert hits[v.HIT_ATTN_BWD_PERSISTENT] == L * nmb


def test_production_fp32_step_vs_oracle(gpu, ref):
    v = gpu
    loss, logits, g, hits = _run(v, ref, v.VIT_FP32, 1)
    _gate(ref, loss, logits, g, parity.FP32, "fp32")
    assert hits[v.HIT_GEMM_F32:v.HIT_GEMM_F32 + 16].sum() > 0


def test_production_fp8_step_vs_oracle(gpu, ref):
    """fp8 mode (BASELINE config 5's MXFP8 forward / input-gradient GEMMs) against the oracle, gated by
    the operand-rounding model of tests/parity.py FP8_MODEL: relative to the bf16 mode on the same
    inputs only the GEMM operands change precision (e4m3, unit roundoff 2^-4, vs bf16's 2^-8), so
    to first order every tensor's error grows by at most 16x the bf16 mode's error on that tensor
    (floored at 16x bf16's unit roundoff), with a 1.5x margin."""
    v = gpu
    lb, zb, gb, _ = _run(v, ref, v.VIT_BF16, 2)
    lf, zf, gf, hits = _run(v, ref, v.VIT_FP8, 2)
    assert hits[v.HIT_GEMM_FP8:v.HIT_GEMM_FP8 + 16].sum() >= 8 * ref["cfg"].num_layers
    pb = parity.tensors(ref["cfg"], zb, gb, ref["logits"], ref["grads"])
    pf = parity.tensors(ref["cfg"], zf, gf, ref["logits"], ref["grads"])
    bad = parity.check_fp8(pf, pb)
    print("\nfp8:", {n: round(x["max"], 4) for n, x in parity.fp8_report(pf).items()})
    lrel_b = abs(lb - ref["loss"]) / abs(ref["loss"])
    lrel_f = abs(lf - ref["loss"]) / abs(ref["loss"])
    assert lrel_f <= parity.fp8_limit(lrel_b), (lrel_f, lrel_b)
    assert not bad, bad
    # regression gate: each tensor's rms error within 1.5x its recorded value (tests/parity.py)
    reg = parity.fp8_rms_gate("production", parity.fp8_report(pf))
    assert not reg, reg


def test_production_bf16_step_is_bitwise_repeatable(gpu, ref):
    """The production kernel set (2 micro-batch streams + the weight-gradient stream) reduces every
    gradient in a fixed order: two steps on fresh trainers give bit-identical gradients."""
    v = gpu
    a = _run(v, ref, v.VIT_BF16, 2)
    b = _run(v, ref, v.VIT_BF16, 2)
    assert a[0] == b[0]
    assert np.array_equal(a[1], b[1])
    assert np.array_equal(a[2], b[2])


@pytest.mark.parametrize("prec_name", ["VIT_BF16", "VIT_FP32"])
def test_production_dp_shard_sum(gpu, ref, prec_name):
    """The DP identity at the production kernel set (VERDICT r03 missing #2): the per-GPU shards
    of a DP=2 step (B=64 each, b_global = 128, dloss = 1/B_global as train_vit.rs:288 / D15) run
    through the HIP trainer on the production engines (64 x 197 = 12 608 tokens = 197 x 64: the
    256x256 epilogues, split-K slab weight gradients, persistent attention backward); their
    gradients summed on the host equal the full-batch oracle gradient within the mode's gate."""
    from test_gpu_model import _shard_sum
    v = gpu
    prec = getattr(v, prec_name)
    cfg = ref["cfg"]
    v.kernel_hits_reset()
    losses, gsum = _shard_sum(v, cfg, prec, ref["params"], ref["px"], ref["lab"], 2)
    hits = v.kernel_hits()
    gate = parity.BF16 if prec == v.VIT_BF16 else parity.FP32
    lrel = abs(np.mean(losses) - ref["loss"]) / abs(ref["loss"])
    assert lrel <= gate["loss"], lrel
    pairs = {n: (a, b) for (n, a), b in zip(cfg.split(gsum.astype(np.float32)).items(), cfg.split(ref["grads"]).values())}
    bad, rep = parity.check(pairs, gate)
    print(f"\n{prec_name} DP=2 shard sum vs oracle: loss {lrel:.2e}, {parity.summary(rep)}")
    assert not bad, bad
    if prec == v.VIT_BF16:
        assert hits[v.HIT_GEMM_128:v.HIT_GEMM_128 + 16].sum() == 0, "128x128 fallback ran"
        assert hits[v.HIT_ATTN_BWD_PERSISTENT] == 2 * cfg.num_layers


@pytest.mark.parametrize("prec_name", ["VIT_BF16", "VIT_FP8"])
def test_production_streaming_engines_bit_identical(gpu, ref, prec_name):
    """The persistent streaming GEMM engines (the production variant 7: g2::gemm_kernel_s for bf16,
    f8::gemm_kernel_s for MXFP8 with its fused row / column MX outputs) against the one-tile engines
    (variant 2) on the whole production step (2 micro-batch streams): loss, logits and every gradient
    bit-identical — same MFMAs in the same order, same epilogue arithmetic."""
    v = gpu
    prec = getattr(v, prec_name)
    out = {}
    try:
        for var in (2, 0):
            v.lib().gemm_bf16_set_variant(var)
            out[var] = _run(v, ref, prec, 2)
    finally:
        v.lib().gemm_bf16_set_variant(0)
    (l2, z2, g2, _), (l7, z7, g7, _) = out[2], out[0]
    assert l2 == l7
    assert np.array_equal(z2, z7)
    assert np.array_equal(g2, g7)
