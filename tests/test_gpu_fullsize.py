"""Oracle parity of the BENCHMARKED configurations at their own batch size.

The forward of a ViT is independent per image (train_vit.rs:188-268: every op is per token or per
(image, head); the batch only sums into the loss), so two chosen images of the full production step
are compared with an oracle forward of just those two images:
  * ViT-B/16 224^2 bf16, B=256 (BASELINE config 2 / the bench.py headline workload), two micro-batch
    streams and stream concurrency on, exactly as bench.py runs it;
  * ViT-L/16 224^2 bf16, B=256 (config 4's per-GPU shard);
  * ViT-H/14 224^2 fp8, B=128, L=32 (config 5's per-GPU shard), under the fp8 error-model gate of
    tests/parity.py: the fp8 logits' error may be at most 1.5 x 16 x the bf16 mode's error on the same
    images (bf16 error floored at 2^-8).
bf16 gate (tests/parity.py BF16): logits max-normalised error <= 2e-2 and the elementwise rule on
>= 99.99 %; per-image loss -log softmax(logits)[label] within 1e-2 relative (train_vit.rs:250-264).
The images are one from each micro-batch (first and last of the batch)."""
import numpy as np
import pytest

import parity

pytestmark = pytest.mark.gpu


def _oracle_forward(oc, o, cfg, params, px, lab):
    c = oc.VitConfig(cfg.img, cfg.patch, cfg.in_ch, cfg.channels, cfg.num_layers, cfg.num_heads,
                     cfg.num_classes)
    m = oc.RefViT(o, c, px.shape[0])
    m.forward(o.arr(params), px, lab)
    return m.logits().copy(), m.losses().copy()


def _image_losses(logits, lab):
    z = logits.astype(np.float64)
    z = z - z.max(1, keepdims=True)
    lse = np.log(np.exp(z).sum(1))
    return lse - z[np.arange(len(lab)), lab]


def _production_logits(v, cfg, prec, B, params, px, lab):
    m = v.ViT.build(cfg, B, prec, params=params)
    m.set_concurrency(True)  # as bench.py (two micro-batch streams by default)
    m.set_batch(px, lab)
    m.zero_grad()
    loss = m.forward()
    logits = m.logits().reshape(B, cfg.num_classes).copy()
    m.close()
    return loss, logits


@pytest.mark.parametrize("name,B,seed", [("vit_b16", 256, 61), ("vit_l16", 256, 63)])
def test_benchmarked_bf16_step_vs_oracle_two_images(gpu, oracle32, name, B, seed):
    import oracle_ctypes as oc
    v = gpu
    cfg = v.data.CONFIGS[name]
    params = v.data.init_params(cfg, "parity", seed=seed)
    px, lab = v.data.synthetic_batch(cfg, B, seed=seed + 1)
    loss, logits = _production_logits(v, cfg, v.VIT_BF16, B, params, px, lab)
    assert np.isfinite(loss)
    pick = np.array([0, B - 1])
    z_r, l_r = _oracle_forward(oc, oracle32, cfg, params, px[pick], lab[pick])
    z = logits[pick]
    met = parity.metrics(z, z_r, parity.BF16["tol"], parity.BF16["floor_rel"])
    l_gpu = _image_losses(z, lab[pick])
    print(f"\n{name} B={B} bf16 images {pick.tolist()}: logits max-norm err {met['max']:.2e} "
          f"frac {met['frac']:.5f}; losses {l_gpu} vs oracle {l_r}")
    assert met["max"] <= parity.BF16["tol"] and met["frac"] >= parity.BF16["frac"], met
    assert np.all(np.abs(l_gpu - l_r) <= parity.BF16["loss"] * np.abs(l_r)), (l_gpu, l_r)


def test_config5_fp8_shard_vs_oracle_two_images(gpu, oracle32):
    import oracle_ctypes as oc
    v = gpu
    cfg = v.data.CONFIGS["vit_h14"]
    B = 128
    params = v.data.init_params(cfg, "parity", seed=65)
    px, lab = v.data.synthetic_batch(cfg, B, seed=66)
    pick = np.array([0, B - 1])
    z_r, l_r = _oracle_forward(oc, oracle32, cfg, params, px[pick], lab[pick])
    err = {}
    for prec in (v.VIT_BF16, v.VIT_FP8):
        loss, logits = _production_logits(v, cfg, prec, B, params, px, lab)
        assert np.isfinite(loss)
        z = logits[pick]
        met = parity.metrics(z, z_r, parity.BF16["tol"], parity.BF16["floor_rel"])
        lerr = float(np.max(np.abs(_image_losses(z, lab[pick]) - l_r) / np.abs(l_r)))
        err[prec] = (met["max"], lerr)
    (eb, lb), (ef, lf) = err[v.VIT_BF16], err[v.VIT_FP8]
    print(f"\nvit_h14 B={B}: logits err bf16 {eb:.2e} fp8 {ef:.2e} (limit {parity.fp8_limit(eb):.2e}); "
          f"loss err bf16 {lb:.2e} fp8 {lf:.2e}")
    assert eb <= parity.BF16["tol"] and lb <= parity.BF16["loss"], (eb, lb)
    assert ef <= parity.fp8_limit(eb), (ef, eb)
    assert lf <= parity.fp8_limit(lb), (lf, lb)
