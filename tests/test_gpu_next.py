"""GPU tests of the SURVEY.md §8f "next" rows over the trainer's C ABI.

- AdamW (§8f-2): vit_trainer_step_adamw against the CPU oracle's ref_adamw_step (which is pinned
  to torch.optim.AdamW in tests/test_oracle.py), fed the GPU's own gradients — bit-exact in both
  precision modes (the update runs on the fp32 master arena; no contraction, IEEE sqrt/divide).
- Eval (§8f-4): forward without targets (mean_loss = -1, train_vit.rs:264-266; backward refused)
  and the device top-1 against numpy.argmax of the logits.
- Checkpoint resume (§8f-1): save after AdamW steps, load into a fresh trainer -> identical
  params / m / v / t, identical forward, and the next step agrees.
"""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu

HP = dict(beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.05)


@pytest.mark.parametrize("prec_name,name,B", [("fp32", "test", 3), ("bf16", "test_h64", 4)])
def test_adamw_matches_oracle(gpu, oracle32, prec_name, name, B):
    v = gpu
    o = oracle32
    cfg = v.data.CONFIGS[name]
    prec = v.VIT_FP32 if prec_name == "fp32" else v.VIT_BF16
    params = v.data.init_params(cfg, "parity", seed=3)
    px, lab = v.data.synthetic_batch(cfg, B, seed=5)
    m = v.ViT.build(cfg, B, prec, params=params)
    m.set_batch(px, lab)
    p_ref = o.arr(params)
    m_ref = o.arr(np.zeros_like(params))
    v_ref = o.arr(np.zeros_like(params))
    losses = []
    for t in range(1, 4):
        m.zero_grad()
        losses.append(m.forward())
        m.backward()
        g = m.grads()
        assert np.isfinite(g).all()
        m.optimizer_step_adamw(3e-3, **HP)
        o.adamw_step(p_ref, o.arr(g), m_ref, v_ref, 3e-3, HP["beta1"], HP["beta2"], HP["eps"],
                     HP["weight_decay"], t)
        p = m.params()
        mm, vv, tt = m.adamw_state()
        assert tt == t
        assert np.array_equal(mm, m_ref) and np.array_equal(vv, v_ref), t
        bad = int((p != p_ref).sum())
        assert bad == 0, (t, bad, float(np.abs(p - p_ref).max()))
    assert losses[-1] < losses[0]
    m.close()


@pytest.mark.parametrize("prec_name", ["fp32", "bf16"])
def test_eval_top1_and_forward_without_targets(gpu, prec_name):
    v = gpu
    cfg = v.data.CONFIGS["test_h64"]
    prec = v.VIT_FP32 if prec_name == "fp32" else v.VIT_BF16
    B = 8
    params = v.data.init_params(cfg, "parity", seed=4)
    px, _ = v.data.synthetic_batch(cfg, B, seed=6)
    m = v.ViT.build(cfg, B, prec, params=params)
    pred, correct = m.evaluate(px, None)
    assert correct == -1
    assert m.forward() == -1.0  # mean_loss of a batch without targets (train_vit.rs:265)
    logits = m.logits()
    assert np.array_equal(pred, np.argmax(logits, axis=1))
    with pytest.raises(v.VitError):
        m.backward()
    v.lib().vit_clear_error()
    lab = pred.copy()
    lab[::2] = (lab[::2] + 1) % cfg.num_classes  # half right, half wrong
    pred2, correct2 = m.evaluate(px, lab)
    assert np.array_equal(pred2, pred) and correct2 == int((pred == lab).sum()) == B // 2
    assert m.forward() > 0
    m.close()


def test_argmax_ties_take_the_first_index(gpu):
    """All-zero head -> all logits equal -> class 0 (numpy.argmax semantics); NC = 1000 spans all
    64 lanes of the row's wave."""
    v = gpu
    cfg = v.data.CONFIGS["vit_tiny16"]
    params = v.data.init_params(cfg, "parity", seed=4)
    sp = cfg.split(params)
    off = 0
    for k, a in sp.items():
        if k in ("head_w", "head_b"):
            params[off:off + a.size] = 0
        off += a.size
    px, _ = v.data.synthetic_batch(cfg, 2, seed=6)
    m = v.ViT.build(cfg, 2, v.VIT_BF16, params=params)
    pred, _ = m.evaluate(px, None)
    assert np.array_equal(pred, np.zeros(2, np.int32))
    # a single maximum in the last lane's range is found
    params[off - cfg.num_classes + 999] = 5.0  # head_b[999]
    m.set_params(params)
    pred, _ = m.evaluate(px, None)
    assert np.array_equal(pred, np.full(2, 999, np.int32))
    m.close()


def test_checkpoint_resume(gpu, tmp_path):
    v = gpu
    cfg = v.data.CONFIGS["test_h64"]
    B = 4
    params = v.data.init_params(cfg, "parity", seed=8)
    px, lab = v.data.synthetic_batch(cfg, B, seed=9)
    a = v.ViT.build(cfg, B, v.VIT_BF16, params=params)
    a.set_batch(px, lab)
    for _ in range(2):
        a.zero_grad(); a.forward(); a.backward(); a.optimizer_step_adamw(1e-3, **HP)
    path = tmp_path / "ck.bin"
    a.save_checkpoint(path)
    info = v.checkpoint_info(path)
    assert info["has_opt"] and info["step"] == 2
    assert np.allclose(info["adamw"], [HP["beta1"], HP["beta2"], HP["eps"], HP["weight_decay"]])
    pa = a.params(); ma, va, ta = a.adamw_state()
    b = v.ViT.build(cfg, B, v.VIT_BF16)
    b.load_checkpoint(path)
    pb = b.params(); mb, vb, tb = b.adamw_state()
    assert np.array_equal(pa, pb) and np.array_equal(ma, mb) and np.array_equal(va, vb) and ta == tb == 2
    b.set_batch(px, lab)
    la, lb = a.forward(), b.forward()  # the bf16 shadow was refreshed by the load
    assert abs(la - lb) <= 1e-6 * abs(la)
    for m in (a, b):
        m.zero_grad(); m.forward(); m.backward(); m.optimizer_step_adamw(1e-3, **HP)
    assert rel_err(b.params(), a.params()) <= 1e-5
    assert b.adamw_state()[2] == 3
    # a parameters-only file written by the host API loads into a trainer too
    v.write_checkpoint(tmp_path / "p.bin", cfg, params)
    b.load_checkpoint(tmp_path / "p.bin")
    assert np.array_equal(b.params(), params)
    a.close(); b.close()


@pytest.mark.parametrize("prec_name", ["fp32", "bf16"])
def test_u8_input_pipeline_matches_host_normalisation(gpu, tmp_path, prec_name):
    """Loader (pinned ring) -> vit_trainer_set_batch_u8 (async upload + device normalise) gives
    the same logits / loss as uploading the numpy-normalised fp32 batch (bit-identical pixels)."""
    v = gpu
    cfg = v.data.CONFIGS["test_h64"]
    prec = v.VIT_FP32 if prec_name == "fp32" else v.VIT_BF16
    B, n = 4, 19
    rng = np.random.default_rng(3)
    imgs = rng.integers(0, 256, size=(n, cfg.img, cfg.img, 3), dtype=np.uint8)
    labs = rng.integers(0, cfg.num_classes, size=n, dtype=np.int32)
    imgs.tofile(tmp_path / "i.u8")
    labs.tofile(tmp_path / "l.i32")
    ld = v.Loader(tmp_path / "i.u8", tmp_path / "l.i32", cfg.img, B, seed=5, pinned=True)
    params = v.data.init_params(cfg, "parity", seed=4)
    a = v.ViT.build(cfg, B, prec, params=params)
    b = v.ViT.build(cfg, B, prec, params=params)
    for seq in range(6):  # past the 2-slot device staging ring and into epoch 2
        ip, lp, ep, st = ld.next_raw()
        ids, _, _ = v.data.loader_batch_records(n, B, 1, 0, 5, seq)
        a.set_batch_u8(ip, lp)
        la = a.forward()
        px = v.data.normalize_u8(imgs[ids], v.IMAGENET_MEAN, v.IMAGENET_STD)
        lb = b.forward(px, labs[ids])
        assert la == lb, (seq, la, lb)
        assert np.array_equal(a.logits(), b.logits())
    # forward-only u8 batch
    a.set_batch_u8(imgs[:B])
    assert a.forward() == -1.0
    ld.close(); a.close(); b.close()
