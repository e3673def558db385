"""Generate the committed golden fixtures (run in the build container, CPU only).

For each tiny config it
  1. builds seeded parity-init params, pixels and labels (vit.rs_amd/data.py),
  2. runs an INDEPENDENT torch-CPU fp64 autograd ViT (written from the model definition, not
     from the oracle) to get logits, mean loss and every parameter gradient,
  3. checks the fp64 oracle (oracle/liboracle_f64.so) against it to ~1e-10 and the fp32 oracle
     to ~1e-4, and
  4. writes tests/golden/<cfg>.npz (inputs + torch fp64 outputs; no pickles).

torch is only an independent cross-check here; it is never needed on the GPU box.
    python tests/golden/make_golden.py
"""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def load_data_module():
    spec = importlib.util.spec_from_file_location("vit_data", os.path.join(ROOT, "vit.rs_amd", "data.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def torch_vit(cfg, flat, pixels, labels):
    """fp64 autograd ViT: patch-embed (conv as unfold+linear), CLS + pos, L pre-LN blocks with
    non-causal MHA and tanh-GELU MLP, final LN + head on CLS, mean cross-entropy."""
    import torch
    import torch.nn.functional as F
    D = load_data_module()
    t = {n: torch.tensor(v.astype(np.float64), requires_grad=True)
         for n, v in cfg.split(flat).items()}
    B, C, L, NH, T = pixels.shape[0], cfg.channels, cfg.num_layers, cfg.num_heads, cfg.T
    hs = C // NH
    x = torch.tensor(pixels.astype(np.float64))
    patches = F.unfold(x, kernel_size=cfg.patch, stride=cfg.patch).transpose(1, 2)  # [B,NP,3PP]
    emb = patches @ t["patch_w"].view(C, -1).T + t["patch_b"]
    cls = t["cls"].view(1, 1, C).expand(B, 1, C)
    h = torch.cat([cls, emb], dim=1) + t["wpe"].view(T, C)
    for l in range(L):
        g = lambda n, *shape: t[n].view(L, *shape)[l]
        a = F.layer_norm(h, (C,), g("ln1w", C), g("ln1b", C), eps=1e-5)
        qkv = a @ g("qkvw", 3 * C, C).T + g("qkvb", 3 * C)
        q, k, v = qkv.split(C, dim=2)
        q = q.view(B, T, NH, hs).transpose(1, 2)
        k = k.view(B, T, NH, hs).transpose(1, 2)
        v = v.view(B, T, NH, hs).transpose(1, 2)
        att = torch.softmax(q @ k.transpose(-1, -2) / np.sqrt(hs), dim=-1)
        y = (att @ v).transpose(1, 2).reshape(B, T, C)
        h = h + y @ g("attprojw", C, C).T + g("attprojb", C)
        a = F.layer_norm(h, (C,), g("ln2w", C), g("ln2b", C), eps=1e-5)
        f = F.gelu(a @ g("fcw", 4 * C, C).T + g("fcb", 4 * C), approximate="tanh")
        h = h + f @ g("fcprojw", C, 4 * C).T + g("fcprojb", C)
    z = F.layer_norm(h[:, 0], (C,), t["lnfw"], t["lnfb"], eps=1e-5)
    logits = z @ t["head_w"].view(cfg.num_classes, C).T + t["head_b"]
    loss = F.cross_entropy(logits, torch.tensor(labels.astype(np.int64)))
    loss.backward()
    grads = np.concatenate([t[n].grad.numpy().ravel() for n in D.PARAM_NAMES])
    return logits.detach().numpy(), float(loss.detach()), grads


def oracle_run(prec, cfg, flat, pixels, labels):
    import oracle_ctypes as oc
    o = oc.Oracle(prec)
    c = oc.VitConfig(cfg.img, cfg.patch, cfg.in_ch, cfg.channels, cfg.num_layers,
                     cfg.num_heads, cfg.num_classes)
    m = oc.RefViT(o, c, pixels.shape[0])
    p = o.arr(flat)
    loss = m.forward(p, pixels, labels)
    g = np.zeros_like(p)
    m.backward(p, g)
    return m.logits(), loss, g


def main():
    D = load_data_module()
    out_dir = os.path.dirname(os.path.abspath(__file__))
    for name, B in (("test", 2), ("test_t10", 3)):
        cfg = D.CONFIGS[name]
        flat = D.init_params(cfg, "parity", seed=7)
        px, lab = D.synthetic_batch(cfg, B, seed=11)
        lt, losst, gt = torch_vit(cfg, flat, px, lab)
        for prec, tol in (("f64", 1e-10), ("f32", 2e-4)):
            lo, losso, go = oracle_run(prec, cfg, flat, px, lab)
            e_l = np.abs(lo - lt).max() / np.abs(lt).max()
            e_g = np.abs(go - gt).max() / np.abs(gt).max()
            e_loss = abs(losso - losst) / abs(losst)
            print(f"{name} oracle {prec} vs torch fp64: logits {e_l:.2e} loss {e_loss:.2e} grads {e_g:.2e}")
            assert max(e_l, e_g, e_loss) < tol, (name, prec)
        np.savez(os.path.join(out_dir, f"{name}.npz"), params=flat, pixels=px, labels=lab,
                 logits=lt, loss=np.float64(losst), grads=gt)
        print("wrote", name)


if __name__ == "__main__":
    main()
