"""Oracle fixtures for the gradient parity of the production step at the BENCHMARKED GEMM shapes
(tests/test_gpu_benchshape.py).

The fp32 CPU oracle (oracle/oracle.c: the reference loops of /root/reference/train_vit.rs:188-373,
forward :188-268, backward :271-373, matmul_backward :530-557) runs the full train-step forward and
backward at the benchmarked per-GPU batch, for three geometries whose every GEMM has the exact shape
the bench times:

  b16: ViT-B/16 width (C=768, NH=12, T=197), L=2, B=256   -> M = 50,432 (two micro-batches of 25,216),
       N in {768, 2304, 3072}, wgrad reduction length 50,432 (25,216 per micro-batch)
  l16: ViT-L/16 width (C=1024, NH=16, T=197), L=1, B=256
  h14: ViT-H/14 width (C=1280, NH=16, T=257, patch 14), L=1, B=128 (config 5's shard; run on the GPU
       in bf16 and in fp8)

Its inputs are the seeded streams of vit.rs_amd/data.py (init_params(cfg, "parity", seed),
synthetic_batch(cfg, B, seed + 1): splitmix64, platform independent), so the GPU test regenerates
them exactly.  A full-size oracle step takes 6-8 CPU-minutes per geometry on 8 cores, too long for
the GPU suite, so it runs HERE once and this script commits what the test compares:
  * the mean loss and all B per-image losses;
  * for the logits and each of the 20 gradient tensors: the values at SAMPLES seeded positions
    (`sample_index`: every element of a tensor with fewer elements), plus the tensor's full
    max |ref| and rms (the normalisers of tests/parity.py's max-normalised and rms errors).
Usage (repo root, ~20 min): python3 tests/golden/make_benchshape.py [b16 l16 h14]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

SAMPLES = 16384
# name -> (img, patch, C, L, NH, B, seed)
GEOMS = {
    "b16": (224, 16, 768, 2, 12, 256, 71),
    "l16": (224, 16, 1024, 1, 16, 256, 73),
    "h14": (224, 14, 1280, 1, 16, 128, 75),
}


def cfg_of(data, name):
    img, patch, C, L, NH, _, _ = GEOMS[name]
    return data.VitCfg(f"bench_{name}", img=img, patch=patch, channels=C, num_layers=L, num_heads=NH,
                       num_classes=1000)


def inputs(data, name):
    cfg = cfg_of(data, name)
    B, seed = GEOMS[name][5], GEOMS[name][6]
    params = data.init_params(cfg, "parity", seed=seed)
    px, lab = data.synthetic_batch(cfg, B, seed=seed + 1)
    return cfg, params, px, lab


def sample_index(n, key, samples=SAMPLES):
    """Sorted seeded positions of a tensor of n elements (all of them when n <= samples)."""
    if n <= samples:
        return np.arange(n)
    seed = sum(ord(c) * 131 ** i for i, c in enumerate(key)) % (2 ** 32)
    return np.sort(np.random.default_rng(seed).choice(n, size=samples, replace=False))


def tensors(cfg, logits, grads):
    """name -> flat array: the logits and the 20 gradient tensors (canonical order)."""
    out = {"logits": np.asarray(logits).ravel()}
    out.update({n: np.asarray(a).ravel() for n, a in cfg.split(grads).items()})
    return out


def make(name, out_dir):
    import oracle_ctypes as oc
    from vitpkg import vit
    cfg, params, px, lab = inputs(vit.data, name)
    B = px.shape[0]
    o = oc.Oracle("f32")
    o.set_num_threads(os.cpu_count())
    c = oc.VitConfig(cfg.img, cfg.patch, cfg.in_ch, cfg.channels, cfg.num_layers, cfg.num_heads, cfg.num_classes)
    t0 = time.time()
    m = oc.RefViT(o, c, B)
    p = o.arr(params)
    loss = m.forward(p, px, lab)
    g = np.zeros_like(p)
    m.backward(p, g)
    rec = {"loss": np.float64(loss), "losses": m.losses().astype(np.float32).copy()}
    for key, a in tensors(cfg, m.logits().copy(), g).items():
        idx = sample_index(a.size, f"{name}.{key}")
        a64 = a.astype(np.float64)
        rec[f"{key}.val"] = a[idx].astype(np.float32)
        rec[f"{key}.absmax"] = np.float64(np.abs(a64).max())
        rec[f"{key}.rms"] = np.float64(np.sqrt(np.mean(a64 * a64)))
        rec[f"{key}.n"] = np.int64(a.size)
    path = os.path.join(out_dir, f"benchshape_{name}.npz")
    np.savez_compressed(path, **rec)
    print(f"{name}: B={B} loss {loss:.6f}  {time.time() - t0:.0f} s -> {path}", flush=True)


if __name__ == "__main__":
    names = sys.argv[1:] or list(GEOMS)
    for n in names:
        make(n, os.path.dirname(os.path.abspath(__file__)))
