"""JPEG input pipeline throughput (include/vit_jpeg.h) on the GPU box.

  python tools/bench_jpeg.py [--n 512] [--batch 256] [--threads 4,8,14] [--steps 8] [--train]

1. makes n ImageNet-like JPEGs (500x375 / 375x500 / 640x480 / 333x500, 4:2:0 mostly, quality
   75-95, smooth colour fields + noise; Pillow), packs them as loader records under /tmp;
2. per thread count: loader.next() + decode_u8(224) (random-resized crops + flips, the training
   policy) over `steps` batches -> images/s of the whole feed (host entropy decode ahead on
   `threads` threads, upload + GPU kernels on the stream);
3. the GPU half alone (decode_u8 of one resident batch, repeated) -> images/s and us per batch;
4. --train: ViT-B/16 bf16 B=256 train steps fed by vit_trainer_set_batch_jpeg each step.
Prints one JSON object."""
import argparse
import io
import json
import os
import sys
import time

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vitpkg import vit  # noqa: E402


def make_jpegs(n, seed=0):
    rng = np.random.default_rng(seed)
    sizes = [(375, 500), (500, 375), (480, 640), (500, 333)]
    out = []
    for i in range(n):
        h, w = sizes[i % 4]
        y, x = np.mgrid[0:h, 0:w]
        ph = rng.uniform(0, 6, 3)
        base = np.stack([np.sin(x / (11.0 + 5 * c) + ph[c]) * 70 + np.cos(y / (9.0 + 3 * c) - ph[c]) * 50 + 128
                         for c in range(3)], -1) + rng.normal(0, 12, (h, w, 3))
        b = io.BytesIO()
        Image.fromarray(np.clip(base, 0, 255).astype(np.uint8)).save(
            b, format="JPEG", quality=int(rng.integers(75, 96)), subsampling=2 if i % 8 else 1)
        out.append(b.getvalue())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--threads", default="4,8,14")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--train", action="store_true")
    a = ap.parse_args()
    assert vit.lib().vit_init(0) == 0
    t0 = time.time()
    jpegs = make_jpegs(a.n)
    labels = np.arange(a.n, dtype=np.int32) % 1000
    prefix = f"/tmp/bench_jpeg_{os.getpid()}"
    paths = vit.write_jpeg_records(prefix, jpegs, labels)
    res = {"records": a.n, "mean_jpeg_bytes": float(np.mean([len(j) for j in jpegs])),
           "make_s": round(time.time() - t0, 1), "batch": a.batch, "img": 224, "feed": {}}
    out = vit.DeviceArray((a.batch, 224, 224, 3), np.uint8)
    for th in [int(t) for t in a.threads.split(",")]:
        L = vit.JpegLoader(*paths, batch=a.batch, seed=1, shuffle=True, augment=True, depth=3, threads=th)
        L.next()
        L.decode_u8(224, out)
        vit.lib().vit_sync()
        t = time.perf_counter()
        for _ in range(a.steps):
            L.next()
            L.decode_u8(224, out)
        vit.lib().vit_sync()
        dt = time.perf_counter() - t
        res["feed"][th] = round(a.steps * a.batch / dt, 1)
        print(f"threads {th}: {res['feed'][th]} img/s", file=sys.stderr, flush=True)
        if th == int(a.threads.split(",")[-1]):
            # GPU half alone: the same resident host batch decoded repeatedly
            reps = 20
            vit.lib().vit_sync()
            t = time.perf_counter()
            for _ in range(reps):
                L.decode_u8(224, out)
            vit.lib().vit_sync()
            dt = time.perf_counter() - t
            res["gpu_half_img_s"] = round(reps * a.batch / dt, 1)
            res["gpu_half_ms_per_batch"] = round(dt / reps * 1e3, 3)
        L.close()
    if a.train:
        cfg = vit.data.CONFIGS["vit_b16"]
        m = vit.ViT.build(cfg, a.batch, vit.VIT_BF16, params=vit.data.init_params(cfg, "ref", seed=1))
        th = int(a.threads.split(",")[-1])
        L = vit.JpegLoader(*paths, batch=a.batch, seed=1, shuffle=True, augment=True, depth=3, threads=th)
        for i in range(a.steps + 2):
            if i == 2:
                m.sync()
                t = time.perf_counter()
            L.next()
            m.set_batch_jpeg(L)
            m.train_step(1e-4)
        m.sync()
        dt = time.perf_counter() - t
        res["train_fed_img_s"] = round(a.steps * a.batch / dt, 1)
        res["train_threads"] = th
        L.close()
        m.close()
    for p in paths:
        os.remove(p)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
