"""Seeded JPEG test files, encoded by Pillow (libjpeg-turbo) in this process (test infrastructure).

Images are smooth colour fields plus Gaussian noise (realistic coefficient statistics), in every
variant the decoder supports: 4:4:4 / 4:2:2 / 4:2:0 / grayscale, odd sizes, qualities 50-100,
optimised Huffman tables, restart intervals."""
import io

import numpy as np
from PIL import Image

# (height, width, subsampling (-1 = grayscale), quality, extra save options)
VARIANTS = [
    (61, 97, 0, 90, {}),
    (61, 97, 1, 90, {}),
    (61, 97, 2, 90, {}),
    (224, 224, 2, 75, {"optimize": True}),
    (33, 17, 2, 100, {}),
    (40, 52, -1, 85, {}),
    (64, 80, 2, 90, {"restart_marker_blocks": 3}),
    (123, 200, 1, 50, {"restart_marker_rows": 1}),
    (16, 16, 0, 95, {}),
    (9, 3, 2, 90, {}),
]


def pixels(h, w, gray, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    ph = rng.uniform(0, 6, size=3)
    base = np.stack([np.sin(x / (5.0 + 3 * c) + ph[c]) * 60 + np.cos(y / (4.0 + 2 * c) - ph[c]) * 50 + 128
                     for c in range(3)], -1) + rng.normal(0, 20, (h, w, 3))
    a = np.clip(base, 0, 255).astype(np.uint8)
    return Image.fromarray(a[..., 0] if gray else a, "L" if gray else "RGB")


def encode(h, w, ss, q, kw, seed=0):
    b = io.BytesIO()
    opts = dict(kw)
    if ss >= 0:
        opts["subsampling"] = ss
    pixels(h, w, ss < 0, seed).save(b, format="JPEG", quality=q, **opts)
    return b.getvalue()


def pil_rgb(data):
    return np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))


def dataset(n, seed=0, sizes=((224, 224), (256, 320), (375, 500), (300, 240))):
    """n seeded JPEGs of mixed sizes / subsampling (a small ImageNet-like set) and labels."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        h, w = sizes[i % len(sizes)]
        ss = [2, 2, 1, 0, -1][i % 5]
        out.append(encode(h, w, ss, int(rng.integers(60, 96)), {}, seed=seed * 1000 + i))
    return out, rng.integers(0, 1000, size=n).astype(np.int32)
