"""Model configurations, canonical parameter layout and seeded synthetic inputs.

The reference builds its config from a checkpoint header (train_vit.rs:89-131) and initialises
parameters with an unseeded `rand` (train_vit.rs:674-713).  Here configs are a static table and
every random stream is a counter-based splitmix64 (seed 1337 by default) so the GPU path, the CPU
oracle and every rank of a data-parallel job see bit-identical inputs.
"""
from dataclasses import dataclass

import numpy as np

PARAM_NAMES = ["patch_w", "patch_b", "cls", "wpe",
               "ln1w", "ln1b", "qkvw", "qkvb", "attprojw", "attprojb",
               "ln2w", "ln2b", "fcw", "fcb", "fcprojw", "fcprojb",
               "lnfw", "lnfb", "head_w", "head_b"]
LAYER_PARAMS = PARAM_NAMES[4:16]


@dataclass(frozen=True)
class VitCfg:
    name: str
    img: int
    patch: int
    channels: int
    num_layers: int
    num_heads: int
    num_classes: int
    in_ch: int = 3

    @property
    def num_patches(self):
        return (self.img // self.patch) ** 2

    @property
    def T(self):
        return self.num_patches + 1

    @property
    def head_size(self):
        return self.channels // self.num_heads

    def param_sizes(self):
        """Canonical (reference type-major) order; train_vit.rs:115-131 with ViT tensors."""
        C, L, P, T, NC = self.channels, self.num_layers, self.patch, self.T, self.num_classes
        K = self.in_ch * P * P
        return [C * K, C, C, T * C,
                L * C, L * C, L * 3 * C * C, L * 3 * C, L * C * C, L * C,
                L * C, L * C, L * 4 * C * C, L * 4 * C, L * C * 4 * C, L * C,
                C, C, NC * C, NC]

    def num_params(self):
        return int(sum(self.param_sizes()))

    def train_gflop_per_image(self):
        """Algorithmic train-step GFLOP per image: 2*M*N*K per GEMM, forward +
        dgrad + wgrad (patch embed: no pixel dgrad), attention 4*T^2*C per layer forward x3."""
        C, L, T, NP = self.channels, self.num_layers, self.T, self.num_patches
        K = self.in_ch * self.patch ** 2
        per_layer = 2 * T * C * (3 * C + C + 4 * C + 4 * C) + 4 * T * T * C
        fwd = L * per_layer + 2 * NP * K * C + 2 * C * self.num_classes
        train = 3 * L * per_layer + 2 * 2 * NP * K * C + 3 * 2 * C * self.num_classes
        return fwd / 1e9, train / 1e9

    def split(self, flat):
        out, off = {}, 0
        for n, s in zip(PARAM_NAMES, self.param_sizes()):
            out[n] = flat[off:off + s]
            off += s
        return out


CONFIGS = {
    # tiny fixture shape
    "test": VitCfg("test", img=32, patch=8, channels=32, num_layers=2, num_heads=2, num_classes=10),
    "test_t10": VitCfg("test_t10", img=48, patch=16, channels=64, num_layers=1, num_heads=1,
                       num_classes=7),
    # head size 64 (the fused bf16 attention's shape) at fixture scale
    "test_h64": VitCfg("test_h64", img=32, patch=8, channels=128, num_layers=2, num_heads=2,
                       num_classes=10),
    # BASELINE.json configs
    "vit_tiny16": VitCfg("vit_tiny16", img=224, patch=16, channels=192, num_layers=12,
                         num_heads=3, num_classes=1000),
    "vit_b16": VitCfg("vit_b16", img=224, patch=16, channels=768, num_layers=12, num_heads=12,
                      num_classes=1000),
    "vit_l16": VitCfg("vit_l16", img=224, patch=16, channels=1024, num_layers=24, num_heads=16,
                      num_classes=1000),
    "vit_h14": VitCfg("vit_h14", img=224, patch=14, channels=1280, num_layers=32, num_heads=16,
                      num_classes=1000),
}

_GOLD = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed, n, offset=0):
    """n outputs of splitmix64(seed) starting at stream position `offset` (counter form:
    output i = mix(seed + (i+1)*golden))."""
    with np.errstate(over="ignore"):
        idx = np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * _GOLD
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform(seed, n, offset=0):
    """U[0,1) float64 from the top 53 bits."""
    return (splitmix64(seed, n, offset) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def normal(seed, n, offset=0):
    """N(0,1) via Box-Muller on consecutive uniform pairs."""
    assert offset % 2 == 0, "normal streams are consumed in Box-Muller pairs"
    m = (n + 1) // 2
    u = uniform(seed, 2 * m, offset)
    u1 = np.maximum(u[0::2], 1e-300)
    u2 = u[1::2]
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.concatenate([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)])
    out = np.empty(2 * m)
    out[0::2] = z[:m]
    out[1::2] = z[m:]
    return out[:n]


def init_params(cfg, mode="parity", seed=1337):
    """Flat canonical fp32 arena.
    mode "ref":    the reference's init (train_vit.rs:674-713): weights U[0,1)*0.02, LN gains 1,
                   biases / LN betas 0 (left unset by the reference, D12).
    mode "parity": weights N(0,0.02), gains 1+N(0,0.1), biases N(0,0.02) so every gradient
                   path is non-degenerate."""
    flat = np.empty(cfg.num_params(), dtype=np.float32)
    views = cfg.split(flat)
    for ti, (name, v) in enumerate(views.items()):
        s = seed * 1000 + ti
        is_gain = name in ("ln1w", "ln2w", "lnfw")
        is_bias = name in ("patch_b", "ln1b", "ln2b", "qkvb", "attprojb", "fcb", "fcprojb",
                           "lnfb", "head_b")
        if mode == "ref":
            if is_gain:
                v[:] = 1.0
            elif is_bias:
                v[:] = 0.0
            else:
                v[:] = uniform(s, v.size) * 0.02
        else:
            if is_gain:
                v[:] = 1.0 + 0.1 * normal(s, v.size)
            else:
                v[:] = 0.02 * normal(s, v.size)
    return flat


def synthetic_batch(cfg, B, seed=1337, offset_images=0):
    """Pixels [B,3,IMG,IMG] ~ N(0,1) and labels uniform in [0, NCLS), images
    [offset_images, offset_images+B) of one seeded stream (so DP ranks take disjoint slices)."""
    per_img = cfg.in_ch * cfg.img * cfg.img
    px = normal(seed, B * per_img, offset_images * per_img).astype(np.float32)
    lab = (splitmix64(seed + 7, B, offset_images) % np.uint64(cfg.num_classes)).astype(np.int32)
    return px.reshape(B, cfg.in_ch, cfg.img, cfg.img), lab


# ------------------------------------------------------------------ input pipeline mirrors
def epoch_permutation(n, seed, epoch, shuffle=True):
    """The loader's per-epoch record order (include/vit_data.h): Fisher-Yates, i = n-1 .. 1,
    swap(i, r mod (i+1)) with r the splitmix64 stream of seed + epoch at position n-1-i."""
    perm = np.arange(n, dtype=np.int64)
    if not shuffle or n < 2:
        return perm
    r = splitmix64((seed + epoch) & 0xFFFFFFFFFFFFFFFF, n - 1)
    for i in range(n - 1, 0, -1):
        j = int(r[n - 1 - i] % np.uint64(i + 1))
        perm[i], perm[j] = perm[j], perm[i]
    return perm


def loader_batch_records(n, batch, world, rank, seed, seq, shuffle=True):
    """Record ids of the loader's batch number `seq` (epochs run back to back) for `rank`."""
    steps = n // (batch * world)
    epoch, step = divmod(seq, steps)
    perm = epoch_permutation(n, seed, epoch, shuffle)
    base = (step * world + rank) * batch
    return perm[base:base + batch], epoch, step


def normalize_u8(images, mean, std):
    """uint8 [B, H, W, 3] -> fp32 [B, 3, H, W]: (x / 255 - mean[c]) / std[c] in fp32."""
    x = np.asarray(images, np.uint8).astype(np.float32) / np.float32(255)
    x = (x - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return np.ascontiguousarray(x.transpose(0, 3, 1, 2))
