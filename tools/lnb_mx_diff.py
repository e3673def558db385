"""Diagnostic: where layernorm_backward_stream_mx's bf16 + lo8 planes differ from layernorm_backward_stream."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402


def main():
    v = vit
    assert v.lib().vit_init(0) == 0
    for R, C in ((100, 256), (197, 768), (4001, 1280)):
        rng = np.random.default_rng(R + C)
        x = (rng.normal(size=(R, C)) * 2 + rng.normal(size=(R, 1))).astype(np.float32)
        mu = x.mean(1).astype(np.float32)
        rs = (1.0 / np.sqrt(x.var(1) + 1e-5)).astype(np.float32)
        w = rng.normal(size=C).astype(np.float32)
        dyb = v.bf16_bits(rng.normal(size=(R, C)).astype(np.float32))
        hib = v.bf16_bits(rng.normal(size=(R, C)).astype(np.float32))
        lo = rng.integers(0, 256, size=(R, C), dtype=np.uint8)
        D = lambda a, dt=np.float32: v.DeviceArray.from_numpy(np.ascontiguousarray(a, dtype=dt))
        Z = lambda n, dt=np.float32: v.DeviceArray.zeros(n, dt)
        args = (D(hib, np.uint16), D(lo, np.uint8))
        com = (D(dyb, np.uint16), D(x), D(w), D(mu), D(rs), R, C)
        ho_ref, lo_ref = Z(R * C, np.uint16), Z(R * C, np.uint8)
        v.call("layernorm_backward_stream", ho_ref, lo_ref, *args, Z(C), Z(C), Z(C), *com)
        kp = int(v.lib().mx_cols_padded(R))
        ho, lo8 = Z(R * C, np.uint16), Z(R * C, np.uint8)
        v.call("layernorm_backward_stream_mx", ho, lo8, *args, Z(C), Z(C), Z(C), *com, Z(R * C, np.uint8),
               Z(int(v.lib().mx_scale_size(R, C)), np.uint8), Z(C * kp, np.uint8),
               Z(int(v.lib().mx_scale_size(C, kp)), np.uint8), kp, 0, kp)
        a, b = ho.numpy().reshape(R, C), ho_ref.numpy().reshape(R, C)
        la, lb = lo8.numpy().reshape(R, C), lo_ref.numpy().reshape(R, C)
        bad = np.argwhere((a != b) | (la != lb))
        fa = v.bf16_to_f32(a.ravel()).reshape(R, C)
        fb = v.bf16_to_f32(b.ravel()).reshape(R, C)
        print(f"R={R} C={C}: {len(bad)} of {R * C} differ; rows {np.unique(bad[:, 0])[:10]} "
              f"cols {np.unique(bad[:, 1])[:10]}; hi diff max {np.abs(fa - fb).max():.3e}, "
              f"|ref| max {np.abs(fb).max():.3e}; lo diffs {np.unique((la.astype(int) - lb.astype(int))[la != lb])[:10]}")


if __name__ == "__main__":
    main()
