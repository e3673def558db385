"""Debug: variant-9 weight-gradient GEMM (M/N-contiguous operands) vs numpy; prints the wrong region."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402

L = vit.lib()
assert L.vit_init(0) == 0
L.gemm_bf16_set_variant(9)
for (M, N, K) in [(512, 512, 128), (512, 512, 256), (304, 520, 128), (256, 256, 128), (768, 3072, 50432 // 8)]:
    rng = np.random.default_rng(1)
    a = rng.normal(size=(M, K)).astype(np.float32)
    b = rng.normal(size=(K, N)).astype(np.float32)
    ab, bb = vit.bf16_bits(a), vit.bf16_bits(b)
    ar = vit.bf16_to_f32(ab).reshape(M, K).astype(np.float64)
    br = vit.bf16_to_f32(bb).reshape(K, N).astype(np.float64)
    A = vit.DeviceArray.from_numpy(np.ascontiguousarray(ab.reshape(M, K).T), np.uint16)
    B = vit.DeviceArray.from_numpy(np.ascontiguousarray(bb.reshape(K, N)), np.uint16)
    out = vit.DeviceArray.zeros(M * N, np.float32)
    vit.call("gemm_bf16_ex", out, N, A, M, 0, B, N, 0, None, None, M, N, K, 2, 0)
    got = out.numpy().reshape(M, N)
    ref = ar @ br
    bad = np.abs(got - ref) > 1e-3 * np.abs(ref).max()
    print(M, N, K, "bad", int(bad.sum()), "of", M * N, flush=True)
    if bad.any():
        r, c = np.nonzero(bad)
        print("  rows", r.min(), r.max(), "cols", c.min(), c.max(), "bad rows", np.unique(r)[:20], "bad cols", np.unique(c)[:20])
        print("  row-blocks of 16 bad:", np.unique(r // 16)[:40], "col-blocks of 16 bad:", np.unique(c // 16)[:40])
