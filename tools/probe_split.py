"""Does splitting a heavy-epilogue GEMM into two launches on two streams overlap one half's
epilogue stores with the other half's main loop?  fc fwd (GELU pair) and fcproj dgrad (GELU' +
colsum) at ViT-B/16 B=256, whole vs two M-halves / N-halves on two HIP streams (torch streams,
HIP events)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402


def main():
    L = vit.lib()
    assert L.vit_init(0) == 0
    C, BT = 768, 256 * 197
    rng = np.random.default_rng(0)

    def dev_bf16(n):
        return vit.DeviceArray.from_numpy(vit.bf16_bits(rng.uniform(-1, 1, size=n).astype(np.float32)), np.uint16)

    act, wts, aux16 = dev_bf16(BT * 4 * C), dev_bf16(4 * C * C), dev_bf16(BT * 4 * C)
    out2, out = vit.DeviceArray.zeros(BT * 4 * C, np.uint16), vit.DeviceArray.zeros(BT * 4 * C, np.uint16)
    bias = vit.DeviceArray.from_numpy(rng.uniform(-1, 1, size=4 * C).astype(np.float32))
    csum = vit.DeviceArray.zeros(4 * C, np.float32)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def gemm(epi, m0, m1, n0, n1):
        M, N, K = m1 - m0, n1 - n0, C
        # C/aux rows of ld 4C; B = weight rows n0..n1 (K-contiguous, ld K)
        L.gemm_bf16_fused(out2.ptr + (m0 * 4 * C + n0) * 2, out.ptr + (m0 * 4 * C + n0) * 2 if epi == 4 else None,
                          4 * C, aux16.ptr + (m0 * 4 * C + n0) * 2 if epi == 6 else None, 4 * C,
                          act.ptr + m0 * C * 2, C, 1, wts.ptr + n0 * C * 2, C, 1,
                          bias.ptr + n0 * 4 if epi == 4 else None, csum.ptr + n0 * 4 if epi == 6 else None,
                          M, N, K, epi)

    def whole(epi):
        L.vit_set_stream(ctypes_ptr(main_s))
        gemm(epi, 0, BT, 0, 4 * C)

    def split(epi, axis):
        ev = torch.cuda.Event()
        ev.record(main_s)
        s1.wait_event(ev)
        s2.wait_event(ev)
        mh = (BT // 2 + 255) // 256 * 256
        for k, st in enumerate((s1, s2)):
            L.vit_set_stream(ctypes_ptr(st))
            if axis == "m":
                gemm(epi, 0 if k == 0 else mh, mh if k == 0 else BT, 0, 4 * C)
            else:
                gemm(epi, 0, BT, 0 if k == 0 else 2 * C, 2 * C if k == 0 else 4 * C)
        for st in (s1, s2):
            e = torch.cuda.Event()
            e.record(st)
            main_s.wait_event(e)
        L.vit_set_stream(ctypes_ptr(main_s))

    def ctypes_ptr(st):
        return st.cuda_stream

    for epi, name in ((4, "fc fwd GELU pair"), (6, "fcproj dgrad GELU'")):
        for label, fn in (("whole", lambda: whole(epi)), ("2 M-halves / 2 streams", lambda: split(epi, "m")),
                          ("2 N-halves / 2 streams", lambda: split(epi, "n"))):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(main_s)
                for _ in range(5):
                    fn()
                e1.record(main_s)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 5)
            vit.check(label)
            print(f"{name:22s} {label:26s} {sorted(ts)[2] * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
