"""Per-wave phase timelines of the attention backward kernels from s_memtime stamps (shader cycles).
Needs a library built with -DVIT_ATTN_DIAG=4 (attn_fused.h), selected with VIT_LIB:
    VIT_LIB=vit.rs_amd/build_diag4/libvit_hip.so python tools/attn_trace.py            # ViT-B/16, attn_bwdp_k
    VIT_LIB=... python tools/attn_trace.py --batch 128 --T 257 --NH 16 --hs 80          # ViT-H/14, attn_bwd1_k
Blocks 0..7 stamp; 16 records of 16 stamps per wave.
attn_bwdp_k (persistent): record = global slice; 0 slice start, 1 after phase A, 2 after phase B,
  3 after put_slice, 4 after the barrier, 5 after put_side; item end in the next item's first record:
  6 after the last phase B + barrier, 8 after the dK / dV stores, 9 after the column sums, 10 after
  the partial-row stores, 7 after bwd_item_end.
attn_bwd1_k (one workgroup per item): record = slice; 0 start, 1 after phase A, 2 after the last-key
  side path + barrier, 3 after put_slice, 4 after phase B, 5 after the barrier; record 15: 0 kernel
  start, 1 after the prologue, 6 loop end, 8 / 9 / 10 / 7 as above."""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit  # noqa: E402


def show_bwdp(tr):
    nw = int((tr[0, 0, :, 0] != 0).sum())
    tr = tr[:, :, :nw, :]
    names = ["A", "B", "put_slice", "barrier", "put_side", "to next"]
    sl = slice(1, 15)
    print(f"waves per workgroup {nw}; cycles per slice (mean over blocks 0-7, slices 1-14)")
    print("wave " + " ".join(f"{n:>10s}" for n in names) + "      total")
    for w in range(nw):
        d = [np.mean(tr[:, sl, w, k + 1] - tr[:, sl, w, k]) for k in range(5)]
        d.append(np.mean(tr[:, 2:16, w, 0] - tr[:, 1:15, w, 5]))
        tot = np.mean(tr[:, 2:16, w, 0] - tr[:, 1:15, w, 0])
        print(f"{w:4d} " + " ".join(f"{x:10.0f}" for x in d) + f" {tot:10.0f}")
    per = tr[:, 2:16, :, 0] - tr[:, 1:15, :, 0]
    first = np.array([(s % 7) == 0 for s in range(2, 16)])
    b = [s for s in range(1, 15) if s % 7 == 0]
    pb = tr[:, [s - 1 for s in b]][..., 5]
    r = tr[:, b]
    print(f"item end: last B + barrier {(r[..., 6] - pb).mean():.0f}, bwd_item_end {(r[..., 7] - r[..., 6]).mean():.0f}, "
          f"load_kv + next start {(r[..., 0] - r[..., 7]).mean():.0f}")
    print(f"  inside: dK/dV stores {(r[..., 8] - r[..., 6]).mean():.0f}, column sums {(r[..., 9] - r[..., 8]).mean():.0f}, "
          f"partial-row stores {(r[..., 10] - r[..., 9]).mean():.0f}, rest {(r[..., 7] - r[..., 10]).mean():.0f}")
    for s in b:
        ph = [np.mean(tr[:, s, :, k + 1] - tr[:, s, :, k]) for k in range(5)]
        print(f"item-start slice {s}: " + " ".join(f"{n} {x:.0f}" for n, x in zip(names, ph)))
    print(f"slice period, item-start slices {per[:, first].mean():.0f}, others {per[:, ~first].mean():.0f}")


def show_bwd1(tr, nsl):
    nw = int((tr[0, 15, :, 0] != 0).sum())
    tr = tr[:, :, :nw, :]
    k = tr[:, 15]
    print(f"waves per workgroup {nw}, slices {nsl}; cycles (mean over blocks 0-7)")
    print(f"prologue {(k[..., 1] - k[..., 0]).mean():.0f}; loop {(k[..., 6] - k[..., 1]).mean():.0f}; "
          f"item end {(k[..., 7] - k[..., 6]).mean():.0f} (dK/dV stores {(k[..., 8] - k[..., 6]).mean():.0f}, "
          f"dK/dV sums {(k[..., 9] - k[..., 8]).mean():.0f}, dQ sums {(k[..., 10] - k[..., 9]).mean():.0f}); "
          f"kernel {(k[..., 7] - k[..., 0]).mean():.0f}")
    names = ["A", "side+bar", "put", "B", "barrier"]
    print("slice " + " ".join(f"{n:>9s}" for n in names))
    for s in range(min(nsl, 15)):
        d = [np.mean(tr[:, s, :, j + 1] - tr[:, s, :, j]) for j in range(5)]
        print(f"{s:5d} " + " ".join(f"{x:9.0f}" for x in d))
    print("per wave, mean over slices:")
    for w in range(nw):
        d = [np.mean(tr[:, :min(nsl, 15), w, j + 1] - tr[:, :min(nsl, 15), w, j]) for j in range(5)]
        print(f"  w{w} " + " ".join(f"{x:9.0f}" for x in d))


def show_fwd(tr, nqt):
    nw = 4
    k = tr[:, 15, :nw]
    print(f"forward, cycles (mean over blocks 0-7): K/V staging {(k[..., 1] - k[..., 0]).mean():.0f}, "
          f"barrier {(k[..., 2] - k[..., 1]).mean():.0f}, tile loop {(k[..., 3] - k[..., 2]).mean():.0f}, "
          f"workgroup {(k[..., 3] - k[..., 0]).mean():.0f}")
    names = ["S", "softmax", "PV", "store", "to next"]
    print("tile " + " ".join(f"{n:>9s}" for n in names))
    for r in range((nqt + 3) // 4):
        rows = []
        for w in range(nw):
            if w + 4 * r >= nqt:
                continue
            d = [tr[:, r, w, j + 1] - tr[:, r, w, j] for j in range(4)]
            nxt = tr[:, r + 1, w, 0] if w + 4 * (r + 1) < nqt else k[:, w, 3]
            d.append(nxt - tr[:, r, w, 4])
            rows.append([np.mean(x) for x in d])
        print(f"{r:4d} " + " ".join(f"{x:9.0f}" for x in np.mean(rows, axis=0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--T", type=int, default=197)
    ap.add_argument("--NH", type=int, default=12)
    ap.add_argument("--hs", type=int, default=64)
    ap.add_argument("--fwd", action="store_true", help="trace the forward kernel instead")
    args = ap.parse_args()
    B, T, NH, hs = args.batch, args.T, args.NH, args.hs
    C = hs * NH
    L = vit.lib()
    assert L.vit_init(0) == 0
    raw = ctypes.CDLL(os.environ["VIT_LIB"])
    rng = np.random.default_rng(0)
    qkv = vit.DeviceArray.from_numpy(vit.bf16_bits(rng.normal(size=B * T * 3 * C).astype(np.float32)), np.uint16)
    dout = vit.DeviceArray.from_numpy(vit.bf16_bits(rng.normal(size=B * T * C).astype(np.float32)), np.uint16)
    out = vit.DeviceArray.zeros(B * T * C, np.uint16)
    lse = vit.DeviceArray.zeros(B * NH * T, np.float32)
    dqkv = vit.DeviceArray.zeros(B * T * 3 * C, np.uint16)
    dbias = vit.DeviceArray.zeros(3 * C, np.float32)
    for _ in range(3 if args.fwd else 1):
        L.attention_forward_fused_bf16(out.ptr, lse.ptr, qkv.ptr, B, T, C, NH)
    for _ in range(0 if args.fwd else 3):
        L.attention_backward_fused_bf16_ex(dqkv.ptr, dout.ptr, qkv.ptr, out.ptr, lse.ptr, B, T, C, NH, dbias.ptr)
    L.vit_sync()
    tr = np.zeros(8 * 16 * 16 * 16, np.uint64)
    fn = getattr(raw, f"vit_attn_trace_read_h{hs}")
    assert fn(tr.ctypes.data_as(ctypes.c_void_p)) == 0
    tr = tr.reshape(8, 16, 16, 16).astype(np.int64)  # [block][record][wave][stamp]
    if args.fwd:
        show_fwd(tr, (T + 15) // 16)
    elif tr[0, 15, 0, 1] != 0 and tr[0, 15, 0, 6] != 0:
        show_bwd1(tr, (T + 31) // 32)
    else:
        show_bwdp(tr)


if __name__ == "__main__":
    main()
