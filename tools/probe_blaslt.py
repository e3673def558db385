"""Library-GEMM reference points (torch.matmul -> hipBLASLt on ROCm) for the trainer's ViT-B/16
B=256 GEMM shapes, bf16 in/out, fp32 accumulate: what a plain library GEMM reaches on the box,
next to tools/bench_gemm.py's numbers for the fused engine.  Timing: CUDA events, median of 5."""
import torch

M = 256 * 197
C = 768
shapes = [  # name, (m, n, k), a transposed, b transposed  (C[m,n] = A[m,k] B[k,n])
    ("fwd_qkv", (M, 3 * C, C)), ("fwd_proj", (M, C, C)), ("fwd_fc", (M, 4 * C, C)), ("fwd_fcproj", (M, C, 4 * C)),
    ("dgrad_fc", (M, C, 4 * C)), ("dgrad_qkv", (M, C, 3 * C)),
    ("wgrad_fcproj", (C, 4 * C, M)), ("wgrad_fc", (4 * C, C, M)), ("wgrad_proj", (C, C, M)), ("wgrad_qkv", (3 * C, C, M)),
]
dev = "cuda"
for name, (m, n, k) in shapes:
    if name.startswith("wgrad"):  # dW = dY^T X: both operands token-major (MN-contiguous)
        a = torch.randn(k, m, device=dev, dtype=torch.bfloat16).t()
        b = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
    else:  # activations K-contiguous, weights [n][k] (K-contiguous) as in the trainer
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        b = torch.randn(n, k, device=dev, dtype=torch.bfloat16).t()
    for _ in range(3):
        c = a @ b
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            c = a @ b
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 5)
    ms = sorted(ts)[2]
    print(f"{name:14s} {m:6d} {n:6d} {k:6d}  {ms * 1e3:8.1f} us  {2 * m * n * k / ms / 1e9:7.0f} TF/s", flush=True)
