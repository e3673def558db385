// ln_common.h — the LayerNorm forward row arithmetic (train_vit.rs:453-480: two-pass mean /
// biased variance, eps 1e-5) shared by ln_fwd_vec_k (ops.hip) and the fused LayerNorm -> MX
// quantizer ln_fwd_mx_k (gemm_fp8.hip), so the two produce the same bf16 values bit for bit.
#pragma once
#include "common.h"

namespace vit {
// one wave per row, C = 256 NV: lane holds the float4s lane + 64 j of the row (v); the row's mean
// and rstd, then each float4's normalised, affine-transformed values (ln_vec_y, weight / bias float4s
// at the same position)
template <int NV>
__device__ __forceinline__ void ln_vec_stats(const float4 (&v)[NV], int C, float& mean, float& rstd) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NV; j++) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
    const float m = warp_sum(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NV; j++) {
        const float a = v[j].x - m, bb = v[j].y - m, c = v[j].z - m, d = v[j].w - m;
        q += (a * a + bb * bb) + (c * c + d * d);
    }
    mean = m;
    rstd = 1.0f / sqrtf(warp_sum(q) / (float)C + 1e-5f);
}
__device__ __forceinline__ float4 ln_vec_y(float4 v, float4 w4, float4 b4, float m, float r) {
    return make_float4((r * (v.x - m)) * w4.x + b4.x, (r * (v.y - m)) * w4.y + b4.y,
                       (r * (v.z - m)) * w4.z + b4.z, (r * (v.w - m)) * w4.w + b4.w);
}
}  // namespace vit
