// ln_common.h — the LayerNorm row arithmetic shared by the vectorised kernels (ops.hip: ln_fwd_vec_k,
// ln_bwd_vec_k) and their fused LayerNorm -> MX forms (gemm_fp8.hip: ln_fwd_mx_k, ln_bwd_mx_k), so both
// produce the same values bit for bit.  Forward: train_vit.rs:453-480 (two-pass mean / biased
// variance, eps 1e-5); backward: train_vit.rs:603-637 (D5).
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
// LayerNorm backward of one row, C = 256 NV, the lane's float4s at lane + 64 j: nr = the normalised
// input (x - mean) * rstd, dv = the input gradient ((w dy - mean(w dy)) - nr mean(w dy nr)) * rstd
// FMA contraction off: which products hipcc fused into the following adds depended on the
// surrounding kernel (ln_bwd_vec_k and ln_bwd_mx_k differed in ~0.1 % of the bf16 outputs), so every
// product here is rounded on its own and both kernels compute the same values
template <int NV>
__device__ __forceinline__ void ln_bwd_row(const float4 (&dy)[NV], const float4 (&x)[NV], const float4 (&w4)[NV],
                                           float mu, float rs, int C, float4 (&nr)[NV], float4 (&dv)[NV]) {
#pragma clang fp contract(off)
    float a = 0.f, bs = 0.f;
#pragma unroll
    for (int j = 0; j < NV; j++) {
        nr[j] = make_float4((x[j].x - mu) * rs, (x[j].y - mu) * rs, (x[j].z - mu) * rs, (x[j].w - mu) * rs);
        const float d0 = w4[j].x * dy[j].x, d1 = w4[j].y * dy[j].y, d2 = w4[j].z * dy[j].z, d3 = w4[j].w * dy[j].w;
        a += (d0 + d1) + (d2 + d3);
        bs += (d0 * nr[j].x + d1 * nr[j].y) + (d2 * nr[j].z + d3 * nr[j].w);
    }
    const float dm = warp_sum(a) / (float)C, dnm = warp_sum(bs) / (float)C;
#pragma unroll
    for (int j = 0; j < NV; j++) {
        dv[j].x = ((w4[j].x * dy[j].x - dm) - nr[j].x * dnm) * rs;
        dv[j].y = ((w4[j].y * dy[j].y - dm) - nr[j].y * dnm) * rs;
        dv[j].z = ((w4[j].z * dy[j].z - dm) - nr[j].z * dnm) * rs;
        dv[j].w = ((w4[j].w * dy[j].w - dm) - nr[j].w * dnm) * rs;
    }
}
}  // namespace vit
