// ops_internal.h — stream-explicit launchers shared by the C-ABI ops and the trainer.
#pragma once
#include "common.h"
#include "gemm.h"
#include "../../include/vit_ops.h"

namespace vit {
int grid_for(long long n, int threads);
void ln_forward_f32(float* out, float* mean, float* rstd, const float* inp, const float* w,
                    const float* b, long long rows, int C, hipStream_t s);
void ln_forward_bf16(bf16_t* out, float* mean, float* rstd, const float* inp, const float* w,
                     const float* b, long long rows, int C, hipStream_t s);
// dinp += LN_dinp(dout); dw / db += the column sums, in a fixed order through per-block partial
// rows in ws (nullptr = thread workspace; ln_bwd_blocks(rows) * 2C floats)
void ln_backward_f32(float* dinp, float* dw, float* db, const float* dout, const float* inp,
                     const float* w, const float* mean, const float* rstd, long long rows, int C,
                     hipStream_t s, float* ws = nullptr);
// the trainer's residual-gradient stream in "bf16 + lo8" form (common.h lo8_*: a bf16 plane, the
// GEMM operand, and a byte plane of the rounding residual; lo planes nullable = plain bf16):
// dres_out = dres_in + LN_dinp(dout); dres_colsum / dw / db as above, taken in fp32 before the
// rounding; part != null: per-block partial rows [ln_bwd_blocks(rows)][2C or 3C] (dw | db |
// dres_colsum) instead of atomics, summed later in a fixed order
void ln_backward_bf16_stream(bf16_t* dres_out, uint8_t* lo_out, const bf16_t* dres_in, const uint8_t* lo_in,
                             float* dw, float* db, float* dres_colsum, const bf16_t* dout, const float* inp,
                             const float* w, const float* mean, const float* rstd, long long rows, int C,
                             hipStream_t s, float* part = nullptr);
int ln_bwd_blocks(long long rows);
void convert_f2bf(bf16_t* out, const float* inp, long long n, hipStream_t s);
void sgd(float* p, const float* g, long long n, float lr, hipStream_t s);
void softmax_rows(float* probs, const float* logits, long long rows, int V, hipStream_t s);
void ce_forward(float* losses, const float* probs, const int* targets, long long rows, int V,
                hipStream_t s);
void ce_backward(float* dlogits, const float* dlosses, const float* probs, const int* targets,
                 long long rows, int V, hipStream_t s);
void im2col_f32(float* out, const float* px, int B, int IMG, int P, hipStream_t s);
void im2col_bf16(bf16_t* out, const float* px, int B, int IMG, int P, hipStream_t s);
// rows padded to KPP columns (zeros past 3*P*P; KPP % 8 == 0): the bf16 GEMM operand of a patch
// whose 3*P*P is not a multiple of 8 (ViT-H/14: 588 -> 640)
void im2col_pad_bf16(bf16_t* out, const float* px, int B, int IMG, int P, int KPP, hipStream_t s);
void patch_assemble(float* enc, const float* emb, const float* cls, const float* wpe, int B,
                    int NP, int C, hipStream_t s);
// out[c][r] = in[r][c] for `count` R x Cc bf16 matrices `stride` elements apart (in and out)
void transpose_bf16(bf16_t* out, const bf16_t* in, int R, int Cc, int count, long long stride,
                    hipStream_t s);
void patch_gather_f32(float* out, const float* denc, int B, int NP, int C, hipStream_t s);
void patch_gather_bf16(bf16_t* out, const float* denc, int B, int NP, int C, hipStream_t s);
// (bf16 + lo8 input: lo nullable)
void patch_gather_f32(float* out, const bf16_t* denc, const uint8_t* lo, int B, int NP, int C, hipStream_t s);
void patch_gather_bf16(bf16_t* out, const bf16_t* denc, int B, int NP, int C, hipStream_t s);
// dcls += sum_b denc[b,0];  dwpe[t] += sum_b denc[b,t];  dpb += sum_{b,t>0} denc[b,t] — fixed order
// (no atomics); ws (nullable = thread workspace): T*C floats of per-position sums
void patch_small_grads(float* dcls, float* dwpe, float* dpb, const float* denc, int B, int T,
                       int C, hipStream_t s, float* ws = nullptr);
// part (nullable): PSG_CHUNKS * T * C floats of per-image-chunk partial sums (the chunked form)
constexpr int PSG_CHUNKS = 16;
void patch_small_grads(float* dcls, float* dwpe, float* dpb, const bf16_t* denc, const uint8_t* lo, int B, int T,
                       int C, hipStream_t s, float* ws = nullptr, float* part = nullptr);
// attention.hip
void attn_forward_f32(float* out, float* preatt, float* att, const float* inp, int B, int T, int C,
                      int NH, hipStream_t s);
void attn_backward_f32(float* dinp, float* dpreatt, float* datt, const float* dout,
                       const float* inp, const float* att, int B, int T, int C, int NH,
                       hipStream_t s);
bool attn_fused_supported(int T, int C, int NH);
bool attn_generic_supported(int T, int C, int NH);  // VALU bf16 kernels (other head sizes, T > 256)
void attn_forward_fused(bf16_t* out, float* lse, const bf16_t* qkv, int B, int T, int C, int NH,
                        hipStream_t s);
// dqkv_colsum (nullable, [3C]) += column sums of dqkv (the qkv bias gradient, fused, fixed order);
// colsum_store: dqkv_colsum = the sums instead (a per-micro-batch partial row the trainer reduces)
// floats of the workspace attn_backward_fused needs (generic delta rows / fused column-sum partials)
size_t attn_backward_ws_floats(int B, int T, int C, int NH);
void attn_backward_fused(bf16_t* dqkv, const bf16_t* dout, const bf16_t* qkv, const bf16_t* out,
                         const float* lse, int B, int T, int C, int NH, hipStream_t s,
                         float* dqkv_colsum = nullptr, float* ws = nullptr, bool colsum_store = false);
// ws (nullable = thread workspace): B*NH*192 floats — per-(b,h) bias partial sums
}  // namespace vit
