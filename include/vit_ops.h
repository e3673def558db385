/*
 * vit_ops.h — C ABI of libvit_hip.so: the reference's layer ops as MI355X (gfx950) HIP kernels.
 *
 * Drop-in boundary.  The reference's layer ops are the free functions of
 * /root/reference/train_vit.rs:376-670 (raw *mut f32 / *const f32 + c_int dims).  Each symbol
 * below keeps the reference's name, argument order (outputs, inputs/weights, dims) and write
 * semantics, with DEVICE pointers:
 *   - forward ops OVERWRITE their outputs; backward ops ACCUMULATE (+=) into dinp/dweight/dbias
 *     (train_vit.rs:524-525, 538, 549, 552, 578-579, 587, 595-596, 626-633, 650);
 *   - a NULL bias means "no bias" (train_vit.rs:388, 548);
 *   - the caller owns every buffer (ops never allocate caller-visible memory);
 *   - ops are enqueued on the calling thread's stream (vit_set_stream); with VIT_SYNC=1 in the
 *     environment every op synchronises before returning, restoring the reference's
 *     synchronous semantics;
 *   - the reference ops return () and have no error channel: failures (bad shapes, HIP errors)
 *     set a sticky thread-local error read with vit_last_error().
 * Semantic fixes relative to the reference text (SURVEY.md §8a defect register) are applied:
 * D1 offsets by T, D2 full normalisation, D3 non-causal attention, D4 GELU derivative,
 * D5 LN backward, D6 -log p loss, D7 patch embedding, D10 64-bit offsets.
 * Activation layouts are the reference's: qkv [B,T,3C] (Q|K|V, head h at h*hs),
 * preatt/att [B,T,NH,T] (row index bth = (b*T+t)*NH+h, train_vit.rs:406-410).
 */
#ifndef VIT_OPS_H
#define VIT_OPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ context */
int vit_init(int device);                 /* select device; 0 on success */
void vit_set_stream(void* hip_stream);    /* hipStream_t; NULL = default stream */
void* vit_get_stream(void);
int vit_sync(void);                        /* hipStreamSynchronize(current stream) */
int vit_last_error(const char** msg);      /* 0 = no error; sticky until vit_clear_error */
void vit_clear_error(void);
/* device memory helpers for hosts without their own device allocator (ctypes tests, C hosts) */
void* vit_malloc(size_t bytes);
void vit_free(void* p);
int vit_memcpy_h2d(void* dst, const void* src, size_t bytes);
int vit_memcpy_d2h(void* dst, const void* src, size_t bytes);
int vit_memcpy_d2d(void* dst, const void* src, size_t bytes);
int vit_memset(void* dst, int value, size_t bytes);
/* launch counters: how many launches of each kernel family ran since the last reset (process-wide,
 * every thread and stream).  GEMM families are indexed base + epilogue (epi < 16, gemm.h Epi). */
enum {
    VIT_HIT_GEMM_128 = 0,            /* bf16 128x128 register-staged (small / ragged shapes) */
    VIT_HIT_GEMM_256x256 = 16,       /* bf16 256x256 LDS-DMA engine, one workgroup per CU */
    VIT_HIT_GEMM_256x128 = 32,       /* bf16 256x128 LDS-DMA engine, two workgroups per CU */
    VIT_HIT_GEMM_FP8 = 48,           /* MXFP8 256x256 engine */
    VIT_HIT_GEMM_F32 = 64,           /* fp32 MFMA (parity path) */
    VIT_HIT_SPLITK_REDUCE = 80,      /* split-K slab reduction (separate launch) */
    VIT_HIT_ATTN_FWD_MFMA = 81,      /* fused MFMA attention forward */
    VIT_HIT_ATTN_BWD_PERSISTENT = 82,/* persistent one-pass MFMA attention backward */
    VIT_HIT_ATTN_BWD_ONEPASS = 83,   /* one-pass backward, one workgroup per (b,h) */
    VIT_HIT_ATTN_BWD_PAIR = 84,      /* paired-role backward */
    VIT_HIT_ATTN_GENERIC = 85,       /* generic VALU attention (T past the MFMA kernels' LDS) */
    VIT_HIT_ATTN_BWD_XKEY = 86,      /* one-pass backward + the last key's side path (T = 32k + 1) */
    VIT_HIT_QUANT_ROWCOL = 87,       /* fused row + column MX quantization */
    VIT_HIT_GEMM_PP = 88,            /* bf16 two-group ping-pong 192x256 engine (variant 11; also counted as 256x256 + epi) */
    VIT_HIT_LN_MX = 89,              /* LayerNorm forward straight into the row + column MX forms (fp8) */
    VIT_HIT_LNB_MX = 90,             /* LayerNorm backward (residual-gradient stream) + both MX forms (fp8) */
    VIT_HIT_COUNT = 96
};
int vit_kernel_hits(long long* out, int n); /* copies min(n, VIT_HIT_COUNT); returns VIT_HIT_COUNT */
void vit_kernel_hits_reset(void);
/* events for per-kernel timing on the current stream */
void* vit_event_create(void);
void vit_event_destroy(void* ev);
int vit_event_record(void* ev);
float vit_event_elapsed_ms(void* start, void* stop);

/* ------------------------------------------------------------------ reference ops (fp32) */
/* train_vit.rs:376 */
void residual_forward(float* out, const float* inp1, const float* inp2, int N);
/* train_vit.rs:384 — out[BT,OC] = inp[BT,C] . weight[OC,C]^T + bias */
void matmul_forward(float* out, const float* inp, const float* weight, const float* bias,
                    int B, int T, int C, int OC);
/* train_vit.rs:400 (+ attention.rs:1) — preatt/att [B,T,NH,T] are materialised like the
 * reference; either may be NULL (fused use: the scores are then not stored) */
void attention_forward(float* out, float* preatt, float* att, const float* inp,
                       int B, int T, int C, int NH);
/* train_vit.rs:453 */
void layernorm_forward(float* out, float* mean, float* rstd, const float* inp,
                       const float* weight, const float* bias, int B, int T, int C);
/* train_vit.rs:482 */
void gelu_forward(float* out, const float* inp, int N);
/* train_vit.rs:493 */
void softmax_forward(float* probs, const float* logits, int B, int T, int V);
/* rusty_vit.rs:836 (called train_vit.rs:256), D6: losses = -log probs[target] */
void crossentropy_forward(float* losses, const float* probs, const int* targets,
                          int B, int T, int V);
/* train_vit.rs:521 (+=) */
void residual_backward(float* dinp1, float* dinp2, const float* dout, int N);
/* train_vit.rs:530 (+=); dinp NULL skips the input gradient, dbias NULL skips the bias */
void matmul_backward(float* dinp, float* dweight, float* dbias, const float* dout,
                     const float* inp, const float* weight, int B, int T, int C, int OC);
/* train_vit.rs:559 (+=); dpreatt/datt: accumulated [B,T,NH,T] scratch, NULL = internal */
void attention_backward(float* dinp, float* dpreatt, float* datt, const float* dout,
                        const float* inp, const float* att, int B, int T, int C, int NH);
/* train_vit.rs:603 (+=) */
void layernorm_backward(float* dinp, float* dweight, float* dbias, const float* dout,
                        const float* inp, const float* weight, const float* mean,
                        const float* rstd, int B, int T, int C);
/* train_vit.rs:639 (+=), D4 */
void gelu_backward(float* dinp, const float* inp, const float* dout, int N);
/* undefined in the reference, called train_vit.rs:293 (+=): dlogits += (p - 1[tgt]) * dloss */
void crossentropy_softmax_backward(float* dlogits, const float* dlosses, const float* probs,
                                   const int* targets, int B, int T, int V);
/* ViT replacement of encoder_forward (train_vit.rs:196): pixels [B,3,IMG,IMG] ->
 * encoded [B,T,C], row 0 = cls + wpe[0], row 1+p = patch_p . patch_w^T + patch_b + wpe[1+p] */
void patch_embed_forward(float* encoded, const float* pixels, const float* patch_w,
                         const float* patch_b, const float* cls, const float* wpe,
                         int B, int IMG, int P, int C);
/* ViT replacement of encoder_backward (train_vit.rs:371), (+=), no pixel gradient */
void patch_embed_backward(float* dpatch_w, float* dpatch_b, float* dcls, float* dwpe,
                          const float* dencoded, const float* pixels, int B, int IMG, int P,
                          int C);
/* optimizer_step (train_vit.rs:737): params -= lr * grads */
void sgd_step(float* params, const float* grads, long long n, float lr);

/* ------------------------------------------------------------------ bf16 fast path
 * Build-side extensions with the same conventions; bf16 storage as raw uint16_t, fp32
 * accumulate; LN statistics, biases, residual stream and gradients stay fp32.           */
/* out_bf16[BT,OC] = inp . W^T + bias */
void matmul_forward_bf16(uint16_t* out, const uint16_t* inp, const uint16_t* weight,
                         const float* bias, int B, int T, int C, int OC);
/* dinp_f32 += dout . W (NULL skips);  dweight_f32 += dout^T . inp (split-K, atomics) */
void matmul_backward_bf16(float* dinp, float* dweight, float* dbias, const uint16_t* dout,
                          const uint16_t* inp, const uint16_t* weight, int B, int T, int C,
                          int OC);
/* fused attention: out_bf16 [B,T,C], lse [B,NH,T] (log2 domain), no T x T HBM traffic.
 * Head sizes 32/64/80/96/128 run the MFMA kernels while the head's operands fit the LDS
 * (T <= 320; <= 288 at head size 128), e.g. ViT-B/16 (hs 64, T 197) and ViT-H/14 (hs 80,
 * T 257); longer sequences run generic VALU kernels with the same outputs; other shapes set
 * vit_last_error.  vit_attention_kernel_kind: 1 = MFMA, 2 = generic, 0 = unsupported. */
int vit_attention_kernel_kind(int T, int C, int NH);
void attention_forward_fused_bf16(uint16_t* out, float* lse, const uint16_t* inp,
                                  int B, int T, int C, int NH);
/* dinp_bf16 [B,T,3C] is OVERWRITTEN (it is produced whole); recomputes P from lse */
void attention_backward_fused_bf16(uint16_t* dinp, const uint16_t* dout, const uint16_t* inp,
                                   const uint16_t* out, const float* lse, int B, int T, int C,
                                   int NH);
/* As attention_backward_fused_bf16, plus the fused qkv-bias gradient the trainer uses:
 * dqkv_bias[j] += sum over the B*T rows of dinp[row][j] (fp32 sums of the unrounded values,
 * deterministic order), j < 3C.  dqkv_bias may be NULL. */
void attention_backward_fused_bf16_ex(uint16_t* dinp, const uint16_t* dout, const uint16_t* inp,
                                      const uint16_t* out, const float* lse, int B, int T, int C, int NH,
                                      float* dqkv_bias);
void layernorm_forward_bf16(uint16_t* out, float* mean, float* rstd, const float* inp,
                            const float* weight, const float* bias, int B, int T, int C);
/* train_vit.rs:603 with the LN-output gradient in bf16 (as the trainer's dgrad GEMMs write it):
 * dinp, dweight, dbias (fp32) += */
void layernorm_backward_bf16(float* dinp, float* dweight, float* dbias, const uint16_t* dout,
                             const float* inp, const float* weight, const float* mean,
                             const float* rstd, int B, int T, int C);
/* train_vit.rs:482 / :639 (D4) in the form the fused GEMM epilogues use (logistic tanh, raw
 * v_exp / v_rcp): out_bf16 = gelu(inp_bf16); dinp_f32 += gelu'(inp_bf16) * dout_bf16 */
void gelu_forward_bf16(uint16_t* out, const uint16_t* inp, int N);
void gelu_backward_bf16(float* dinp, const uint16_t* inp, const uint16_t* dout, int N);
/* generic bf16 GEMM (the engine under matmul_*_bf16), for tests and tools:
 * C[M,N] (epilogue)= A . B with A(m,k) = a_kcontig ? A[m*lda+k] : A[k*lda+m],
 * B(k,n) = b_kcontig ? B[n*ldb+k] : B[k*ldb+n].  epi: 0 f32 store, 1 f32 +=, 2 f32 atomic +=
 * (split-K), 3 bf16 store; bias (nullable) is added for 0/1/3; dbias (nullable, epi 2 with an
 * M-contig A) receives the row sums of A. */
void gemm_bf16_ex(void* C, long long ldc, const uint16_t* A, long long lda, int a_kcontig,
                  const uint16_t* B, long long ldb, int b_kcontig, const float* bias,
                  float* dbias, int M, int N, int K, int epi, int splitk);
/* the fused epilogues of the trainer's GEMMs: epi 4 C = pre = acc + bias, C2 = gelu(pre)
 * (both bf16); 5 C_f32 = acc + bias + aux_f32; 6 C_bf16 = acc * gelu'(aux_bf16) and, when
 * colsum_out is not NULL, colsum_out[n] += sum_m C[m][n]; 0 / 3 as gemm_bf16_ex.  The pair the
 * trainer uses for the MLP (fc forward -> fcproj dgrad): epi 8 C = gelu'(pre), C2 = gelu(pre)
 * (both bf16, pre = acc + bias, one sigmoid for both); 9 C_bf16 = acc * aux_bf16 (aux = the
 * stored gelu') with the colsum_out of epi 6. */
void gemm_bf16_fused(void* C, void* C2, long long ldc, const void* aux, long long ldaux,
                     const uint16_t* A, long long lda, int a_kcontig, const uint16_t* B,
                     long long ldb, int b_kcontig, const float* bias, float* colsum_out, int M,
                     int N, int K, int epi);
/* ------------------------------------------------------------------ fp8 (MXFP8) GEMM path
 * OCP fp8 e4m3 operands with one E8M0 scale per 32 consecutive k-elements of a row (OCP MX block
 * scaling) on v_mfma_scale_f32_32x32x64_f8f6f4, fp32 accumulate: the fp8 mode's forward and
 * input-gradient GEMMs (matmul_forward, train_vit.rs:384; dinp of matmul_backward, :530-541).
 * Scales use the lane-native layout [K/64][Rpad/32][64] bytes (Rpad = rows rounded up to 256;
 * byte h*32 + r of row group g at step s scales row 32g + r, k-block 2s + h): mx_scale_size
 * bytes per operand.  quantize_mx_*: x [R][K] (row stride ldx elements, K % 64 == 0) -> q [R][K]
 * e4m3 (row stride ldq bytes) + scales; scale 2^X with X = ceil(log2(amax / 448)) per block,
 * x * 2^-X rounded to nearest even.  gemm_fp8_fused: C = A . B^T with A [M][K], B [N][K]
 * (K-contiguous bytes) and the epilogues of gemm_bf16_fused (epi 0, 1, 2, 3, 4, 5, 6, 8, 9; epi 2 =
 * C += A . B^T through K-split fp32 slabs and a fixed-order reduce: the fp8 weight gradient of
 * matmul_backward, train_vit.rs:543-555, with A / B from quantize_mx_cols_bf16_ex). */
long long mx_scale_size(long long rows, int K);
void quantize_mx_bf16_ex(uint8_t* q, uint8_t* scales, const uint16_t* x, long long R, int K,
                         long long ldx, long long ldq);
void quantize_mx_f32_ex(uint8_t* q, uint8_t* scales, const float* x, long long R, int K,
                        long long ldx, long long ldq);
/* column-wise MX (blocks of 32 consecutive ROWS of x: the token axis a weight gradient reduces
 * over): x [R][C] bf16 (row stride ldx, C % 64 == 0) -> q [C][Kp] e4m3, Kp = mx_cols_padded(R)
 * (R rounded up to 64, padding tokens zero) + scales (mx_scale_size(C, Kp) bytes); equal, byte for
 * byte, to quantize_mx_bf16_ex of the zero-padded transpose. */
long long mx_cols_padded(long long R);
void quantize_mx_cols_bf16_ex(uint8_t* q, uint8_t* scales, const uint16_t* x, long long R, int C,
                              long long ldx);
/* both forms in one read of x [R][C] (row stride ldx): qr [R][C] + scales_r exactly as
 * quantize_mx_bf16_ex(qr, scales_r, x, R, C, ldx, C), and the column form of tokens
 * [tok_off, tok_off + ntok) of a [C][ldqc] matrix + scales_c (mx_scale_size(C, ldqc) bytes) exactly
 * as the same span of quantize_mx_cols_bf16_ex over the whole token axis; tok_off % 64 == 0,
 * R <= ntok <= R rounded up to 64 (tokens R .. ntok-1 are zero padding). */
void quantize_mx_rowcol_bf16_ex(uint8_t* qr, uint8_t* scales_r, uint8_t* qc, uint8_t* scales_c,
                                const uint16_t* x, long long R, int C, long long ldx, long long ldqc,
                                long long tok_off, long long ntok);
/* LayerNorm forward (train_vit.rs:453-480) straight into both MX forms: exactly
 * layernorm_forward_bf16 (mean / rstd as it writes them) followed by quantize_mx_rowcol_bf16_ex of
 * its bf16 output, without the bf16 tensor; inp [R][C] fp32, C a multiple of 256 in 256 .. 2048
 * (not 1792). */
/* the trainer's residual-gradient LayerNorm backward (train_vit.rs:603-637 + the residual add,
 * "bf16 + lo8" planes: dres_out = dres_in + LN_dinp(dout); dweight / dbias / dres_colsum (nullable)
 * += the column sums of dout * xhat / dout / dres_out in a fixed order) ... */
void layernorm_backward_stream(uint16_t* dres_out, uint8_t* lo_out, const uint16_t* dres_in, const uint8_t* lo_in,
                               float* dweight, float* dbias, float* dres_colsum, const uint16_t* dout, const float* inp,
                               const float* weight, const float* mean, const float* rstd, long long R, int C);
/* ... and the same with both MX forms of dres_out's bf16 plane written beside it (exactly
 * quantize_mx_rowcol_bf16_ex of dres_out; the column sums group rows differently: equal within fp32
 * rounding, not bitwise); C a multiple of 256 in 256 .. 1280 */
void layernorm_backward_stream_mx(uint16_t* dres_out, uint8_t* lo_out, const uint16_t* dres_in, const uint8_t* lo_in,
                                  float* dweight, float* dbias, float* dres_colsum, const uint16_t* dout,
                                  const float* inp, const float* weight, const float* mean, const float* rstd,
                                  long long R, int C, uint8_t* qr, uint8_t* scales_r, uint8_t* qc, uint8_t* scales_c,
                                  long long ldqc, long long tok_off, long long ntok);
void layernorm_forward_mx(uint8_t* qr, uint8_t* scales_r, uint8_t* qc, uint8_t* scales_c, float* mean,
                          float* rstd, const float* inp, const float* weight, const float* bias, long long R,
                          int C, long long ldqc, long long tok_off, long long ntok);
void gemm_fp8_fused(void* C, void* C2, long long ldc, const void* aux, long long ldaux,
                    const uint8_t* A, const uint8_t* a_scale, long long lda, const uint8_t* B,
                    const uint8_t* b_scale, long long ldb, const float* bias, float* colsum_out,
                    int M, int N, int K, int epi);
/* gemm_fp8_fused with the fused MX copy of the bf16 output (epi 4 / 8: the GELU output C2; epi 6 / 9: C):
 * mx_q [M][N] e4m3 (ld N), mx_s lane-native scales for mx_rows_padded(M) rows, bit-identical to
 * quantize_mx_bf16_ex of that bf16 output (padding rows' scales are left as given). */
void gemm_fp8_fused_mx(void* C, void* C2, long long ldc, const void* aux, long long ldaux, const uint8_t* A,
                       const uint8_t* a_scale, long long lda, const uint8_t* B, const uint8_t* b_scale,
                       long long ldb, const float* bias, float* colsum_out, int M, int N, int K, int epi,
                       uint8_t* mx_q, uint8_t* mx_s);
/* gemm_fp8_fused_mx plus the column-wise MX copy of the same output (the weight gradient's
 * operand): output row m -> token mxc_off + m of mxc_q [N][mxc_ld] + scales mxc_s
 * (mx_scale_size(N, mxc_ld) bytes), equal byte for byte to quantize_mx_cols_bf16_ex of the bf16
 * output; M % 64 == 0, N % 64 == 0, mxc_off % 64 == 0.  The MX-copied bf16 output (C2 of epi 4 / 8,
 * C of epi 6 / 9) may be NULL: not stored. */
void gemm_fp8_fused_mxc(void* C, void* C2, long long ldc, const void* aux, long long ldaux, const uint8_t* A,
                        const uint8_t* a_scale, long long lda, const uint8_t* B, const uint8_t* b_scale,
                        long long ldb, const float* bias, float* colsum_out, int M, int N, int K, int epi,
                        uint8_t* mx_q, uint8_t* mx_s, uint8_t* mxc_q, uint8_t* mxc_s, long long mxc_ld,
                        long long mxc_off);
/* tools: GEMM engine selection (0 = the default; 1 = 128x128 everywhere, 2 = 256x256 one tile per
 * workgroup with the split-K weight gradients on 256x128, 4 = 256x128 two per CU everywhere,
 * 5 = 4 with a software-pipelined main loop, 7 = production: 2 with the persistent streaming
 * 256x256 engine for the K-contiguous GEMMs) and diagnostics (flag 2: skip epilogues, main-loop
 * timing only; flag 16: the persistent engine drains its stores after each epilogue; flag 32: every
 * output row stored onto row 0 (timing only, wrong outputs: no HBM write traffic); (flags >> 8) &
 * 0xFF: first-round stagger in 0.5 us units; (flags >> 16) & 0xF = g + 1: persistent-engine tile
 * groups of g row panels, 0 = column-major ... default 8 for K <= 768, else row-major) */
void gemm_bf16_set_variant(int variant);
void gemm_bf16_set_debug(int flags);
/* diagnostic: per-workgroup timestamps of the 256x256 / 256x128 bf16 engines into trace (device,
 * 16 x u64 per workgroup of the next launches, 100 MHz s_memrealtime: 0 start, 1 main-loop end,
 * 2 end of wave 0, 3 hardware id = XCC_ID << 32 | HW_ID, 4 + w end of wave w, 12 first K-step's
 * operands landed); NULL turns it off */
void gemm_bf16_set_trace(unsigned long long* trace);
void convert_f32_to_bf16(uint16_t* out, const float* inp, long long n);
void convert_bf16_to_f32(float* out, const uint16_t* inp, long long n);

#ifdef __cplusplus
}
#endif
#endif
