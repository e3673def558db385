// gemm.h — internal GEMM launcher API shared by the C-ABI ops and the trainer.
//
// C[M,N] (epilogue)= A[M,K] . B[K,N] with per-operand storage:
//   A(m,k) = a_kcontig ? A[m*lda + k] : A[k*lda + m]
//   B(k,n) = b_kcontig ? B[n*ldb + k] : B[k*ldb + n]
// The three products of matmul_forward/backward (train_vit.rs:384-398, 530-557) map to
//   forward  (out = inp . W^T):   A = inp  (K-contig), B = W (K-contig, W[n][k])
//   dgrad    (dinp = dout . W):   A = dout (K-contig), B = W (N-contig, W[k][n])
//   wgrad    (dW = dout^T . inp): A = dout (M-contig), B = inp (N-contig); K = B*T rows
#pragma once
#include "common.h"

namespace vit {

enum Epi {
    EPI_F32_STORE = 0,   // C_f32 = acc (+ bias[n])
    EPI_F32_ACC = 1,     // C_f32 += acc (+ bias[n])
    EPI_F32_ATOMIC = 2,  // C_f32 += acc, K split into fp32 slabs + one fixed-order reduce (no atomics)
    EPI_BF16_STORE = 3,  // C_bf16 = acc (+ bias)
    EPI_BF16_GELU = 4,   // C_bf16 = pre = acc + bias; C2_bf16 = gelu(pre)
    EPI_F32_RESID = 5,   // C_f32 = acc + bias + aux_f32[m*ldaux + n]
    EPI_BF16_DGELU = 6,  // C_bf16 = acc * gelu'(aux_bf16[m*ldaux + n])
    EPI_F32_SLAB = 7,    // internal: split-K partial -> workspace slab[split][M][N] (float4 stores)
    // the trainer's pair: the fc forward stores gelu'(pre) in place of pre, so the fcproj dgrad
    // epilogue is one multiply instead of a second sigmoid (exp + rcp) per element
    EPI_BF16_GELU_D = 8,  // C_bf16 = gelu'(pre), pre = acc + bias; C2_bf16 = gelu(pre)
    EPI_BF16_MUL = 9,     // C_bf16 = acc * aux_bf16[m*ldaux + n]   (aux = a stored gelu')
};
// epilogues that read a bf16 aux operand / that may sum the output's columns (colsum_out)
constexpr bool epi_aux16(int e) { return e == EPI_BF16_DGELU || e == EPI_BF16_MUL; }
// epilogues that add the bias
constexpr bool epi_bias(int e) { return e != EPI_F32_ATOMIC && e != EPI_F32_SLAB && !epi_aux16(e); }
// epilogues with an MX copy of a bf16 output (gelu for the GELU pairs, the product for the aux ones)
constexpr bool epi_mx(int e) { return e == EPI_BF16_GELU || e == EPI_BF16_GELU_D || epi_aux16(e); }

struct GemmArgs {
    const void* A = nullptr;
    long long lda = 0;
    bool a_kcontig = true;
    const void* B = nullptr;
    long long ldb = 0;
    bool b_kcontig = true;
    void* C = nullptr;
    long long ldc = 0;
    void* C2 = nullptr;
    const void* aux = nullptr;
    long long ldaux = 0;
    const float* bias = nullptr;
    float* dbias = nullptr;  // bf16 wgrad with an M-contig A: dbias[m] += sum_k A(m,k) (fused colsum)
    // EPI_BF16_DGELU / EPI_BF16_MUL column sums of the output, deterministic: the epilogue stores
    // partial rows colsum_part[gemm_colsum_rows(a)][N] (row r = output rows 128r..128r+127, 96r.. on the
    // ping-pong engine; nullptr = thread workspace) and, with colsum_out set, the launcher adds them
    // into colsum_out in a fixed order.
    // colsum_part without colsum_out: the caller reduces the rows (the trainer, across micro-batches).
    float* colsum_out = nullptr;
    float* colsum_part = nullptr;
    int M = 0, N = 0, K = 0;
    int epi = EPI_F32_STORE;
    int splitk = 0;  // 0 = choose automatically (only EPI_F32_ATOMIC may split)
    // automatic split-K: the share of the engine's slots one round of work items should fill, percent
    // (0 = the engine's default, 45: a weight gradient beside other streams; the trainer passes 80 when
    // the kernel has the GPU to itself)
    int fill_pct = 0;
    // split-K workspace for EPI_F32_ATOMIC on the 256x256 kernel: partials go to fp32 slabs and
    // one reduce kernel adds them into C (no atomics).  nullptr = the calling thread's workspace
    // (ordered on the context stream); the trainer passes its own buffer for its stream.
    float* ws = nullptr;
    size_t ws_bytes = 0;
    // fp8 operands (gemm_fp8): MX scales of A and B in the lane-native layout of gemm_fp8.hip
    const void* a_scale = nullptr;
    const void* b_scale = nullptr;
    // fused MX copy of the epilogue's bf16 output (EPI_BF16_GELU / _GELU_D: the GELU output C2;
    // EPI_BF16_DGELU / _MUL: C), laid out as the next GEMM's A operand ([M][N] fp8, ld N, lane-native
    // scales for mx_rows_padded(M) rows; the padding rows' scales are the caller's zeros).  Staged
    // epilogues of the 256x256 engines only (N % 64 == 0); bit-identical to quantize_mx_bf16 of
    // the bf16 output.
    uint8_t* mx_q = nullptr;
    uint8_t* mx_s = nullptr;
    // fused column-wise MX copy of the same output (fp8 engine: the weight gradient's operand, MX
    // blocks of 32 consecutive output rows): output row m -> token mxc_off + m of a [N][mxc_ld]
    // fp8 matrix + lane-native scales for mx_rows_padded(N) rows; M % 64 == 0, N % 64 == 0,
    // mxc_off % 64 == 0.  Bit-identical to quantize_mx_cols_bf16 of the bf16 output.  With
    // mx_q / mxc_q set, the MX-copied bf16 output (C2 of GELU / GELU_D, C of DGELU / MUL) may be
    // nullptr: not stored.
    uint8_t* mxc_q = nullptr;
    uint8_t* mxc_s = nullptr;
    long long mxc_ld = 0;
    long long mxc_off = 0;
    // variant 10 (split tail of the persistent engine): fp32 partial tiles of the last round, one buffer
    // per concurrent stream (nullptr = the thread workspace); up to 64 MiB at 256 CUs
    float* tail_ws = nullptr;
    size_t tail_ws_bytes = 0;
};

// fp32 operands, exact-fp32 MFMA (v_mfma_f32_16x16x4_f32); any shape/stride. Parity path.
void gemm_f32(const GemmArgs& a, hipStream_t s);
// bf16 operands, fp32 accumulate (v_mfma_f32_16x16x32_bf16); requires K%8==0, 16-B aligned
// operands, lda/ldb%8==0, the contiguous dim of an M/N-contig operand %8==0, N%4==0.
void gemm_bf16(const GemmArgs& a, hipStream_t s);
bool gemm_bf16_supported(const GemmArgs& a);
// engine selection for A/B measurements in one process: 1 = 128x128 everywhere, 2 = production
// (256x256, 1 WG/CU; split-K weight gradients on 256x128, 2 WG/CU), 4 = 256x128 everywhere;
// anything else = 2.  Debug flag 2 = skip the epilogues (main-loop-only timing).
// 0 (or any unknown value) clears the selection: the next GEMM re-reads VIT_GEMM (default 7)
void gemm_set_variant(int v);
void gemm_set_debug(int flags);
// compute units of the current device: the persistent engines' grid (one workgroup per CU)
int gemm_cu_count();
int gemm_persist_grid();  // workgroups of the persistent engines (VIT_PERSIST_CUS; default gemm_cu_count())
int gemm_variant_selected();  // the engine variant in effect (VIT_GEMM / gemm_set_variant)
struct GemmParams;
// variant 9: the one-wave-per-SIMD persistent engine (gemm_w4.hip) for K-contiguous operands without
// split-K (K % 64 == 0, K >= 128); false = shape not taken
bool gemm_bf16_w4(const GemmArgs& a, const GemmParams& p, int tiles, hipStream_t s);
void gemm_set_trace(unsigned long long* trace);
// variant 11: the two-group ping-pong engine (gemm_pp.hip, 192x256 tiles) for the shapes it takes
bool gemm_pp_shape(const GemmArgs& a);
void gemm_bf16_pp(const GemmArgs& a, const GemmParams& p, hipStream_t s);
// the number of column-sum partial rows gemm_bf16 (fp8 = false) or gemm_fp8 (true) writes for an
// x-aux epilogue of these arguments (GemmArgs::colsum_part): cdiv(M, 96) on the ping-pong engine,
// cdiv(M, 128) on every other engine
int gemm_colsum_rows(const GemmArgs& a, bool fp8);
bool gemm_streaming();  // the production variant: persistent streaming engines (bf16 and fp8)

// fp8 (OCP e4m3) operands with MX block scales (one E8M0 per 32 k-elements), fp32 accumulate
// (v_mfma_scale_f32_32x32x64_f8f6f4): A [M][K], B [N][K] K-contiguous byte rows (lda/ldb in
// bytes, % 16 == 0), K % 64 == 0, scales from quantize_mx_* (a_scale / b_scale); every epilogue,
// EPI_F32_ATOMIC as K-split fp32 slabs + a fixed-order reduce (a.ws or the thread workspace).
void gemm_fp8(const GemmArgs& a, hipStream_t s);
bool gemm_fp8_supported(const GemmArgs& a);
// MX quantizer: x [R][K] (row stride ldx elements) -> q [R][K] e4m3 (row stride ldq bytes) +
// scales sl (mx_scale_bytes(R, K) bytes, layout of gemm_fp8.hip)
void quantize_mx_bf16(uint8_t* q, uint8_t* sl, const bf16_t* x, long long R, int K, long long ldx,
                      long long ldq, hipStream_t s);
void quantize_mx_f32(uint8_t* q, uint8_t* sl, const float* x, long long R, int K, long long ldx,
                     long long ldq, hipStream_t s);
// `count` dense [R][K] matrices xs elements apart -> q matrices qs bytes apart, scales ss apart
void quantize_mx_batched_bf16(uint8_t* q, uint8_t* sl, const bf16_t* x, long long R, int K, int count,
                              long long xs, long long qs, long long ss, hipStream_t s);
void quantize_mx_batched_f32(uint8_t* q, uint8_t* sl, const float* x, long long R, int K, int count,
                             long long xs, long long qs, long long ss, hipStream_t s);
// column-wise MX for the fp8 weight gradients: x [R tokens][C] bf16 (row stride ldx, C % 64 == 0)
// -> q [C][Kp] e4m3, Kp = mx_cols_kp(R) (R rounded up to 64; padding tokens are zeros) + scales
// for C rows and K = Kp (mx_scale_bytes(C, Kp)): the MX quantization of the padded transpose
void quantize_mx_cols_bf16(uint8_t* q, uint8_t* sl, const bf16_t* x, long long R, int C, long long ldx, hipStream_t s);
// `count` matrices xs elements apart -> outputs qs / ss bytes apart
void quantize_mx_cols_batched_bf16(uint8_t* q, uint8_t* sl, const bf16_t* x, long long R, int C, long long ldx,
                                   int count, long long xs, long long qs, long long ss, hipStream_t s);
// both forms in one read: qr [R][C] (row stride C) + row scales, and the column form of tokens
// [tok_off, tok_off + ntok) of qc [C][ldqc] + its scales (false + set_error on a bad shape)
bool quantize_mx_rowcol_bf16(uint8_t* qr, uint8_t* slr, uint8_t* qc, uint8_t* slc, const bf16_t* x, long long R,
                             int C, long long ldx, long long ldqc, long long tok_off, long long ntok, hipStream_t s);
long long mx_cols_kp(long long R);
long long mx_rows_padded(long long rows);
size_t mx_scale_bytes(long long rows, int K);
// LayerNorm forward into both MX forms (no bf16 tensor): qr/slr as quantize_mx_rowcol_bf16's row
// form of ln_forward_bf16's output, qc/slc its column form over [tok_off, tok_off + ntok)
bool ln_forward_mx_supported(int C);
// LayerNorm backward of the bf16 + lo8 residual-gradient stream (as ln_backward_bf16_stream, part rows
// [ln_bwd_blocks(R)][2C | 3C] or, part == nullptr, reduced into dw / db / dres_colsum) plus both MX
// forms of its bf16 plane (as quantize_mx_rowcol_bf16); C a multiple of 256 up to 1280
bool ln_backward_mx_supported(int C);
bool ln_backward_bf16_stream_mx(bf16_t* dres_out, uint8_t* lo_out, const bf16_t* dres_in, const uint8_t* lo_in,
                                float* dw, float* db, float* dres_colsum, const bf16_t* dout, const float* inp,
                                const float* w, const float* mean, const float* rstd, long long R, int C,
                                hipStream_t s, float* part, uint8_t* qr, uint8_t* slr, uint8_t* qc, uint8_t* slc,
                                long long ldqc, long long tok_off, long long ntok, uint8_t* scratch);
// bytes of the scratch ln_backward_bf16_stream_mx needs (nullptr there: the thread workspace; a caller
// with work in flight on other streams passes its own)
size_t ln_backward_mx_scratch_bytes(int C);
// scratch: ln_mx_scratch_bytes(C) (the last partial round's rows; nullptr: no leftover path, every
// tile through the LDS-tile kernel)
bool ln_forward_mx(uint8_t* qr, uint8_t* slr, uint8_t* qc, uint8_t* slc, float* mean, float* rstd, const float* x,
                   const float* w, const float* b, long long R, int C, long long ldqc, long long tok_off, long long ntok,
                   hipStream_t s, uint8_t* scratch);
size_t ln_mx_scratch_bytes(int C);

// column sums: dbias[n] += sum_m X[m*ld + n]   (X fp32 or bf16), in a fixed order: one pass when
// M <= 256, else per-256-row partial rows in ws (nullptr = thread workspace; cdiv(M,256) * N
// floats) + rows_reduce_add
void colsum_f32(float* dbias, const float* X, int M, int N, long long ld, hipStream_t s, float* ws = nullptr);
void colsum_bf16(float* dbias, const bf16_t* X, int M, int N, long long ld, hipStream_t s, float* ws = nullptr);
// dst[c] += sum_{r < nrows} src[r * ld + c] for c < ncols, the rows added in a fixed order
// (deterministic): the final step of every partial-row reduction (bias / LayerNorm gradients)
struct RowsJob {
    float* dst;
    const float* src;
    int nrows;
    long long ld;
    int ncols;
};
constexpr int ROWS_MAX_JOBS = 8;
void rows_reduce_add(const RowsJob* jobs, int njobs, hipStream_t s);

}  // namespace vit
