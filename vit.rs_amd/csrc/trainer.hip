// trainer.hip — native ViT training step (include/vit_trainer.h).
//
// Host orchestration of the reference's ViT::forward / ViT::backward / optimizer_step
// (/root/reference/train_vit.rs:188-373, 737-743) over the HIP kernels of this library, with
//   * one device arena for params and one for grads, layer-major in REVERSE layer order
//     [head | layer L-1 | ... | layer 0 | embed] so backward finalises one contiguous range per
//     layer; tensors 256-B aligned;
//   * a bf16 shadow of the params (GEMM operands), refreshed by the fused SGD kernel;
//   * data parallelism: one process per GPU, RCCL all-reduce (sum) of each finished gradient
//     chunk on a side stream, ordered by events, overlapped with the rest of backward;
//   * optional per-kernel-class HIP-event timing on the compute stream.
#include <rccl/rccl.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ops_internal.h"
#include "../../include/vit_trainer.h"
#include "../../include/vit_checkpoint.h"
#include "../../include/vit_data.h"
#include "../../include/vit_jpeg.h"

namespace vit {
// jpeg.hip: the JPEG loader's current batch -> device uint8 [B][img][img][3] on st
bool jpeg_loader_decode_to(vit_jpeg_loader_t* l, uint8_t* out, int img, hipStream_t st, const int** labels,
                           int expect_n);
namespace {

enum TIdx {
    P_PATCH_W, P_PATCH_B, P_CLS, P_WPE, P_LN1W, P_LN1B, P_QKVW, P_QKVB, P_ATTPROJW, P_ATTPROJB,
    P_LN2W, P_LN2B, P_FCW, P_FCB, P_FCPROJW, P_FCPROJB, P_LNFW, P_LNFB, P_HEADW, P_HEADB
};

enum TimerClass {
    TC_PATCH, TC_LN_FWD, TC_QKV_FWD, TC_ATTN_FWD, TC_PROJ_FWD, TC_FC_FWD, TC_FCPROJ_FWD, TC_HEAD,
    TC_FCPROJ_DGRAD, TC_FCPROJ_WGRAD, TC_FC_DGRAD, TC_FC_WGRAD, TC_PROJ_DGRAD, TC_PROJ_WGRAD,
    TC_ATTN_BWD, TC_QKV_DGRAD, TC_QKV_WGRAD, TC_LN_BWD, TC_COLSUM, TC_PATCH_BWD, TC_SGD, TC_MISC,
    TC_QUANT, TC_COUNT
};
const char* kTimerNames[TC_COUNT] = {
    "patch_embed_fwd", "layernorm_fwd", "gemm_qkv_fwd", "attention_fwd", "gemm_proj_fwd",
    "gemm_fc_fwd", "gemm_fcproj_fwd", "head", "gemm_fcproj_dgrad", "gemm_fcproj_wgrad",
    "gemm_fc_dgrad", "gemm_fc_wgrad", "gemm_proj_dgrad", "gemm_proj_wgrad", "attention_bwd",
    "gemm_qkv_dgrad", "gemm_qkv_wgrad", "layernorm_bwd", "bias_colsum", "patch_embed_bwd", "sgd",
    "misc", "quantize_mx"};

// out[r][n] = vec[n] for r < rows (the bias start value of a split-K head GEMM)
__global__ void bcast_rows_k(float* __restrict__ out, const float* __restrict__ vec, int rows, int n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < (long long)rows * n) out[i] = vec[i % n];
}
// the CLS rows of a "bf16 + lo8" [B, T, C] tensor (common.h lo8_*) from fp32 rows in[b][c]
__global__ void rows_to_bf16_k(bf16_t* __restrict__ out, uint8_t* __restrict__ lo, long long ldo,
                               const float* __restrict__ in, int rows, int C) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= (long long)rows * C) return;
    const long long b = i / C, o = b * ldo + (i - b * C);
    const bf16_t h = f2bf(in[i]);
    out[o] = h;
    lo[o] = (uint8_t)lo8_encode(in[i], bf2f(h));
}
// dst [rows][n] += src [rows][lds] (its first n columns)
__global__ void add_cols_k(float* __restrict__ dst, const float* __restrict__ src, int rows, int n, int lds) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (long long)rows * n;
         i += (long long)gridDim.x * blockDim.x) {
        const long long r = i / n;
        dst[i] += src[r * lds + (i - r * n)];
    }
}
__global__ void fill_k(float* p, float v, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
// p -= lr*g; pbf = bf16(p)   (optimizer_step, train_vit.rs:737-743, + bf16 shadow)
__global__ void sgd_bf16_k(float* __restrict__ p, bf16_t* __restrict__ pbf,
                           const float* __restrict__ g, long long n, float lr) {
    const long long n4 = n / 4;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
         i += (long long)gridDim.x * blockDim.x) {
        float4 pv = reinterpret_cast<float4*>(p)[i];
        const float4 gv = reinterpret_cast<const float4*>(g)[i];
        pv.x = sgd_update(pv.x, gv.x, lr); pv.y = sgd_update(pv.y, gv.y, lr);
        pv.z = sgd_update(pv.z, gv.z, lr); pv.w = sgd_update(pv.w, gv.w, lr);
        reinterpret_cast<float4*>(p)[i] = pv;
        reinterpret_cast<uint2*>(pbf)[i] = make_uint2(pack_bf16x2(pv.x, pv.y), pack_bf16x2(pv.z, pv.w));
    }
    for (long long i = n4 * 4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        p[i] = sgd_update(p[i], g[i], lr);
        pbf[i] = f2bf(p[i]);
    }
}
// AdamW over the whole arena (oracle ref_adamw_step), + the bf16 shadow.  One
// pass: reads p, g, m, v and writes p, m, v (+ pbf) = 7 x 4 B (+2 B) per parameter, HBM-bound.
__global__ void adamw_k(float* __restrict__ p, bf16_t* __restrict__ pbf, const float* __restrict__ g,
                        float* __restrict__ m, float* __restrict__ v, long long n, float lr, float b1,
                        float b2, float omb1, float omb2, float bc1, float bc2, float eps, float wd) {
    const long long n4 = n / 4;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
         i += (long long)gridDim.x * blockDim.x) {
        float4 pv = reinterpret_cast<float4*>(p)[i];
        const float4 gv = reinterpret_cast<const float4*>(g)[i];
        float4 mv = reinterpret_cast<float4*>(m)[i];
        float4 vv = reinterpret_cast<float4*>(v)[i];
        pv.x = adamw_update(pv.x, gv.x, mv.x, vv.x, lr, b1, b2, omb1, omb2, bc1, bc2, eps, wd);
        pv.y = adamw_update(pv.y, gv.y, mv.y, vv.y, lr, b1, b2, omb1, omb2, bc1, bc2, eps, wd);
        pv.z = adamw_update(pv.z, gv.z, mv.z, vv.z, lr, b1, b2, omb1, omb2, bc1, bc2, eps, wd);
        pv.w = adamw_update(pv.w, gv.w, mv.w, vv.w, lr, b1, b2, omb1, omb2, bc1, bc2, eps, wd);
        reinterpret_cast<float4*>(p)[i] = pv;
        reinterpret_cast<float4*>(m)[i] = mv;
        reinterpret_cast<float4*>(v)[i] = vv;
        if (pbf)
            reinterpret_cast<uint2*>(pbf)[i] = make_uint2(pack_bf16x2(pv.x, pv.y), pack_bf16x2(pv.z, pv.w));
    }
    for (long long i = n4 * 4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        p[i] = adamw_update(p[i], g[i], m[i], v[i], lr, b1, b2, omb1, omb2, bc1, bc2, eps, wd);
        if (pbf) pbf[i] = f2bf(p[i]);
    }
}
// top-1 of each logits row (first index among equal maxima, as numpy.argmax) and the count of
// rows whose prediction equals the label (eval path).  One wave per row.
__global__ void argmax_rows_k(int* __restrict__ pred, int* __restrict__ correct,
                              const float* __restrict__ logits, const int* __restrict__ labels,
                              int B, int NC) {
    const int row = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64, lane = threadIdx.x & 63;
    if (row >= B) return;
    const float* x = logits + (long long)row * NC;
    float best = -INFINITY;
    int bi = NC;  // sentinel above every real index
    for (int j = lane; j < NC; j += 64) {
        const float xv = x[j];
        if (xv > best || bi == NC) { best = xv; bi = j; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (oi < NC && (bi == NC || ob > best || (ob == best && oi < bi))) { best = ob; bi = oi; }
    }
    if (lane == 0) {
        pred[row] = bi;
        if (labels && bi == labels[row]) atomicAdd(correct, 1);
    }
}
// input pipeline: uint8 HWC images -> normalised fp32 CHW pixels, and the
// labels out of the staging buffer.  One thread per pixel: 3 B read, 3 x 4 B written (each channel
// plane coalesced across the wave).  pixel = (x / 255 - mean[c]) / std[c], correctly rounded.
__global__ void normalize_u8_k(float* __restrict__ px, int* __restrict__ lab_out,
                               const unsigned char* __restrict__ u8, const int* __restrict__ lab_in,
                               int B, int HW, float m0, float m1, float m2, float s0, float s1,
                               float s2) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (lab_in && i < B) lab_out[i] = lab_in[i];
    if (i >= (long long)B * HW) return;
    const long long b = i / HW, pix = i - b * HW;
    const unsigned char* src = u8 + i * 3;
    float* dst = px + b * 3 * HW + pix;
    dst[0] = ((float)src[0] / 255.0f - m0) / s0;
    dst[HW] = ((float)src[1] / 255.0f - m1) / s1;
    dst[2 * HW] = ((float)src[2] / 255.0f - m2) / s2;
}
__global__ void to_bf16_k(bf16_t* __restrict__ out, const float* __restrict__ in, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        out[i] = f2bf(in[i]);
}

// Device arena layout (no GPU needed; vit_layout_query exposes it): layer-major in REVERSE layer
// order [head | layer L-1 | ... | layer 0 | embed], each tensor 64-element aligned, so backward
// finalises one contiguous range per layer.  off[ti*L + l] = element offset of tensor ti, layer l
// (unlayered tensors: l = 0); chunk c = [chunk_off[c], chunk_off[c+1]): c = 0 head + final LN,
// 1..L layers L-1..0 (backward's completion order), L+1 embedding.
void compute_layout(int C, int L, int T, int KP, int NC, long long (&canon_size)[20], long long& n_params,
                    std::vector<long long>& off, long long (&chunk_off)[VIT_MAX_LAYERS + 3], int& n_chunks, long long& arena_elems) {
    const long long C_ = C, K = KP;
    const long long sz[20] = {C_ * K, C_, C_, (long long)T * C_,
                              L * C_, L * C_, L * 3 * C_ * C_, L * 3 * C_, L * C_ * C_, L * C_,
                              L * C_, L * C_, L * 4 * C_ * C_, L * 4 * C_, L * C_ * 4 * C_, L * C_,
                              C_, C_, (long long)NC * C_, NC};
    n_params = 0;
    for (int i = 0; i < 20; i++) {
        canon_size[i] = sz[i];
        n_params += sz[i];
    }
    off.assign(20 * L, 0);
    long long cur = 0;
    auto place = [&](int ti, int l, long long n) {
        off[ti * L + l] = cur;
        cur += (n + 63) & ~63LL;
    };
    n_chunks = L + 2;
    chunk_off[0] = 0;
    const int head[4] = {P_HEADW, P_HEADB, P_LNFW, P_LNFB};
    for (int ti : head) place(ti, 0, canon_size[ti]);
    chunk_off[1] = cur;
    for (int c = 1; c <= L; c++) {
        const int l = L - c;
        for (int ti = P_LN1W; ti <= P_FCPROJB; ti++) place(ti, l, canon_size[ti] / L);
        chunk_off[c + 1] = cur;
    }
    const int emb[4] = {P_PATCH_W, P_PATCH_B, P_CLS, P_WPE};
    for (int ti : emb) place(ti, 0, canon_size[ti]);
    chunk_off[L + 2] = cur;
    arena_elems = cur;
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

}  // namespace

struct Trainer {
    vit_config_t cfg{};
    int B = 0, T = 0, NP = 0, C = 0, L = 0, NH = 0, NC = 0, KP = 0, prec = 0, device = 0;
    long long BT = 0;
    long long n_params = 0;       // canonical count
    long long arena_elems = 0;    // device arena (with alignment padding)
    long long canon_size[20]{};
    // device offsets: tensor ti, layer l (l=0 for unlayered)
    std::vector<long long> off;   // [20 * L]
    long long chunk_off[VIT_MAX_LAYERS + 3]{};  // chunk c: [chunk_off[c], chunk_off[c+1]) ; c=0 head, 1..L layers L-1..0, L+1 embed
    int n_chunks = 0;

    hipStream_t s = nullptr, s_comm = nullptr;
    // backward weight-gradient stream: the wgrad GEMMs of a layer run beside the dgrad / LN /
    // attention kernels of the main stream (they only read activations and write grads)
    hipStream_t s2 = nullptr;
    bool two_streams = true;
    enum BwdEv { EV_RESA, EV_RESB, EV_DFCH, EV_DQKV, EV_W1, EV_W2, EV_W3, EV_W4, EV_JOIN, EV_SG, EV_PRE_IN, EV_PRE, EV_COUNT };
    hipEvent_t bev[EV_COUNT]{};
    // micro-batches: the batch is processed as NMB row ranges on NMB streams (ms[0] = s), so the
    // kernels of one half (GEMM epilogue bursts, LayerNorm, attention) overlap the other's GEMM
    // main loops; wgrads (on s2) still reduce over the whole batch
    static constexpr int MAXMB = 4;
    int nmb = 1, mb_want = 2;
    int pick_nmb(int want) const {
        if (!two_streams) return 1;
        for (int k = want < MAXMB ? want : MAXMB; k >= 2; k--)
            if (B % k == 0) return k;
        return 1;
    }
    hipStream_t ms[MAXMB]{};
    hipEvent_t mev[MAXMB][EV_COUNT]{};
    hipEvent_t fork_ev = nullptr, join_ev[MAXMB]{};
    std::vector<hipEvent_t> chunk_evm;
    std::vector<hipEvent_t> chunk_ev2;
    std::vector<hipEvent_t> chunk_ev;
    hipEvent_t comm_done = nullptr;

    float* params = nullptr;
    float* grads = nullptr;
    float* gemm_ws = nullptr;     // split-K slabs of the wgrad GEMMs (stream-ordered on s)
    // GEMM variant 10 (split tail round): fp32 partial tiles, one buffer per concurrent stream
    // (ms[0..MAXMB-1], s2): 256 x 256 KiB at most per GEMM (gemm.hip launch_g2)
    float* tail_buf[MAXMB + 1]{};
    size_t tail_bytes = 0;
    float* attn_part = nullptr;   // per-(b,h) qkv-bias partial sums of the attention backward
    size_t gemm_ws_bytes = 0;
    bf16_t* pbf = nullptr;
    bf16_t* pbfT = nullptr;  // same offsets as pbf; only the four layer weight tensors are used
    float* pixels = nullptr;
    int* labels = nullptr;
    bool has_targets = true;  // false after set_batch without labels: forward only (:264-266)
    int* preds = nullptr;     // eval: [B] top-1 + one counter
    // uint8 upload: double-buffered device staging filled on s_copy, normalised on s
    hipStream_t s_copy = nullptr;
    unsigned char* u8_stage[2]{};
    int* lab_stage[2]{};
    hipEvent_t u8_copied[2]{}, u8_used[2]{};
    int u8_k = 0;
    // AdamW state (allocated on the first AdamW step / a checkpoint load with optimizer state)
    float *adam_m = nullptr, *adam_v = nullptr;
    int adam_t = 0;
    vit_adamw_t adam_hp{};
    std::vector<DevBuf> allocs;
    size_t dev_bytes = 0;
    int b_global = 0;

    // ---- bf16 activations
    struct LayerActs {
        bf16_t *ln1, *qkv, *atty, *ln2, *fchd, *fchg;  // fchd = gelu'(fc pre-activation), fchg = gelu(.)
        float *ln1_mean, *ln1_rstd, *lse, *res2, *ln2_mean, *ln2_rstd, *res3;
        // fp32-mode extras
        float *ln1f, *qkvf, *attyf, *preatt, *att, *attproj, *ln2f, *fchf, *fchgf, *fcproj;
    };
    std::vector<LayerActs> la;
    float* encoded = nullptr;
    bool patch_f32 = false;  // bf16 mode, KP % 8 != 0 and VIT_PATCH_PAD=0: patch embedding on the fp32 GEMM
    // bf16 / fp8 mode, KP % 8 != 0 (ViT-H/14: 588): the patch GEMMs run on the bf16 engine over
    // KPP = KP rounded up to 64 columns: zero-padded im2col rows, a zero-padded bf16 weight copy
    // (refreshed with the transposed copies) and a padded fp32 weight-gradient scratch whose first
    // KP columns are added to the gradient arena
    bool patch_pad = false;
    int KPP = 0;
    bf16_t* wpatch_pad = nullptr;
    float* dwpatch_pad = nullptr;
    bf16_t* patches_bf = nullptr;
    float* patches_f = nullptr;
    float* emb_tmp = nullptr;
    float *cls_x = nullptr, *lnf = nullptr, *lnf_mean = nullptr, *lnf_rstd = nullptr;
    float *logits = nullptr, *probs = nullptr, *losses = nullptr;
    // grads scratch
    float *dlosses = nullptr, *dlogits = nullptr, *dlnf = nullptr, *dcls_x = nullptr;
    float *dres_a = nullptr, *dres_b = nullptr, *dln = nullptr;
    float* pos_sums = nullptr;  // [T][C] per-position column sums of the patch-embedding backward
    float* psg_part = nullptr;  // [PSG_CHUNKS][T][C] per-image-chunk partial sums of the same
    uint8_t *dres_lo = nullptr, *dres_lo2 = nullptr;  // lo8 planes of the bf16 residual-gradient stream
    // deterministic small gradients (no float atomics): stream-s scratch for the fixed-order column
    // sums of the head / fp32 path, and in bf16 / fp8 mode the per-layer partial rows of the
    // micro-batches' LayerNorm (dw | db | next bias), fc-bias and qkv-bias sums, double-buffered by
    // layer parity and reduced once per layer on the weight-gradient stream (sg_finalize)
    float* red_ws = nullptr;
    float* sg_part[2]{};
    long long sg_ln2 = 0, sg_ln1 = 0, sg_fcb = 0, sg_qkv = 0;  // offsets (floats) in sg_part[p]
    int fcb_rows = 0;  // fc-bias column-sum partial rows per micro-batch (gemm_colsum_rows of the fcproj dgrad)
    bf16_t* dln_bf = nullptr;  // bf16 mode: LN-output gradient from the fc / qkv dgrad GEMMs
    bf16_t *dres_bf = nullptr, *dres_bf2 = nullptr, *dfch = nullptr, *datty = nullptr, *dqkv = nullptr, *dpatch_bf = nullptr;
    float* dpatch_f = nullptr;
    // fp32-mode per-layer grad scratch (one layer, zeroed per layer)
    float *g_block = nullptr;
    long long g_block_elems = 0;
    float *g_dres2, *g_dfcproj, *g_dfchg, *g_dfch, *g_dln2, *g_dattproj, *g_datty, *g_dpreatt,
        *g_datt, *g_dqkv, *g_dln1;

    // ---- DP
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1, overlap = 1;
    // option "dp_probe": each chunk is also copied, on s_comm right after its all-reduce, into this
    // snapshot arena (same layout as grads): snapshot == final grads bitwise proves every chunk
    // was final when the comm stream reduced it (at world 1 the sum itself is an identity)
    float* dp_snap = nullptr;
    bool dp_probe_on = false;

    // ---- timing
    bool timing = false;
    struct Rec { int cls; hipEvent_t a, b; hipStream_t st; };
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    std::vector<Rec> recs;
    double t_ms[TC_COUNT]{};
    long long t_calls[TC_COUNT]{};
    double t_flops[TC_COUNT]{};

    // ------------------------------------------------------------------------------
    template <typename TT>
    TT* alloc(long long elems) {
        size_t bytes = (size_t)std::max<long long>(elems, 1) * sizeof(TT);
        bytes = (bytes + 255) & ~(size_t)255;
        void* p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) {
            set_error("trainer: hipMalloc(%zu) failed", bytes);
            return nullptr;
        }
        allocs.push_back({p, bytes});
        dev_bytes += bytes;
        return (TT*)p;
    }

    bool layered(int ti) const { return ti >= P_LN1W && ti <= P_FCPROJB; }
    bool lowp() const { return prec != VIT_FP32; }  // bf16 or fp8 mode (the fast path)
    bool fp8() const { return prec == VIT_FP8; }
    // ---- fp8 mode: MXFP8 copies of the four layer weights (forward B operand, [N][K]) and of their
    // transposes (input-gradient B operand, [Cin][OC]), refreshed after every optimizer step, and
    // per-micro-batch scratch for the quantized A operand of each fp8 GEMM
    static constexpr int NWK = 4;
    const int wkinds[NWK] = {P_QKVW, P_ATTPROJW, P_FCW, P_FCPROJW};
    struct QMat { uint8_t* q = nullptr; uint8_t* s = nullptr; };
    QMat wq[NWK], wtq[NWK];            // [L] matrices each, in the source's memory order
    long long wq_n[NWK]{}, wq_k[NWK]{};  // forward view: N x K per layer
    uint8_t* act_q[4]{};
    uint8_t* act_s[4]{};
    // fused MX outputs (fp8 mode): the GELU output of fc fwd / the GELU' output of fcproj dgrad,
    // written by those GEMMs' epilogues and read as the next GEMM's A operand (VIT_FP8_FUSE=0
    // quantizes them in separate passes instead, for A/B)
    uint8_t* act_q2[4]{};
    uint8_t* act_s2[4]{};
    bool fuse_mx = true;
    // fp8 weight gradients (VIT_FP8_WGRAD=0: bf16 as before): dout and inp quantized column-wise
    // (MX blocks of 32 consecutive tokens: the axis the weight gradient reduces over) into [OC][Kp] /
    // [Cin][Kp] e4m3 rows on the weight-gradient stream, then the MXFP8 engine with K-split slabs
    bool fp8_wgrad = true;
    bool wt_cols = true;  // fp8: the dgrads' MX weight copy by column-quantizing W (VIT_FP8_WT_COLS=0: transpose + rows)
    QMat wg_a, wg_b;  // column-quantized dout / inp of the running weight gradient (stream-ordered)
    // fused row+column quantization (quantize_mx_rowcol_bf16): the column forms of ln1, atty, ln2
    // per layer (written by the forward GEMMs' quantize step, read by the backward's weight
    // gradients) and of dres3, dres2, dqkv (written by the input-gradient GEMMs' quantize step on
    // the micro-batch streams, read by the next weight gradient on s2; the waits that already
    // order dres / dqkv reuse order these too)
    bool rowcol_ok = false;
    long long kp_tok = 0;  // mx_cols_kp(B*T)
    QMat actc[3], dcol[3];
    // ... and of the 4C-wide GELU output (fc fwd epilogue, per layer) and its gradient dfch (fcproj
    // dgrad epilogue): with those and the row forms fused too (fuse_mx), neither bf16 tensor is
    // stored (GemmArgs::mxc_q; nothing else reads them in fp8 mode)
    QMat fchgc, dfchc;
    bool rowcol_on() const { return fp8() && rowcol_ok && ((long long)(B / nmb) * T) % 64 == 0; }
    bool epicol_on() const { return rowcol_on() && fuse_mx && (4 * C) % 64 == 0; }
    // fp8: LayerNorm forward straight into the MX forms (ln_forward_mx; VIT_FP8_LN_MX=0: bf16 + rowcol)
    bool ln_mx = true;
    bool lnmx_on() const { return rowcol_on() && ln_mx && ln_forward_mx_supported(C); }
    // fp8: the residual-gradient LayerNorm backwards also write both MX forms of dres2 / dres3
    // (ln_backward_bf16_stream_mx; VIT_FP8_LNB_MX=0 / option fp8_lnb_mx: the rowcol quantize instead)
    bool lnb_mx = true;
    // option fp8_ln_leftover: the LayerNorm -> MX forward's leftover-row path.  Alone 36.4 -> 32.5 us per
    // ViT-H/14 micro-batch (tools/bench_lnmx.py), in the step 119.70 vs 119.47 ms without it (the other
    // micro-batch stream already fills the partial round): off
    bool ln_left = false;
    uint8_t* lnb_scr[4]{};  // per micro-batch stream: the LayerNorm -> MX kernels' scratch (ln_mx_scratch_bytes)
    bool lnbmx_on() const { return rowcol_on() && lnb_mx && ln_backward_mx_supported(C); }
    // the column-form span of micro-batch mb (R rows): the last one carries the padding tokens
    long long mb_ntok(int mb, long long R) const { return mb == nmb - 1 ? kp_tok - (long long)mb * R : R; }
    QMat fchgc_of(int l) const {
        return {fchgc.q + (long long)l * 4 * C * kp_tok, fchgc.s + (long long)l * mx_scale_bytes(4LL * C, (int)kp_tok)};
    }
    QMat actc_of(int k, int l) const {
        return {actc[k].q + (long long)l * C * kp_tok, actc[k].s + (long long)l * mx_scale_bytes(C, (int)kp_tok)};
    }
    int wslot(int k, int l) const {    // memory-order index of layer l's copy of weight kind k
        const long long stride = L > 1 ? off[wkinds[k] * L + 1] - off[wkinds[k] * L] : 0;
        return stride < 0 ? L - 1 - l : l;
    }
    int wkind_of(int ti) const {
        for (int k = 0; k < NWK; k++) if (wkinds[k] == ti) return k;
        return -1;
    }
    long long per_layer(int ti) const { return canon_size[ti] / L; }
    float* P(int ti, int l = 0) const { return params + off[ti * L + l]; }
    float* G(int ti, int l = 0) const { return grads + off[ti * L + l]; }
    bf16_t* W(int ti, int l = 0) const { return pbf + off[ti * L + l]; }
    // transposed bf16 copy of a layer weight ([Cin][OC]): the dgrad GEMMs read it K-contiguous
    bf16_t* WT(int ti, int l = 0) const { return pbfT + off[ti * L + l]; }
    bool dgrad_wt = true;  // option "dgrad_transposed": dgrad B operand from pbfT (K-contig)
    // dgrad B operand: the transposed copy (K-contiguous, ldb = OC) or W itself (N-contiguous)
    void dgrad_b(GemmArgs& g, int ti, int l, int OC, int Cin) const {
        if (dgrad_wt) { g.B = WT(ti, l); g.ldb = OC; g.b_kcontig = true; }
        else { g.B = W(ti, l); g.ldb = Cin; g.b_kcontig = false; }
    }

    void build_layout() {
        compute_layout(C, L, T, KP, NC, canon_size, n_params, off, chunk_off, n_chunks, arena_elems);
    }

    // canonical <-> device copies (host staging)
    void canon_to_device(const float* host, float* dev) {
        pre_side_wait();  // (the arena clear / transposes on s2 must not race this copy)
        std::vector<float> stage((size_t)arena_elems, 0.f);
        long long c = 0;
        for (int ti = 0; ti < 20; ti++) {
            if (layered(ti)) {
                const long long n = per_layer(ti);
                for (int l = 0; l < L; l++, c += n) memcpy(&stage[off[ti * L + l]], host + c, n * 4);
            } else {
                memcpy(&stage[off[ti * L]], host + c, canon_size[ti] * 4);
                c += canon_size[ti];
            }
        }
        VIT_HIP(hipMemcpyAsync(dev, stage.data(), arena_elems * 4, hipMemcpyHostToDevice, s));
        VIT_HIP(hipStreamSynchronize(s));
    }
    void device_to_canon(const float* dev, float* host) {
        pre_side_wait();
        std::vector<float> stage((size_t)arena_elems);
        VIT_HIP(hipMemcpyAsync(stage.data(), dev, arena_elems * 4, hipMemcpyDeviceToHost, s));
        VIT_HIP(hipStreamSynchronize(s));
        long long c = 0;
        for (int ti = 0; ti < 20; ti++) {
            if (layered(ti)) {
                const long long n = per_layer(ti);
                for (int l = 0; l < L; l++, c += n) memcpy(host + c, &stage[off[ti * L + l]], n * 4);
            } else {
                memcpy(host + c, &stage[off[ti * L]], canon_size[ti] * 4);
                c += canon_size[ti];
            }
        }
    }

    // ---- timing helpers
    void tbeg(int cls, double flops, hipStream_t st = nullptr) {
        if (!timing) return;
        if (!st) st = s;
        if (ev_used + 2 > ev_pool.size()) {
            for (int k = 0; k < 64; k++) {
                hipEvent_t e;
                VIT_HIP(hipEventCreate(&e));
                ev_pool.push_back(e);
            }
        }
        Rec r{cls, ev_pool[ev_used], ev_pool[ev_used + 1], st};
        ev_used += 2;
        VIT_HIP(hipEventRecord(r.a, st));
        recs.push_back(r);
        t_flops[cls] += flops;
    }
    void tend() {
        if (!timing) return;
        VIT_HIP(hipEventRecord(recs.back().b, recs.back().st));
    }
    void collect() {
        if (recs.empty()) return;
        VIT_HIP(hipStreamSynchronize(s));
        VIT_HIP(hipStreamSynchronize(s2));
        for (int k = 1; k < MAXMB; k++) VIT_HIP(hipStreamSynchronize(ms[k]));
        for (auto& r : recs) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
                t_ms[r.cls] += ms;
                t_calls[r.cls] += 1;
            }
        }
        recs.clear();
        ev_used = 0;
    }

    // the stream's own partial-tile buffer for GEMM variant 10 (never the shared thread workspace:
    // the micro-batch streams run GEMMs concurrently)
    void set_tail(GemmArgs& a, hipStream_t st) {
        if (a.tail_ws || !tail_bytes) return;
        int k = MAXMB;  // s2
        for (int i = 0; i < MAXMB; i++)
            if (st == ms[i]) k = i;
        a.tail_ws = tail_buf[k];
        a.tail_ws_bytes = tail_bytes;
    }
    void gemm(int cls, GemmArgs a, bool bf, hipStream_t st = nullptr) {
        if (!st) st = s;
        if (bf) set_tail(a, st);
        tbeg(cls, 2.0 * a.M * (double)a.N * a.K, st);
        if (bf) gemm_bf16(a, st); else gemm_f32(a, st);
        tend();
    }
    // fork the micro-batch streams off s / join them back into s
    void mb_fork() {
        if (nmb < 2) return;
        VIT_HIP(hipEventRecord(fork_ev, s));
        for (int k = 1; k < nmb; k++) VIT_HIP(hipStreamWaitEvent(ms[k], fork_ev, 0));
    }
    void mb_join() {
        for (int k = 1; k < nmb; k++) {
            VIT_HIP(hipEventRecord(join_ev[k], ms[k]));
            VIT_HIP(hipStreamWaitEvent(s, join_ev[k], 0));
        }
    }

    // ------------------------------------------------------------------------------
    bool init(const vit_config_t* c, int batch, int precision, int dev) {
        cfg = *c;
        B = batch;
        C = c->channels; L = c->num_layers; NH = c->num_heads; NC = c->num_classes;
        NP = (c->img / c->patch) * (c->img / c->patch);
        T = NP + 1;
        KP = 3 * c->patch * c->patch;
        BT = (long long)B * T;
        prec = precision;
        device = dev;
        if (c->in_ch != 3 || C % NH || L < 1 || L > VIT_MAX_LAYERS || B < 1 || prec < VIT_FP32 || prec > VIT_FP8) {
            set_error("trainer: unsupported config");
            return false;
        }
        if (prec == VIT_FP8 && C % 64) {
            set_error("trainer: fp8 mode needs C %% 64 == 0 (MX k-steps of 64), C=%d", C);
            return false;
        }
        if (hipSetDevice(dev) != hipSuccess) { set_error("trainer: hipSetDevice(%d)", dev); return false; }
        // stream priorities (VIT_STREAM_PRIO overrides): 1 = micro-batch streams high, weight-gradient
        // stream low; 2 = the reverse; 0 = all equal.  Measured (bench.py, three interleaved rounds each,
        // profiles/r06_stream_prio.txt): ViT-B/16 bf16 2 vs 0: 7102-7106 vs 7059-7062 img/s (+0.65 %),
        // 1: -0.2 %; ViT-H/14 fp8 2 vs 0: 1088 vs 1098 img/s (-0.8 %), 1: -2 %.  So 2 in bf16 mode and
        // 0 in fp8 (a measured choice: which stream's kernels fill the others' partial rounds)
        int prio_mode = prec == VIT_BF16 ? 2 : 0, p_lo = 0, p_hi = 0;
        {
            const char* e = getenv("VIT_STREAM_PRIO");
            if (e) prio_mode = atoi(e);
            if (prio_mode) VIT_HIP(hipDeviceGetStreamPriorityRange(&p_lo, &p_hi));
        }
        // (3 / 4, A/B only: micro-batch stream 0 high and 1 low, the weight-gradient stream high / low)
        auto mk_stream = [&](hipStream_t* st, int role) {  // role: 0 = micro-batch 0, 1 = other micro-batch, 2 = wgrad
            if (!prio_mode) {
                VIT_HIP(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
            } else {
                bool hi;
                if (prio_mode == 1) hi = role != 2;
                else if (prio_mode == 2) hi = role == 2;
                else hi = role == 0 || (role == 2 && prio_mode == 3);
                VIT_HIP(hipStreamCreateWithPriority(st, hipStreamNonBlocking, hi ? p_hi : p_lo));
            }
        };
        mk_stream(&s, 0);
        VIT_HIP(hipStreamCreateWithFlags(&s_comm, hipStreamNonBlocking));
        mk_stream(&s2, 2);
        {
            const char* e = getenv("VIT_BWD_STREAMS");
            two_streams = !(e && atoi(e) == 1);
        }
        for (auto& e : bev) VIT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ms[0] = s;
        for (int k = 1; k < MAXMB; k++) mk_stream(&ms[k], 1);
        for (auto& row : mev)
            for (auto& e : row) VIT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        VIT_HIP(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
        for (auto& e : join_ev) VIT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        {
            const char* e = getenv("VIT_MICROBATCH");
            mb_want = e ? atoi(e) : 2;
            nmb = pick_nmb(mb_want);
        }
        chunk_evm.resize((size_t)(L + 2) * MAXMB);
        for (auto& e : chunk_evm) VIT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        chunk_ev.resize(L + 2);
        for (auto& e : chunk_ev) VIT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        chunk_ev2.resize(L + 2);
        for (auto& e : chunk_ev2) VIT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        VIT_HIP(hipEventCreateWithFlags(&comm_done, hipEventDisableTiming));
        build_layout();
        params = alloc<float>(arena_elems);
        grads = alloc<float>(arena_elems);
        pixels = alloc<float>((long long)B * 3 * c->img * c->img);
        labels = alloc<int>(B);
        preds = alloc<int>(B + 1);
        encoded = alloc<float>(BT * C);
        cls_x = alloc<float>((long long)B * C);
        lnf = alloc<float>((long long)B * C);
        lnf_mean = alloc<float>(B);
        lnf_rstd = alloc<float>(B);
        logits = alloc<float>((long long)B * NC);
        probs = alloc<float>((long long)B * NC);
        losses = alloc<float>(B);
        dlosses = alloc<float>(B);
        dlogits = alloc<float>((long long)B * NC);
        dlnf = alloc<float>((long long)B * C);
        dcls_x = alloc<float>((long long)B * C);
        if (!lowp()) {  // the bf16 / fp8 residual-gradient stream is bf16 (dres_bf / dres_bf2)
            dres_a = alloc<float>(BT * C);
            dres_b = alloc<float>(BT * C);
        }
        pos_sums = alloc<float>((long long)T * C);
        if (lowp()) psg_part = alloc<float>((long long)PSG_CHUNKS * T * C);
        {  // column-sum / LayerNorm partial rows on s (head, fp32 path)
            const long long a1 = (long long)ln_bwd_blocks(BT) * 2 * C;
            const long long a2 = (long long)cdiv(BT, 256) * std::max(4 * C, NC);
            red_ws = alloc<float>(std::max(a1, a2));
        }
        emb_tmp = alloc<float>((long long)B * NP * C);
        la.resize(L);
        if (!lowp()) {  // the fp32 engine's split-K slabs (<= ~16 MB: splits x tiles <= 1024 tiles of 64 x 64)
            gemm_ws_bytes = (size_t)32 << 20;
            gemm_ws = alloc<float>((long long)(gemm_ws_bytes / sizeof(float)));
        }
        if (lowp() && gemm_variant_selected() == 10) {  // (A/B runs only: VIT_GEMM=10 at build time)
            tail_bytes = (size_t)gemm_cu_count() * 256 * 256 * sizeof(float);
            for (int k = 0; k <= MAXMB; k++) tail_buf[k] = alloc<float>((long long)(tail_bytes / sizeof(float)));
        }
        if (lowp()) {
            if (!(attn_fused_supported(T, C, NH) || attn_generic_supported(T, C, NH)) || C % 8) {
                set_error("trainer: bf16 / fp8 path needs head size 32, 64, 80, 96 or 128 and C %% 8 == 0 (T=%d C=%d NH=%d)", T, C, NH);
                return false;
            }
            // a patch whose im2col row (3*P*P) is not a multiple of 8 bf16 (ViT-H/14: 588) cannot
            // feed the bf16 GEMM's 16-B loads as it is: padded to KPP columns (the fp32 GEMM from
            // the fp32 master weights with VIT_PATCH_PAD=0, the round-2 form: 3 ms/step at H/14)
            const char* pp = getenv("VIT_PATCH_PAD");
            patch_f32 = KP % 8 != 0 && pp && pp[0] == '0';
            patch_pad = KP % 8 != 0 && !patch_f32;
            KPP = patch_pad ? (KP + 63) / 64 * 64 : KP;
            pbf = alloc<bf16_t>(arena_elems);
            pbfT = alloc<bf16_t>(arena_elems);
            if (patch_f32) {
                patches_f = alloc<float>((long long)B * NP * KP);
                dpatch_f = alloc<float>((long long)B * NP * C);
            } else {
                patches_bf = alloc<bf16_t>((long long)B * NP * KPP);
            }
            if (patch_pad) {
                wpatch_pad = alloc<bf16_t>((long long)C * KPP);
                dwpatch_pad = alloc<float>((long long)C * KPP);
                if (wpatch_pad) VIT_HIP(hipMemset(wpatch_pad, 0, (size_t)C * KPP * 2));
            }
            for (int l = 0; l < L; l++) {
                LayerActs& a = la[l];
                a.ln1 = alloc<bf16_t>(BT * C);
                a.ln1_mean = alloc<float>(BT);
                a.ln1_rstd = alloc<float>(BT);
                a.qkv = alloc<bf16_t>(BT * 3 * C);
                a.atty = alloc<bf16_t>(BT * C);
                a.lse = alloc<float>(BT * NH);
                a.res2 = alloc<float>(BT * C);
                a.ln2 = alloc<bf16_t>(BT * C);
                a.ln2_mean = alloc<float>(BT);
                a.ln2_rstd = alloc<float>(BT);
                a.fchd = alloc<bf16_t>(BT * 4 * C);
                a.fchg = alloc<bf16_t>(BT * 4 * C);
                a.res3 = alloc<float>(BT * C);
            }
            dln_bf = alloc<bf16_t>(BT * C);
            dres_bf = alloc<bf16_t>(BT * C);
            dres_bf2 = alloc<bf16_t>(BT * C);
            dres_lo = alloc<uint8_t>(BT * C);
            dres_lo2 = alloc<uint8_t>(BT * C);
            dfch = alloc<bf16_t>(BT * 4 * C);
            datty = alloc<bf16_t>(BT * C);
            dqkv = alloc<bf16_t>(BT * 3 * C);
            if (!patch_f32) dpatch_bf = alloc<bf16_t>((long long)B * NP * C);
            // slabs: <= 32 splits of the largest weight gradient (4C x C)
            gemm_ws_bytes = (size_t)32 * 4 * C * (size_t)std::max(C, KP) * sizeof(float);
            gemm_ws = alloc<float>((long long)(gemm_ws_bytes / sizeof(float)));
            attn_part = alloc<float>((long long)attn_backward_ws_floats(B, T, C, NH) + MAXMB * 3LL * C);  // bias partials | delta
            {  // per-layer small-gradient partial rows for up to MAXMB micro-batches
                const long long lnr = (long long)MAXMB * ln_bwd_blocks(BT), fcr = cdiv(BT, 96) + MAXMB;  // (96: ping-pong engine)
                sg_ln2 = 0;
                sg_ln1 = sg_ln2 + lnr * 3 * C;
                sg_fcb = sg_ln1 + lnr * 3 * C;
                sg_qkv = sg_fcb + fcr * 4 * C;
                const long long n = sg_qkv + (long long)MAXMB * 3 * C;
                sg_part[0] = alloc<float>(n);
                sg_part[1] = alloc<float>(n);
            }
            if (fp8()) {
                const long long ns[NWK] = {3LL * C, C, 4LL * C, C}, ks[NWK] = {C, C, C, 4LL * C};
                for (int k = 0; k < NWK; k++) {
                    wq_n[k] = ns[k];
                    wq_k[k] = ks[k];
                    wq[k].q = alloc<uint8_t>(L * ns[k] * ks[k]);
                    wq[k].s = alloc<uint8_t>((long long)L * mx_scale_bytes(ns[k], (int)ks[k]));
                    wtq[k].q = alloc<uint8_t>(L * ns[k] * ks[k]);
                    wtq[k].s = alloc<uint8_t>((long long)L * mx_scale_bytes(ks[k], (int)ns[k]));
                }
                // A-operand scratch per micro-batch stream: rows x (widest K = 4C) bytes + scales.
                // Stream k runs only when there are > k micro-batches, so it holds at most
                // B/(k+1) images' rows.
                for (int k = 0; k < MAXMB; k++) {
                    const long long rows = (long long)(B / (k + 1)) * T;
                    if (rows <= 0) continue;
                    act_q[k] = alloc<uint8_t>(rows * 4 * C);
                    act_s[k] = alloc<uint8_t>((long long)mx_scale_bytes(rows, 4 * C));
                    act_q2[k] = alloc<uint8_t>(rows * 4 * C);
                    act_s2[k] = alloc<uint8_t>((long long)mx_scale_bytes(rows, 4 * C));
                    // the padding rows' scales (never written by the fused epilogues) stay 0
                    VIT_HIP(hipMemset(act_s2[k], 0, mx_scale_bytes(rows, 4 * C)));
                }
                const char* fe = getenv("VIT_FP8_FUSE");
                fuse_mx = !(fe && fe[0] == '0');
                const char* wc = getenv("VIT_FP8_WT_COLS");
                wt_cols = !(wc && wc[0] == '0') && C % 64 == 0;
                const char* fw = getenv("VIT_FP8_WGRAD");
                fp8_wgrad = !(fw && fw[0] == '0') && C % 64 == 0;
                if (fp8_wgrad) {
                    const long long kp = mx_cols_kp(BT);
                    wg_a.q = alloc<uint8_t>(4LL * C * kp);
                    wg_a.s = alloc<uint8_t>((long long)mx_scale_bytes(4LL * C, (int)kp));
                    wg_b.q = alloc<uint8_t>(4LL * C * kp);
                    wg_b.s = alloc<uint8_t>((long long)mx_scale_bytes(4LL * C, (int)kp));
                    const char* lx = getenv("VIT_FP8_LN_MX");
                ln_mx = !(lx && lx[0] == '0');
                const char* lbx = getenv("VIT_FP8_LNB_MX");
                lnb_mx = !(lbx && lbx[0] == '0');
                const char* rc = getenv("VIT_FP8_ROWCOL");
                    rowcol_ok = !(rc && rc[0] == '0');
                    kp_tok = kp;
                    if (rowcol_ok) {
                        for (int k = 0; k < 3; k++) {
                            actc[k].q = alloc<uint8_t>((long long)L * C * kp);
                            actc[k].s = alloc<uint8_t>((long long)L * mx_scale_bytes(C, (int)kp));
                            const long long w = k == 2 ? 3LL * C : C;
                            dcol[k].q = alloc<uint8_t>(w * kp);
                            dcol[k].s = alloc<uint8_t>((long long)mx_scale_bytes(w, (int)kp));
                        }
                        fchgc.q = alloc<uint8_t>((long long)L * 4 * C * kp);
                        fchgc.s = alloc<uint8_t>((long long)L * mx_scale_bytes(4LL * C, (int)kp));
                        dfchc.q = alloc<uint8_t>(4LL * C * kp);
                        dfchc.s = alloc<uint8_t>((long long)mx_scale_bytes(4LL * C, (int)kp));
                        if (ln_backward_mx_supported(C) || ln_forward_mx_supported(C))
                            for (int k = 0; k < MAXMB; k++) lnb_scr[k] = alloc<uint8_t>((long long)ln_mx_scratch_bytes(C));
                    }
                }
            }
        } else {
            patches_f = alloc<float>((long long)B * NP * KP);
            dpatch_f = alloc<float>((long long)B * NP * C);
            const long long att_n = BT * NH * T;
            for (int l = 0; l < L; l++) {
                LayerActs& a = la[l];
                a.ln1f = alloc<float>(BT * C);
                a.ln1_mean = alloc<float>(BT);
                a.ln1_rstd = alloc<float>(BT);
                a.qkvf = alloc<float>(BT * 3 * C);
                a.attyf = alloc<float>(BT * C);
                a.preatt = alloc<float>(att_n);
                a.att = alloc<float>(att_n);
                a.attproj = alloc<float>(BT * C);
                a.res2 = alloc<float>(BT * C);
                a.ln2f = alloc<float>(BT * C);
                a.ln2_mean = alloc<float>(BT);
                a.ln2_rstd = alloc<float>(BT);
                a.fchf = alloc<float>(BT * 4 * C);
                a.fchgf = alloc<float>(BT * 4 * C);
                a.fcproj = alloc<float>(BT * C);
                a.res3 = alloc<float>(BT * C);
            }
            // one layer of reference grads_acts (train_vit.rs:346-357), zeroed per layer
            const long long sizes[11] = {BT * C, BT * C, BT * 4 * C, BT * 4 * C, BT * C, BT * C,
                                         BT * C, att_n, att_n, BT * 3 * C, BT * C};
            float** slots[11] = {&g_dres2, &g_dfcproj, &g_dfchg, &g_dfch, &g_dln2, &g_dattproj,
                                 &g_datty, &g_dpreatt, &g_datt, &g_dqkv, &g_dln1};
            g_block_elems = 0;
            for (int k = 0; k < 11; k++) g_block_elems += (sizes[k] + 63) & ~63LL;
            g_block = alloc<float>(g_block_elems);
            long long o = 0;
            for (int k = 0; k < 11; k++) {
                *slots[k] = g_block ? g_block + o : nullptr;
                o += (sizes[k] + 63) & ~63LL;
            }
        }
        VIT_HIP(hipMemsetAsync(grads, 0, arena_elems * 4, s));
        VIT_HIP(hipStreamSynchronize(s));
        return !has_error();
    }

    void destroy() {
        if (s_copy) (void)hipStreamSynchronize(s_copy);
        for (int k = 0; k < 2; k++) {
            if (u8_copied[k]) (void)hipEventDestroy(u8_copied[k]);
            if (u8_used[k]) (void)hipEventDestroy(u8_used[k]);
        }
        if (s_copy) (void)hipStreamDestroy(s_copy);
        if (s) (void)hipStreamSynchronize(s);
        if (s_comm) (void)hipStreamSynchronize(s_comm);
        if (s2) (void)hipStreamSynchronize(s2);
        for (int k = 1; k < MAXMB; k++) if (ms[k]) (void)hipStreamSynchronize(ms[k]);
        if (comm) ncclCommDestroy(comm);
        for (auto& a : allocs) (void)hipFree(a.p);
        for (auto e : chunk_ev) (void)hipEventDestroy(e);
        for (auto e : chunk_ev2) (void)hipEventDestroy(e);
        for (auto e : bev) if (e) (void)hipEventDestroy(e);
        for (auto& row : mev)
            for (auto e : row) if (e) (void)hipEventDestroy(e);
        if (fork_ev) (void)hipEventDestroy(fork_ev);
        for (auto e : join_ev) if (e) (void)hipEventDestroy(e);
        for (auto e : chunk_evm) if (e) (void)hipEventDestroy(e);
        for (int k = 1; k < MAXMB; k++) if (ms[k]) (void)hipStreamDestroy(ms[k]);
        for (auto e : ev_pool) (void)hipEventDestroy(e);
        if (comm_done) (void)hipEventDestroy(comm_done);
        if (s) (void)hipStreamDestroy(s);
        if (s_comm) (void)hipStreamDestroy(s_comm);
        if (s2) (void)hipStreamDestroy(s2);
    }

    // side pre-work (option pre_side, bf16 / fp8 with two streams, timing off): the gradient-arena
    // clear and the transposed weight copies run on s2 beside the forward instead of ahead of it on s.
    // pre_side_begin orders s2 after everything enqueued on s so far; pre_side_end records EV_PRE,
    // which s waits for before the backward's first gradient write (backward_bf16)
    bool pre_side = true;
    bool pre_side_on() const { return pre_side && two_streams && lowp() && !timing && s2; }
    hipStream_t pre_side_begin() {
        VIT_HIP(hipEventRecord(bev[EV_PRE_IN], s));
        VIT_HIP(hipStreamWaitEvent(s2, bev[EV_PRE_IN], 0));
        return s2;
    }
    void pre_side_end() {
        VIT_HIP(hipEventRecord(bev[EV_PRE], s2));
        pre_pending = true;
    }
    bool pre_pending = false;
    void pre_side_wait() {
        if (!pre_pending) return;
        VIT_HIP(hipStreamWaitEvent(s, bev[EV_PRE], 0));
        pre_pending = false;
    }
    void refresh_bf16() {
        if (!lowp()) return;
        pre_side_wait();  // an earlier refresh's transposes on s2 still read pbf
        to_bf16_k<<<grid_for(arena_elems, 256), 256, 0, s>>>(pbf, params, arena_elems);
        after_launch("params_to_bf16");
        refresh_transposed();
    }
    // pbfT <- transposes of the layer weights in pbf (after every SGD step): one launch per
    // weight kind over all L layers (the layers of a kind are a constant stride apart)
    void refresh_transposed() {
        const int kinds[4] = {P_QKVW, P_ATTPROJW, P_FCW, P_FCPROJW};
        const int rows[4] = {3 * C, C, 4 * C, C}, cols[4] = {C, C, C, 4 * C};
        tbeg(TC_MISC, 0);
        // bf16 mode: only the backward's dgrads read the transposes, so with side pre-work on they run
        // on s2 beside the next forward (s waits for them at the start of the backward).  fp8 mode
        // keeps them on s: refresh_fp8 below row-quantizes them (VIT_FP8_WT_COLS=0) right away
        const bool side = pre_side_on() && !fp8();
        hipStream_t ts = side ? pre_side_begin() : s;
        // fp8 mode reads no bf16 transposed copy (refresh_fp8 column-quantizes W for the dgrads)
        for (int k = 0; k < 4 && !(fp8() && wt_cols); k++) {
            const long long stride = L > 1 ? off[kinds[k] * L + 1] - off[kinds[k] * L] : 0;
            // negative stride: pass the lowest-addressed layer (layers are stored in reverse)
            const int l0 = stride < 0 ? L - 1 : 0;
            transpose_bf16(WT(kinds[k], l0), W(kinds[k], l0), rows[k], cols[k], L, stride < 0 ? -stride : stride, ts);
        }
        if (side) pre_side_end();
        if (patch_pad)  // the patch weight's padded copy (columns KP .. KPP-1 stay zero)
            VIT_HIP(hipMemcpy2DAsync(wpatch_pad, (size_t)KPP * 2, W(P_PATCH_W), (size_t)KP * 2, (size_t)KP * 2, C,
                                     hipMemcpyDeviceToDevice, s));
        tend();
        if (fp8()) refresh_fp8();
    }
    // MXFP8 weight copies: W [N][K] from the fp32 master, WT [Cin][OC] from the bf16 transpose;
    // one batched launch per kind over the L layers (a constant stride apart in the arena)
    void refresh_fp8() {
        tbeg(TC_QUANT, 0);
        for (int k = 0; k < NWK; k++) {
            const long long stride = L > 1 ? off[wkinds[k] * L + 1] - off[wkinds[k] * L] : 0;
            const int l0 = stride < 0 ? L - 1 : 0;
            const long long as = stride < 0 ? -stride : stride;
            const long long N = wq_n[k], K = wq_k[k];
            quantize_mx_batched_f32(wq[k].q, wq[k].s, P(wkinds[k], l0), N, (int)K, L, as, N * K,
                                    (long long)mx_scale_bytes(N, (int)K), s);
            if (wt_cols)  // Wt's MX rows = W's MX columns: byte-identical, without the bf16 transpose
                quantize_mx_cols_batched_bf16(wtq[k].q, wtq[k].s, W(wkinds[k], l0), N, (int)K, K, L, as, N * K,
                                              (long long)mx_scale_bytes(K, (int)N), s);
            else
                quantize_mx_batched_bf16(wtq[k].q, wtq[k].s, WT(wkinds[k], l0), K, (int)N, L, as, N * K,
                                         (long long)mx_scale_bytes(K, (int)N), s);
        }
        tend();
    }
    QMat wq_of(int ti, int l) const {
        const int k = wkind_of(ti), j = wslot(k, l);
        return {wq[k].q + (long long)j * wq_n[k] * wq_k[k], wq[k].s + (long long)j * mx_scale_bytes(wq_n[k], (int)wq_k[k])};
    }
    QMat wtq_of(int ti, int l) const {
        const int k = wkind_of(ti), j = wslot(k, l);
        return {wtq[k].q + (long long)j * wq_n[k] * wq_k[k], wtq[k].s + (long long)j * mx_scale_bytes(wq_k[k], (int)wq_n[k])};
    }
    // a forward (transposed = false) or input-gradient (true) GEMM of weight ti, layer l: bf16
    // mode as given; fp8 mode quantizes the bf16 A operand into the stream's scratch and runs the
    // MXFP8 engine against the weight's fp8 copy
    // pre: the A operand already in MX form (a fused epilogue wrote it); otherwise it is quantized
    // here.  mx_out: ask this GEMM's epilogue for the MX copy of its bf16 output (fp8 mode, fused)
    // colq: also write the column form of this micro-batch's A rows into colq (rowcol_on());
    // rec_ev: then record micro-batch event rec_ev (the weight gradient that reads colq waits on it)
    // pre: PRE_EPI = in act_q2 (a fused GEMM epilogue wrote it), PRE_LN = in act_q (ln_forward_mx)
    enum { PRE_NONE = 0, PRE_EPI = 1, PRE_LN = 2 };
    void gemm_w(int cls, GemmArgs a, int ti, int l, bool transposed, int mb, hipStream_t st, int pre = PRE_NONE,
                bool mx_out = false, const QMat* colq = nullptr, int rec_ev = -1) {
        if (!fp8()) { gemm(cls, a, true, st); return; }
        if (mx_out) { a.mx_q = act_q2[mb]; a.mx_s = act_s2[mb]; }
        const uint8_t* aq = act_q[mb];
        const uint8_t* as = act_s[mb];
        if (pre == PRE_EPI) {
            aq = act_q2[mb];
            as = act_s2[mb];
        } else if (pre == PRE_NONE) {
            tbeg(TC_QUANT, 0, st);
            if (colq) {
                const long long r0 = (long long)mb * (B / nmb) * T;
                const long long ntok = mb_ntok(mb, a.M);
                quantize_mx_rowcol_bf16(act_q[mb], act_s[mb], colq->q, colq->s, (const bf16_t*)a.A, a.M, a.K, a.lda,
                                        kp_tok, r0, ntok, st);
            } else {
                quantize_mx_bf16(act_q[mb], act_s[mb], (const bf16_t*)a.A, a.M, a.K, a.lda, a.K, st);
            }
            tend();
            if (rec_ev >= 0 && two_streams) VIT_HIP(hipEventRecord(mev[mb][rec_ev], st));
        }
        const QMat w = transposed ? wtq_of(ti, l) : wq_of(ti, l);
        a.A = aq; a.lda = a.K; a.a_scale = as;
        a.B = w.q; a.ldb = a.K; a.b_scale = w.s; a.b_kcontig = true;
        tbeg(cls, 2.0 * a.M * (double)a.N * a.K, st);
        gemm_fp8(a, st);
        tend();
    }

    // ------------------------------------------------------------------ head (both modes)
    // split-K of the M = B head GEMMs (bf16 / fp8 modes): about four 16-deep K-steps per work item.
    // The engine's rule stops at >= 8 K-steps per split (192-256 workgroups of 12-16 dependent
    // K-steps: 20-47 us per GEMM at B = 256, on the critical path between forward and backward);
    // bounded by the slab workspace
    bool head_sk = true;  // option head_splitk (A/B): 0 = the engine's split rule
    // option patch_tail (A/B): the patch embedding backward after the join with its weight gradient
    // split for 80 % of the slots and the small gradients on s2 beside it (0: 45 %, all on s)
    bool patch_tail = true;
    int head_split(int M, int N, int K) const {
        if (!head_sk) return 0;
        int sp = std::min(16, std::max(1, K / 64));
        while (sp > 1 && (size_t)sp * M * N * sizeof(float) > gemm_ws_bytes) sp--;
        return sp;
    }
    void head_forward() {
        tbeg(TC_HEAD, 2.0 * B * C * NC);
        // lnf on the CLS row of each image (D15)
        const float* last = la[L - 1].res3;
        VIT_HIP(hipMemcpy2DAsync(cls_x, C * 4, last, (size_t)T * C * 4, C * 4, B, hipMemcpyDeviceToDevice, s));
        ln_forward_f32(lnf, lnf_mean, lnf_rstd, cls_x, P(P_LNFW), P(P_LNFB), B, C, s);
        GemmArgs a;
        a.A = lnf; a.lda = C; a.B = P(P_HEADW); a.ldb = C; a.C = logits; a.ldc = NC;
        a.bias = P(P_HEADB); a.M = B; a.N = NC; a.K = C; a.epi = EPI_F32_STORE;
        if (lowp()) {
            // fast path: the M = B head GEMMs have 64 output tiles for 256 CUs, so they run
            // split-K through fp32 slabs onto the broadcast bias (fp32 mode keeps the ordered sums)
            bcast_rows_k<<<cdiv((long long)B * NC, 256), 256, 0, s>>>(logits, P(P_HEADB), B, NC);
            a.bias = nullptr;
            a.epi = EPI_F32_ATOMIC;
            a.splitk = head_split(a.M, a.N, a.K);
        }
        a.ws = gemm_ws; a.ws_bytes = gemm_ws_bytes;
        gemm_f32(a, s);
        softmax_rows(probs, logits, B, NC, s);
        if (has_targets) ce_forward(losses, probs, labels, B, NC, s);
        tend();
    }
    // dres_cur (zeroed) <- lnf backward on CLS rows (fp32 dres, or the bf16 stream dres_bf)
    void head_backward(float* dres, bf16_t* dres_bf = nullptr, uint8_t* dres_lo = nullptr) {
        tbeg(TC_HEAD, 4.0 * B * C * NC);
        fill_k<<<cdiv(B, 256), 256, 0, s>>>(dlosses, 1.0f / (float)b_global, B);
        VIT_HIP(hipMemsetAsync(dlogits, 0, (size_t)B * NC * 4, s));
        ce_backward(dlogits, dlosses, probs, labels, B, NC, s);
        VIT_HIP(hipMemsetAsync(dlnf, 0, (size_t)B * C * 4, s));
        GemmArgs a;  // dlnf += dlogits . head_w
        a.A = dlogits; a.lda = NC; a.a_kcontig = true;
        a.B = P(P_HEADW); a.ldb = C; a.b_kcontig = false;
        a.C = dlnf; a.ldc = C; a.M = B; a.N = C; a.K = NC; a.epi = lowp() ? EPI_F32_ATOMIC : EPI_F32_ACC;
        if (lowp()) a.splitk = head_split(a.M, a.N, a.K);
        a.ws = gemm_ws; a.ws_bytes = gemm_ws_bytes;
        gemm_f32(a, s);
        GemmArgs w;  // dhead_w += dlogits^T . lnf
        w.A = dlogits; w.lda = NC; w.a_kcontig = false;
        w.B = lnf; w.ldb = C; w.b_kcontig = false;
        w.C = G(P_HEADW); w.ldc = C; w.M = NC; w.N = C; w.K = B; w.epi = lowp() ? EPI_F32_ATOMIC : EPI_F32_ACC;
        if (lowp()) w.splitk = head_split(w.M, w.N, w.K);
        w.ws = gemm_ws; w.ws_bytes = gemm_ws_bytes;
        gemm_f32(w, s);
        colsum_f32(G(P_HEADB), dlogits, B, NC, NC, s, red_ws);
        VIT_HIP(hipMemsetAsync(dcls_x, 0, (size_t)B * C * 4, s));
        ln_backward_f32(dcls_x, G(P_LNFW), G(P_LNFB), dlnf, cls_x, P(P_LNFW), lnf_mean, lnf_rstd, B, C, s, red_ws);
        if (dres_bf) {
            VIT_HIP(hipMemsetAsync(dres_bf, 0, (size_t)BT * C * 2, s));
            VIT_HIP(hipMemsetAsync(dres_lo, 0, (size_t)BT * C, s));
            rows_to_bf16_k<<<cdiv((long long)B * C, 256), 256, 0, s>>>(dres_bf, dres_lo, (long long)T * C, dcls_x, B, C);
        } else {
            VIT_HIP(hipMemsetAsync(dres, 0, (size_t)BT * C * 4, s));
            VIT_HIP(hipMemcpy2DAsync(dres, (size_t)T * C * 4, dcls_x, C * 4, C * 4, B, hipMemcpyDeviceToDevice, s));
        }
        tend();
    }

    // ------------------------------------------------------------------ bf16 fast path
    void forward_bf16() {
        const int Bm = B / nmb;
        const long long R = (long long)Bm * T;  // rows per micro-batch
        mb_fork();
        for (int mb = 0; mb < nmb; mb++) {
            // patch embedding (encoder_forward, train_vit.rs:196 -> ViT)
            hipStream_t st = ms[mb];
            const long long img0 = (long long)mb * Bm;
            tbeg(TC_PATCH, 2.0 * Bm * NP * (double)KP * C, st);
            GemmArgs a;
            a.C = emb_tmp + img0 * NP * C; a.ldc = C; a.bias = P(P_PATCH_B);
            a.M = Bm * NP; a.N = C; a.K = KP; a.epi = EPI_F32_STORE;
            if (patch_f32) {
                im2col_f32(patches_f + img0 * NP * KP, pixels + img0 * 3 * cfg.img * cfg.img, Bm, cfg.img,
                           cfg.patch, st);
                a.A = patches_f + img0 * NP * KP; a.lda = KP; a.B = P(P_PATCH_W); a.ldb = KP;
                gemm_f32(a, st);
            } else if (patch_pad) {
                im2col_pad_bf16(patches_bf + img0 * NP * KPP, pixels + img0 * 3 * cfg.img * cfg.img, Bm, cfg.img,
                                cfg.patch, KPP, st);
                a.A = patches_bf + img0 * NP * KPP; a.lda = KPP; a.B = wpatch_pad; a.ldb = KPP; a.K = KPP;
                set_tail(a, st);
                gemm_bf16(a, st);
            } else {
                im2col_bf16(patches_bf + img0 * NP * KP, pixels + img0 * 3 * cfg.img * cfg.img, Bm, cfg.img,
                            cfg.patch, st);
                a.A = patches_bf + img0 * NP * KP; a.lda = KP; a.B = W(P_PATCH_W); a.ldb = KP;
                set_tail(a, st);
                gemm_bf16(a, st);
            }
            patch_assemble(encoded + img0 * T * C, emb_tmp + img0 * NP * C, P(P_CLS), P(P_WPE), Bm, NP, C, st);
            tend();
        }
        for (int l = 0; l < L; l++) {
            LayerActs& a = la[l];
            const float* xl = l == 0 ? encoded : la[l - 1].res3;
            for (int mb = 0; mb < nmb; mb++) {
                hipStream_t st = ms[mb];
                const long long r0 = (long long)mb * R;
                const float* x = xl + r0 * C;
                const bool rc = rowcol_on(), lm = lnmx_on();
                QMat c_ln1 = rc ? actc_of(0, l) : QMat{}, c_atty = rc ? actc_of(1, l) : QMat{},
                     c_ln2 = rc ? actc_of(2, l) : QMat{};
                tbeg(TC_LN_FWD, 0, st);
                if (lm)  // ln1 only in its two MX forms (the qkv GEMM's A operand, the qkv wgrad's B)
                    ln_forward_mx(act_q[mb], act_s[mb], c_ln1.q, c_ln1.s, a.ln1_mean + r0, a.ln1_rstd + r0, x,
                                  P(P_LN1W, l), P(P_LN1B, l), R, C, kp_tok, r0, mb_ntok(mb, R), st,
                                  ln_left ? lnb_scr[mb] : nullptr);
                else
                    ln_forward_bf16(a.ln1 + r0 * C, a.ln1_mean + r0, a.ln1_rstd + r0, x, P(P_LN1W, l), P(P_LN1B, l), R, C, st);
                tend();
                GemmArgs q;
                q.A = a.ln1 + r0 * C; q.lda = C; q.B = W(P_QKVW, l); q.ldb = C; q.C = a.qkv + r0 * 3 * C;
                q.ldc = 3 * C; q.bias = P(P_QKVB, l); q.M = (int)R; q.N = 3 * C; q.K = C; q.epi = EPI_BF16_STORE;
                gemm_w(TC_QKV_FWD, q, P_QKVW, l, false, mb, st, lm ? PRE_LN : PRE_NONE, false,
                       rc && !lm ? &c_ln1 : nullptr);
                tbeg(TC_ATTN_FWD, 4.0 * Bm * (double)T * T * C, st);
                attn_forward_fused(a.atty + r0 * C, a.lse + (long long)mb * Bm * NH * T, a.qkv + r0 * 3 * C, Bm, T, C, NH, st);
                tend();
                GemmArgs pr;
                pr.A = a.atty + r0 * C; pr.lda = C; pr.B = W(P_ATTPROJW, l); pr.ldb = C; pr.C = a.res2 + r0 * C;
                pr.ldc = C; pr.bias = P(P_ATTPROJB, l); pr.aux = x; pr.ldaux = C;
                pr.M = (int)R; pr.N = C; pr.K = C; pr.epi = EPI_F32_RESID;
                gemm_w(TC_PROJ_FWD, pr, P_ATTPROJW, l, false, mb, st, PRE_NONE, false, rc ? &c_atty : nullptr);
                tbeg(TC_LN_FWD, 0, st);
                if (lm)
                    ln_forward_mx(act_q[mb], act_s[mb], c_ln2.q, c_ln2.s, a.ln2_mean + r0, a.ln2_rstd + r0,
                                  a.res2 + r0 * C, P(P_LN2W, l), P(P_LN2B, l), R, C, kp_tok, r0, mb_ntok(mb, R), st,
                                  ln_left ? lnb_scr[mb] : nullptr);
                else
                    ln_forward_bf16(a.ln2 + r0 * C, a.ln2_mean + r0, a.ln2_rstd + r0, a.res2 + r0 * C, P(P_LN2W, l),
                                    P(P_LN2B, l), R, C, st);
                tend();
                GemmArgs f;
                // fc: fchg = gelu(pre) for fcproj, fchd = gelu'(pre) for the fcproj dgrad (one sigmoid)
                f.A = a.ln2 + r0 * C; f.lda = C; f.B = W(P_FCW, l); f.ldb = C; f.C = a.fchd + r0 * 4 * C;
                f.C2 = a.fchg + r0 * 4 * C; f.ldc = 4 * C; f.bias = P(P_FCB, l); f.M = (int)R; f.N = 4 * C;
                f.K = C; f.epi = EPI_BF16_GELU_D;
                if (epicol_on()) {  // the GELU output only as its row (mx_out) and column MX forms
                    const QMat g = fchgc_of(l);
                    f.C2 = nullptr;
                    f.mxc_q = g.q; f.mxc_s = g.s; f.mxc_ld = kp_tok; f.mxc_off = r0;
                }
                gemm_w(TC_FC_FWD, f, P_FCW, l, false, mb, st, lm ? PRE_LN : PRE_NONE, fuse_mx,
                       rc && !lm ? &c_ln2 : nullptr);
                GemmArgs fp;
                fp.A = a.fchg + r0 * 4 * C; fp.lda = 4 * C; fp.B = W(P_FCPROJW, l); fp.ldb = 4 * C;
                fp.C = a.res3 + r0 * C; fp.ldc = C; fp.bias = P(P_FCPROJB, l); fp.aux = a.res2 + r0 * C;
                fp.ldaux = C; fp.M = (int)R; fp.N = C; fp.K = 4 * C; fp.epi = EPI_F32_RESID;
                gemm_w(TC_FCPROJ_FWD, fp, P_FCPROJW, l, false, mb, st, fuse_mx ? PRE_EPI : PRE_NONE);
            }
        }
        mb_join();
        head_forward();
    }

    // dW[OC,Cin] += dout^T . inp (reduction over all B*T rows, split-K slabs) on the weight-
    // gradient stream once every micro-batch stream has passed `ready` (dout final there); the
    // event `done` marks the end of its reads of dout / inp
    // dout_c / inp_c: column forms already written (rowcol_on(); dout_c's producer recorded `ready`)
    void wgrad(int cls, const bf16_t* dout, int OC, const bf16_t* inp, int Cin, float* dW, int ready,
               int done, const QMat* dout_c = nullptr, const QMat* inp_c = nullptr) {
        GemmArgs w;
        w.A = dout; w.lda = OC; w.a_kcontig = false;
        w.B = inp; w.ldb = Cin; w.b_kcontig = false;
        w.C = dW; w.ldc = Cin; w.M = OC; w.N = Cin; w.K = (int)BT; w.epi = EPI_F32_ATOMIC;
        w.ws = gemm_ws; w.ws_bytes = gemm_ws_bytes;
        // split-K fill: beside the micro-batch streams (concurrency on) the engine default (45 %: fewer
        // splits, their half-filled rounds shared); alone on the GPU (concurrency off: the bench's
        // per-kernel timing pass) 80 % of the slots
        w.fill_pct = two_streams ? 0 : 80;
        hipStream_t st = two_streams ? s2 : s;
        if (two_streams) {
            for (int mb = 0; mb < nmb; mb++) {
                if (!dout_c) VIT_HIP(hipEventRecord(mev[mb][ready], ms[mb]));
                VIT_HIP(hipStreamWaitEvent(s2, mev[mb][ready], 0));
            }
        }
        if (fp8() && fp8_wgrad) {
            const long long kp = mx_cols_kp(BT);
            const QMat qa = dout_c ? *dout_c : wg_a, qb = inp_c ? *inp_c : wg_b;
            if (!dout_c || !inp_c) {
                tbeg(TC_QUANT, 0, st);
                if (!dout_c) quantize_mx_cols_bf16(wg_a.q, wg_a.s, dout, BT, OC, OC, st);
                if (!inp_c) quantize_mx_cols_bf16(wg_b.q, wg_b.s, inp, BT, Cin, Cin, st);
                tend();
            }
            w.A = qa.q; w.lda = kp; w.a_kcontig = true; w.a_scale = qa.s;
            w.B = qb.q; w.ldb = kp; w.b_kcontig = true; w.b_scale = qb.s;
            w.K = (int)kp;
            tbeg(cls, 2.0 * w.M * (double)w.N * BT, st);
            gemm_fp8(w, st);
            tend();
        } else {
            tbeg(cls, 2.0 * w.M * (double)w.N * w.K, st);
            gemm_bf16(w, st);
            tend();
        }
        if (two_streams) VIT_HIP(hipEventRecord(bev[done], s2));
    }
    // a micro-batch stream may overwrite a buffer once the wgrad that reads it (`done`) finished
    void after_wgrad(int done, hipStream_t st) {
        if (two_streams) VIT_HIP(hipStreamWaitEvent(st, bev[done], 0));
    }

    float* sg_rows(int l, long long off) { return sg_part[l & 1] + off; }
    // the layer's small gradients from the micro-batches' partial rows, in a fixed order, on the
    // weight-gradient stream once every micro-batch stream has finished the layer (LN1 backward).
    // Layer l-2 reuses this parity's rows only after waits on wgrad events recorded after this
    // reduce (after_wgrad in layer l-1 / l-2), so one pair of buffers suffices.
    void sg_finalize(int l, long long R) {
        hipStream_t st = two_streams ? s2 : s;
        if (two_streams) {
            for (int mb = 0; mb < nmb; mb++) {
                VIT_HIP(hipEventRecord(mev[mb][EV_SG], ms[mb]));
                VIT_HIP(hipStreamWaitEvent(s2, mev[mb][EV_SG], 0));
            }
        }
        const int nb = nmb * ln_bwd_blocks(R), w1 = l > 0 ? 3 * C : 2 * C;
        const float* p2 = sg_rows(l, sg_ln2);
        const float* p1 = sg_rows(l, sg_ln1);
        RowsJob jobs[8] = {
            {G(P_LN2W, l), p2, nb, 3 * C, C},
            {G(P_LN2B, l), p2 + C, nb, 3 * C, C},
            {G(P_ATTPROJB, l), p2 + 2 * C, nb, 3 * C, C},
            {G(P_LN1W, l), p1, nb, w1, C},
            {G(P_LN1B, l), p1 + C, nb, w1, C},
            {G(P_FCB, l), sg_rows(l, sg_fcb), nmb * fcb_rows, 4 * C, 4 * C},
            {G(P_QKVB, l), sg_rows(l, sg_qkv), nmb, 3 * C, 3 * C},
            {l > 0 ? G(P_FCPROJB, l - 1) : nullptr, p1 + 2 * C, nb, w1, C},
        };
        tbeg(TC_COLSUM, 0, st);
        rows_reduce_add(jobs, l > 0 ? 8 : 7, st);
        tend();
    }

    void backward_bf16() {
        pre_side_wait();  // the arena clear and the transposed weights (side pre-work on s2)
        // the residual-gradient stream is "bf16 + lo8" (common.h: a bf16 plane, the GEMM operand,
        // plus a byte plane of its rounding residual; a 16-bit significand in 3 bytes): dres3 (the
        // layer output's gradient) in rbA/loA, dres2 in rbB/loB; each LayerNorm backward reads one
        // and writes the other (its column sum, the next bias gradient, is taken in fp32)
        bf16_t* rbA = dres_bf;   // dres3 (read by the fcproj dgrad / wgrad and LN2 backward)
        bf16_t* rbB = dres_bf2;  // dres2 (read by the attproj dgrad / wgrad and LN1 backward)
        uint8_t* loA = dres_lo;
        uint8_t* loB = dres_lo2;
        head_backward(nullptr, rbA, loA);
        chunk_done(0);
        // bias gradients are fused into the kernels that produce each gradient tensor:
        //   fcproj_b += colsum(dres3): LN1-backward of layer l+1 (head rows for the last layer)
        //   fc_b     += colsum(dfch):  fcproj dgrad epilogue
        //   attproj_b+= colsum(dres2): LN2-backward
        //   qkv_b    += colsum(dqkv):  attention backward
        colsum_f32(G(P_FCPROJB, L - 1), dcls_x, B, C, C, s, red_ws);
        mb_fork();
        const int Bm = B / nmb;
        const long long R = (long long)Bm * T;
        for (int l = L - 1; l >= 0; l--) {
            LayerActs& a = la[l];
            const float* xl = l == 0 ? encoded : la[l - 1].res3;
            // rowcol: the weight gradients whose dout column form the dgrads' quantize step writes
            // are issued after those dgrads (s2 waits on the event recorded after the quantize)
            const bool rc = rowcol_on();
            QMat c_ln1 = rc ? actc_of(0, l) : QMat{}, c_atty = rc ? actc_of(1, l) : QMat{}, c_ln2 = rc ? actc_of(2, l) : QMat{};
            // lbm: the LayerNorm backwards write dres2 / dres3's MX forms (dres3 of the last layer comes
            // from the head and is quantized by the fcproj dgrad as before)
            const bool lbm = lnbmx_on(), resa_pre = lbm && l < L - 1;
            // fcproj: dfch = (dres3 . fcprojw) * gelu'(fch) (stored as fchd);  fcprojw += dres3^T . fchg
            const bool ec = epicol_on();
            QMat c_fchg = ec ? fchgc_of(l) : QMat{};
            if (!rc) wgrad(TC_FCPROJ_WGRAD, rbA, C, a.fchg, 4 * C, G(P_FCPROJW, l), EV_RESA, EV_W1);
            for (int mb = 0; mb < nmb; mb++) {
                const long long r0 = mb * R;
                after_wgrad(EV_W2, ms[mb]);  // the previous layer's fc wgrad has read dfch
                GemmArgs d1;
                d1.A = rbA + r0 * C; d1.lda = C; dgrad_b(d1, P_FCPROJW, l, C, 4 * C);
                d1.C = dfch + r0 * 4 * C; d1.ldc = 4 * C; d1.aux = a.fchd + r0 * 4 * C; d1.ldaux = 4 * C;
                d1.M = (int)R; d1.N = 4 * C; d1.K = C; d1.epi = EPI_BF16_MUL;
                fcb_rows = gemm_colsum_rows(d1, fp8());  // partial rows per micro-batch (engine-dependent)
                d1.colsum_part = sg_rows(l, sg_fcb) + (long long)mb * fcb_rows * 4 * C;
                if (ec) {  // dfch only as its row (mx_out) and column MX forms
                    d1.C = nullptr;
                    d1.mxc_q = dfchc.q; d1.mxc_s = dfchc.s; d1.mxc_ld = kp_tok; d1.mxc_off = r0;
                }
                gemm_w(TC_FCPROJ_DGRAD, d1, P_FCPROJW, l, true, mb, ms[mb], resa_pre ? PRE_LN : PRE_NONE, fuse_mx,
                       rc && !resa_pre ? &dcol[0] : nullptr, resa_pre ? -1 : EV_RESA);
                if (ec && two_streams) VIT_HIP(hipEventRecord(mev[mb][EV_DFCH], ms[mb]));  // dfchc final
            }
            if (rc) wgrad(TC_FCPROJ_WGRAD, rbA, C, a.fchg, 4 * C, G(P_FCPROJW, l), EV_RESA, EV_W1, &dcol[0],
                          ec ? &c_fchg : nullptr);
            // fc: dln2 = dfch . fcw;  fcw += dfch^T . ln2
            wgrad(TC_FC_WGRAD, dfch, 4 * C, a.ln2, C, G(P_FCW, l), EV_DFCH, EV_W2, ec ? &dfchc : nullptr,
                  rc ? &c_ln2 : nullptr);
            for (int mb = 0; mb < nmb; mb++) {
                const long long r0 = mb * R;
                GemmArgs d2;
                d2.A = dfch + r0 * 4 * C; d2.lda = 4 * C; dgrad_b(d2, P_FCW, l, 4 * C, C);
                d2.C = dln_bf + r0 * C; d2.ldc = C; d2.M = (int)R; d2.N = C; d2.K = 4 * C; d2.epi = EPI_BF16_STORE;
                gemm_w(TC_FC_DGRAD, d2, P_FCW, l, true, mb, ms[mb], fuse_mx ? PRE_EPI : PRE_NONE);
                // ln2 backward + residual: dres2 = dres3 + LN2'(dln2); attproj_b += colsum(dres2)
                after_wgrad(EV_W3, ms[mb]);  // the previous layer's attproj wgrad has read rbB
                tbeg(TC_LN_BWD, 0, ms[mb]);
                if (lbm) {  // + dres2's MX forms (the attproj dgrad's A operand, the attproj wgrad's dout)
                    ln_backward_bf16_stream_mx(rbB + r0 * C, loB + r0 * C, rbA + r0 * C, loA + r0 * C, G(P_LN2W, l),
                                               G(P_LN2B, l), G(P_ATTPROJB, l), dln_bf + r0 * C, a.res2 + r0 * C,
                                               P(P_LN2W, l), a.ln2_mean + r0, a.ln2_rstd + r0, R, C, ms[mb],
                                               sg_rows(l, sg_ln2) + (long long)mb * ln_bwd_blocks(R) * 3 * C,
                                               act_q[mb], act_s[mb], dcol[1].q, dcol[1].s, kp_tok, r0, mb_ntok(mb, R),
                                               lnb_scr[mb]);
                    if (two_streams) VIT_HIP(hipEventRecord(mev[mb][EV_RESB], ms[mb]));
                } else {
                    ln_backward_bf16_stream(rbB + r0 * C, loB + r0 * C, rbA + r0 * C, loA + r0 * C, G(P_LN2W, l),
                                            G(P_LN2B, l), G(P_ATTPROJB, l), dln_bf + r0 * C, a.res2 + r0 * C,
                                            P(P_LN2W, l), a.ln2_mean + r0, a.ln2_rstd + r0, R, C, ms[mb],
                                            sg_rows(l, sg_ln2) + (long long)mb * ln_bwd_blocks(R) * 3 * C);
                }
                tend();
            }
            // attproj
            if (!rc) wgrad(TC_PROJ_WGRAD, rbB, C, a.atty, C, G(P_ATTPROJW, l), EV_RESB, EV_W3);
            for (int mb = 0; mb < nmb; mb++) {
                const long long r0 = mb * R;
                GemmArgs d3;
                d3.A = rbB + r0 * C; d3.lda = C; dgrad_b(d3, P_ATTPROJW, l, C, C);
                d3.C = datty + r0 * C; d3.ldc = C; d3.M = (int)R; d3.N = C; d3.K = C; d3.epi = EPI_BF16_STORE;
                gemm_w(TC_PROJ_DGRAD, d3, P_ATTPROJW, l, true, mb, ms[mb], lbm ? PRE_LN : PRE_NONE, false,
                       rc && !lbm ? &dcol[1] : nullptr, lbm ? -1 : EV_RESB);
                // attention (+ qkv_b)
                after_wgrad(EV_W4, ms[mb]);  // the previous layer's qkv wgrad has read dqkv
                tbeg(TC_ATTN_BWD, 8.0 * Bm * (double)T * T * C, ms[mb]);
                attn_backward_fused(dqkv + r0 * 3 * C, datty + r0 * C, a.qkv + r0 * 3 * C, a.atty + r0 * C,
                                    a.lse + (long long)mb * Bm * NH * T, Bm, T, C, NH, ms[mb],
                                    sg_rows(l, sg_qkv) + (long long)mb * 3 * C,
                                    attn_part + (long long)attn_backward_ws_floats(mb * Bm, T, C, NH), true);
                tend();
            }
            if (rc) wgrad(TC_PROJ_WGRAD, rbB, C, a.atty, C, G(P_ATTPROJW, l), EV_RESB, EV_W3, &dcol[1], &c_atty);
            // qkv
            if (!rc) wgrad(TC_QKV_WGRAD, dqkv, 3 * C, a.ln1, C, G(P_QKVW, l), EV_DQKV, EV_W4);
            for (int mb = 0; mb < nmb; mb++) {
                const long long r0 = mb * R;
                GemmArgs d4;
                d4.A = dqkv + r0 * 3 * C; d4.lda = 3 * C; dgrad_b(d4, P_QKVW, l, 3 * C, C);
                d4.C = dln_bf + r0 * C; d4.ldc = C; d4.M = (int)R; d4.N = C; d4.K = 3 * C; d4.epi = EPI_BF16_STORE;
                gemm_w(TC_QKV_DGRAD, d4, P_QKVW, l, true, mb, ms[mb], PRE_NONE, false, rc ? &dcol[2] : nullptr, EV_DQKV);
                // ln1 backward: dres = dres2 + LN1'(dln1); fcproj_b of layer l-1 += colsum(dres)
                after_wgrad(EV_W1, ms[mb]);  // this layer's fcproj wgrad has read rbA
                tbeg(TC_LN_BWD, 0, ms[mb]);
                if (lbm && l > 0) {  // + dres3's MX forms for layer l-1's fcproj dgrad / wgrad
                    ln_backward_bf16_stream_mx(rbA + r0 * C, loA + r0 * C, rbB + r0 * C, loB + r0 * C, G(P_LN1W, l),
                                               G(P_LN1B, l), G(P_FCPROJB, l - 1), dln_bf + r0 * C, xl + r0 * C,
                                               P(P_LN1W, l), a.ln1_mean + r0, a.ln1_rstd + r0, R, C, ms[mb],
                                               sg_rows(l, sg_ln1) + (long long)mb * ln_bwd_blocks(R) * 3 * C,
                                               act_q[mb], act_s[mb], dcol[0].q, dcol[0].s, kp_tok, r0, mb_ntok(mb, R),
                                               lnb_scr[mb]);
                    if (two_streams) VIT_HIP(hipEventRecord(mev[mb][EV_RESA], ms[mb]));
                } else {
                    ln_backward_bf16_stream(rbA + r0 * C, loA + r0 * C, rbB + r0 * C, loB + r0 * C, G(P_LN1W, l),
                                            G(P_LN1B, l), l > 0 ? G(P_FCPROJB, l - 1) : nullptr, dln_bf + r0 * C,
                                            xl + r0 * C, P(P_LN1W, l), a.ln1_mean + r0, a.ln1_rstd + r0, R, C, ms[mb],
                                            sg_rows(l, sg_ln1) + (long long)mb * ln_bwd_blocks(R) * (l > 0 ? 3 : 2) * C);
                }
                tend();
            }
            if (rc) wgrad(TC_QKV_WGRAD, dqkv, 3 * C, a.ln1, C, G(P_QKVW, l), EV_DQKV, EV_W4, &dcol[2], &c_ln1);
            sg_finalize(l, R);
            chunk_done(L - l);
        }
        mb_join();
        if (two_streams) {  // every wgrad done before the slab workspace / grads are reused
            VIT_HIP(hipEventRecord(bev[EV_JOIN], s2));
            VIT_HIP(hipStreamWaitEvent(s, bev[EV_JOIN], 0));
        }
        // patch embedding backward (encoder_backward, train_vit.rs:371 -> ViT)
        tbeg(TC_PATCH_BWD, 2.0 * B * NP * (double)KP * C);
        // cls / position / patch-bias gradients (psg: three small kernels, 43 us) on s2 beside the
        // patch weight gradient on s; s waits for them before the chunk is final
        const bool psg_side = two_streams && lowp() && patch_tail;
        if (psg_side) {
            VIT_HIP(hipEventRecord(bev[EV_SG], s));
            VIT_HIP(hipStreamWaitEvent(s2, bev[EV_SG], 0));
            patch_small_grads(G(P_CLS), G(P_WPE), G(P_PATCH_B), rbA, loA, B, T, C, s2, pos_sums, psg_part);
            VIT_HIP(hipEventRecord(bev[EV_JOIN], s2));
        }
        if (patch_f32) {
            patch_gather_f32(dpatch_f, rbA, loA, B, NP, C, s);
            GemmArgs w;
            w.A = dpatch_f; w.lda = C; w.a_kcontig = false; w.B = patches_f; w.ldb = KP; w.b_kcontig = false;
            w.C = G(P_PATCH_W); w.ldc = KP; w.M = C; w.N = KP; w.K = B * NP; w.epi = EPI_F32_ATOMIC;
            gemm_f32(w, s);
        } else {
            patch_gather_bf16(dpatch_bf, rbA, B, NP, C, s);
            GemmArgs w;
            w.A = dpatch_bf; w.lda = C; w.a_kcontig = false;
            w.B = patches_bf; w.ldb = KPP; w.b_kcontig = false;
            w.C = G(P_PATCH_W); w.ldc = KP; w.M = C; w.N = KP; w.K = B * NP; w.epi = EPI_F32_ATOMIC;
            w.ws = gemm_ws; w.ws_bytes = gemm_ws_bytes;
            // after the join nothing but the small-gradient kernels runs beside it: split-K for 80 %
            // of the slots (the 45 % default leaves half the CUs idle: 102 us with 234 workgroups)
            w.fill_pct = patch_tail ? 80 : 0;
            if (patch_pad) {  // dW over KPP columns into the scratch, then its first KP columns into G
                VIT_HIP(hipMemsetAsync(dwpatch_pad, 0, (size_t)C * KPP * 4, s));
                w.C = dwpatch_pad; w.ldc = KPP; w.N = KPP;
            }
            gemm_bf16(w, s);
            if (patch_pad)
                add_cols_k<<<grid_for((long long)C * KP, 256), 256, 0, s>>>(G(P_PATCH_W), dwpatch_pad, C, KP, KPP);
        }
        if (psg_side)
            VIT_HIP(hipStreamWaitEvent(s, bev[EV_JOIN], 0));
        else
            patch_small_grads(G(P_CLS), G(P_WPE), G(P_PATCH_B), rbA, loA, B, T, C, s, pos_sums, psg_part);
        tend();
        chunk_done(L + 1);
    }

    // ------------------------------------------------------------------ fp32 reference path
    void forward_f32() {
        im2col_f32(patches_f, pixels, B, cfg.img, cfg.patch, s);
        {
            GemmArgs a;
            a.A = patches_f; a.lda = KP; a.B = P(P_PATCH_W); a.ldb = KP; a.C = emb_tmp; a.ldc = C;
            a.bias = P(P_PATCH_B); a.M = B * NP; a.N = C; a.K = KP; a.epi = EPI_F32_STORE;
            gemm_f32(a, s);
        }
        patch_assemble(encoded, emb_tmp, P(P_CLS), P(P_WPE), B, NP, C, s);
        for (int l = 0; l < L; l++) {
            LayerActs& a = la[l];
            const float* x = l == 0 ? encoded : la[l - 1].res3;
            ln_forward_f32(a.ln1f, a.ln1_mean, a.ln1_rstd, x, P(P_LN1W, l), P(P_LN1B, l), BT, C, s);
            mm_fwd(a.qkvf, a.ln1f, P(P_QKVW, l), P(P_QKVB, l), C, 3 * C);
            attn_forward_f32(a.attyf, a.preatt, a.att, a.qkvf, B, T, C, NH, s);
            mm_fwd(a.attproj, a.attyf, P(P_ATTPROJW, l), P(P_ATTPROJB, l), C, C);
            add(a.res2, x, a.attproj, BT * C);
            ln_forward_f32(a.ln2f, a.ln2_mean, a.ln2_rstd, a.res2, P(P_LN2W, l), P(P_LN2B, l), BT, C, s);
            mm_fwd(a.fchf, a.ln2f, P(P_FCW, l), P(P_FCB, l), C, 4 * C);
            gelu(a.fchgf, a.fchf, BT * 4 * C);
            mm_fwd(a.fcproj, a.fchgf, P(P_FCPROJW, l), P(P_FCPROJB, l), 4 * C, C);
            add(a.res3, a.res2, a.fcproj, BT * C);
        }
        head_forward();
    }
    void mm_fwd(float* out, const float* inp, const float* w, const float* b, int Cin, int OC) {
        GemmArgs a;
        a.A = inp; a.lda = Cin; a.B = w; a.ldb = Cin; a.C = out; a.ldc = OC; a.bias = b;
        a.M = (int)BT; a.N = OC; a.K = Cin; a.epi = EPI_F32_STORE;
        gemm_f32(a, s);
    }
    void mm_bwd(float* dinp, float* dw, float* db, const float* dout, const float* inp,
                const float* w, int Cin, int OC) {
        GemmArgs d;
        d.A = dout; d.lda = OC; d.B = w; d.ldb = Cin; d.b_kcontig = false; d.C = dinp; d.ldc = Cin;
        d.M = (int)BT; d.N = Cin; d.K = OC; d.epi = EPI_F32_ACC;
        gemm_f32(d, s);
        GemmArgs g;
        g.A = dout; g.lda = OC; g.a_kcontig = false; g.B = inp; g.ldb = Cin; g.b_kcontig = false;
        g.C = dw; g.ldc = Cin; g.M = OC; g.N = Cin; g.K = (int)BT; g.epi = EPI_F32_ATOMIC;
        g.ws = gemm_ws; g.ws_bytes = gemm_ws_bytes;
        gemm_f32(g, s);
        colsum_f32(db, dout, (int)BT, OC, OC, s, red_ws);
    }
    void add(float* out, const float* a, const float* b, long long n);
    void gelu(float* out, const float* in, long long n);
    void gelu_bwd(float* dinp, const float* in, const float* dout, long long n);
    void res_bwd(float* d1, float* d2, const float* dout, long long n);

    void backward_f32() {
        float* dcur = dres_a;
        float* dnxt = dres_b;
        head_backward(dcur);
        chunk_done(0);
        for (int l = L - 1; l >= 0; l--) {
            LayerActs& a = la[l];
            const float* x = l == 0 ? encoded : la[l - 1].res3;
            VIT_HIP(hipMemsetAsync(g_block, 0, g_block_elems * 4, s));
            VIT_HIP(hipMemsetAsync(dnxt, 0, BT * C * 4, s));
            // train_vit.rs:359-368
            res_bwd(g_dres2, g_dfcproj, dcur, BT * C);
            mm_bwd(g_dfchg, G(P_FCPROJW, l), G(P_FCPROJB, l), g_dfcproj, a.fchgf, P(P_FCPROJW, l), 4 * C, C);
            gelu_bwd(g_dfch, a.fchf, g_dfchg, BT * 4 * C);
            mm_bwd(g_dln2, G(P_FCW, l), G(P_FCB, l), g_dfch, a.ln2f, P(P_FCW, l), C, 4 * C);
            ln_backward_f32(g_dres2, G(P_LN2W, l), G(P_LN2B, l), g_dln2, a.res2, P(P_LN2W, l),
                            a.ln2_mean, a.ln2_rstd, BT, C, s, red_ws);
            res_bwd(dnxt, g_dattproj, g_dres2, BT * C);
            mm_bwd(g_datty, G(P_ATTPROJW, l), G(P_ATTPROJB, l), g_dattproj, a.attyf, P(P_ATTPROJW, l), C, C);
            attn_backward_f32(g_dqkv, g_dpreatt, g_datt, g_datty, a.qkvf, a.att, B, T, C, NH, s);
            mm_bwd(g_dln1, G(P_QKVW, l), G(P_QKVB, l), g_dqkv, a.ln1f, P(P_QKVW, l), C, 3 * C);
            ln_backward_f32(dnxt, G(P_LN1W, l), G(P_LN1B, l), g_dln1, x, P(P_LN1W, l), a.ln1_mean,
                            a.ln1_rstd, BT, C, s, red_ws);
            std::swap(dcur, dnxt);
            chunk_done(L - l);
        }
        im2col_f32(patches_f, pixels, B, cfg.img, cfg.patch, s);
        patch_gather_f32(dpatch_f, dcur, B, NP, C, s);
        GemmArgs w;
        w.A = dpatch_f; w.lda = C; w.a_kcontig = false; w.B = patches_f; w.ldb = KP; w.b_kcontig = false;
        w.C = G(P_PATCH_W); w.ldc = KP; w.M = C; w.N = KP; w.K = B * NP; w.epi = EPI_F32_ATOMIC;
        w.ws = gemm_ws; w.ws_bytes = gemm_ws_bytes;
        gemm_f32(w, s);
        patch_small_grads(G(P_CLS), G(P_WPE), G(P_PATCH_B), dcur, B, T, C, s, pos_sums);
        chunk_done(L + 1);
    }

    // ------------------------------------------------------------------ DP
    // Early SGD (option early_sgd, one GPU, bf16 / fp8, two streams, the fused train step): chunk c's
    // gradients are final at chunk_done(c) (the DP overlap's ordering, checked bit-for-bit by the
    // dp_probe test), and no later backward kernel reads chunk c's weights, so its SGD update runs
    // on s_comm (no extra stream: a seventh stream re-maps the streams onto the 4 hardware queues
    // and cost bf16 6 %) right there, beside the rest of the backward, instead of one 216 us pass.
    // The update is elementwise: the same bits as the whole-arena pass.  step() then only waits.
    // Measured (tools/ab_step.py, same process, profiles/r06_early_sgd_ab.txt): on s_comm ViT-B/16
    // 35.57 vs 35.56 and 35.65 vs 35.54 ms/step (-0.2 %), ViT-L/16 114.47 vs 114.79 (+0.3 %), ViT-H/14
    // fp8 114.68 vs 116.08 and 114.99 vs 115.72 (+1.2 / +0.6 %) on two boxes: on in fp8 mode (-1: auto)
    int early_sgd = -1;
    bool early_sgd_on() const { return early_sgd < 0 ? fp8() : early_sgd != 0; }
    bool early_on = false, early_done = false;
    float early_lr = 0.f;
    void sgd_chunk(int c) {
        VIT_HIP(hipEventRecord(chunk_ev[c], s));
        VIT_HIP(hipStreamWaitEvent(s_comm, chunk_ev[c], 0));
        VIT_HIP(hipEventRecord(chunk_ev2[c], s2));
        VIT_HIP(hipStreamWaitEvent(s_comm, chunk_ev2[c], 0));
        for (int k = 1; k < nmb; k++) {
            hipEvent_t e = chunk_evm[(size_t)c * MAXMB + k];
            VIT_HIP(hipEventRecord(e, ms[k]));
            VIT_HIP(hipStreamWaitEvent(s_comm, e, 0));
        }
        const long long o = chunk_off[c], n = chunk_off[c + 1] - chunk_off[c];
        sgd_bf16_k<<<grid_for(n / 4, 256), 256, 0, s_comm>>>(params + o, pbf + o, grads + o, n, early_lr);
        after_launch("sgd_bf16_chunk");
    }
    void chunk_done(int c) {
        if (early_on) {
            sgd_chunk(c);
            return;
        }
        if (!comm || !overlap) return;
        VIT_HIP(hipEventRecord(chunk_ev[c], s));
        VIT_HIP(hipStreamWaitEvent(s_comm, chunk_ev[c], 0));
        if (two_streams && lowp()) {  // the chunk's gradients also come from s2 / ms[]
            VIT_HIP(hipEventRecord(chunk_ev2[c], s2));
            VIT_HIP(hipStreamWaitEvent(s_comm, chunk_ev2[c], 0));
            for (int k = 1; k < nmb; k++) {
                hipEvent_t e = chunk_evm[(size_t)c * MAXMB + k];
                VIT_HIP(hipEventRecord(e, ms[k]));
                VIT_HIP(hipStreamWaitEvent(s_comm, e, 0));
            }
        }
        const long long o = chunk_off[c], n = chunk_off[c + 1] - chunk_off[c];
        ncclResult_t r = ncclAllReduce(grads + o, grads + o, (size_t)n, ncclFloat32, ncclSum, comm, s_comm);
        if (r != ncclSuccess) set_error("ncclAllReduce(chunk %d): %s", c, ncclGetErrorString(r));
        if (dp_probe_on)
            VIT_HIP(hipMemcpyAsync(dp_snap + o, grads + o, (size_t)n * 4, hipMemcpyDeviceToDevice, s_comm));
    }
    void finish_allreduce() {
        if (!comm) return;  // (world 1 with a communicator still runs RCCL: the tested path)
        if (!overlap) {
            ncclResult_t r = ncclAllReduce(grads, grads, (size_t)arena_elems, ncclFloat32, ncclSum, comm, s);
            if (r != ncclSuccess) set_error("ncclAllReduce: %s", ncclGetErrorString(r));
            if (dp_probe_on)
                VIT_HIP(hipMemcpyAsync(dp_snap, grads, (size_t)arena_elems * 4, hipMemcpyDeviceToDevice, s));
            return;
        }
        VIT_HIP(hipEventRecord(comm_done, s_comm));
        VIT_HIP(hipStreamWaitEvent(s, comm_done, 0));
    }

    // upload one uint8 batch (host) and normalise it into `pixels` (include/vit_data.h)
    bool set_batch_u8(const unsigned char* img, const int* lab, const float* mean, const float* sd) {
        return stage_batch(img, nullptr, lab, mean, sd);
    }
    // the JPEG loader's current batch (include/vit_jpeg.h): decoded on the copy stream into the
    // same uint8 staging, then the same normalise
    bool set_batch_jpeg(vit_jpeg_loader_t* jl, const float* mean, const float* sd) {
        return stage_batch(nullptr, jl, nullptr, mean, sd);
    }
    bool stage_batch(const unsigned char* img, vit_jpeg_loader_t* jl, const int* lab, const float* mean,
                     const float* sd) {
        const int HW = cfg.img * cfg.img;
        const size_t bytes = (size_t)B * HW * 3;
        if (!s_copy) {
            VIT_HIP(hipStreamCreateWithFlags(&s_copy, hipStreamNonBlocking));
            for (int k = 0; k < 2; k++) {
                u8_stage[k] = alloc<unsigned char>((long long)bytes);
                lab_stage[k] = alloc<int>(B);
                VIT_HIP(hipEventCreateWithFlags(&u8_copied[k], hipEventDisableTiming));
                VIT_HIP(hipEventCreateWithFlags(&u8_used[k], hipEventDisableTiming));
                VIT_HIP(hipEventRecord(u8_used[k], s));
            }
            if (has_error()) return false;
        }
        const int k = u8_k & 1;
        u8_k++;
        // the staging slot is free once the normalise of two uploads ago has run
        VIT_HIP(hipStreamWaitEvent(s_copy, u8_used[k], 0));
        if (jl) {  // host entropy decode already done by the loader; the pixel work runs here
            if (!jpeg_loader_decode_to(jl, u8_stage[k], cfg.img, s_copy, &lab, B)) return false;
        } else {
            VIT_HIP(hipMemcpyAsync(u8_stage[k], img, bytes, hipMemcpyHostToDevice, s_copy));
        }
        if (lab) VIT_HIP(hipMemcpyAsync(lab_stage[k], lab, (size_t)B * 4, hipMemcpyHostToDevice, s_copy));
        VIT_HIP(hipEventRecord(u8_copied[k], s_copy));
        VIT_HIP(hipStreamWaitEvent(s, u8_copied[k], 0));
        has_targets = lab != nullptr;
        const long long n = (long long)B * HW;
        normalize_u8_k<<<cdiv(n, 256), 256, 0, s>>>(pixels, labels, u8_stage[k], lab ? lab_stage[k] : nullptr,
                                                     B, HW, mean[0], mean[1], mean[2], sd[0], sd[1], sd[2]);
        after_launch("normalize_u8");
        VIT_HIP(hipEventRecord(u8_used[k], s));
        // the host buffers may be reused once the DMA has read them (overlaps the GPU's queue)
        VIT_HIP(hipEventSynchronize(u8_copied[k]));
        return !has_error();
    }

    bool ensure_adam() {
        if (adam_m) return true;
        adam_m = alloc<float>(arena_elems);
        adam_v = alloc<float>(arena_elems);
        if (!adam_m || !adam_v) return false;
        VIT_HIP(hipMemsetAsync(adam_m, 0, arena_elems * 4, s));
        VIT_HIP(hipMemsetAsync(adam_v, 0, arena_elems * 4, s));
        return true;
    }
    // AdamW update t = adam_t + 1 (llm.c's update, which the reference's m/v buffers —
    // train_vit.rs:73-74 — were allocated for; its optimizer_step :737 is SGD)
    void step_adamw(float lr, const vit_adamw_t& hp) {
        pre_side_wait();
        finish_allreduce();
        if (!ensure_adam()) return;
        adam_t += 1;
        adam_hp = hp;
        // bias corrections and 1-beta exactly as the oracle rounds them (pow in double -> fp32)
        const float bc1 = 1.0f - (float)pow((double)hp.beta1, (double)adam_t);
        const float bc2 = 1.0f - (float)pow((double)hp.beta2, (double)adam_t);
        tbeg(TC_SGD, 0);
        adamw_k<<<grid_for(arena_elems / 4, 256), 256, 0, s>>>(
            params, lowp() ? pbf : nullptr, grads, adam_m, adam_v, arena_elems, lr,
            hp.beta1, hp.beta2, 1.0f - hp.beta1, 1.0f - hp.beta2, bc1, bc2, hp.eps, hp.weight_decay);
        after_launch("adamw");
        tend();
        if (lowp()) refresh_transposed();
    }

    void step(float lr) {
        pre_side_wait();
        if (early_done) {  // every chunk already updated on s_comm (train_step with early SGD)
            early_done = false;
            VIT_HIP(hipEventRecord(comm_done, s_comm));
            VIT_HIP(hipStreamWaitEvent(s, comm_done, 0));
            refresh_transposed();
            return;
        }
        finish_allreduce();
        tbeg(TC_SGD, 0);
        if (lowp()) {
            sgd_bf16_k<<<grid_for(arena_elems / 4, 256), 256, 0, s>>>(params, pbf, grads, arena_elems, lr);
            after_launch("sgd_bf16");
        } else {
            sgd(params, grads, arena_elems, lr, s);
        }
        tend();
        if (lowp()) refresh_transposed();
    }
};

__global__ void add_k(float* o, const float* a, const float* b, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        o[i] = a[i] + b[i];
}
__global__ void gelu_k(float* o, const float* a, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        o[i] = gelu_f(a[i]);
}
__global__ void gelu_bwd_k2(float* d, const float* x, const float* g, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        d[i] += gelu_grad_f(x[i]) * g[i];
}
__global__ void resbwd_k(float* d1, float* d2, const float* g, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        d1[i] += g[i];
        d2[i] += g[i];
    }
}
void Trainer::add(float* out, const float* a, const float* b, long long n) {
    add_k<<<grid_for(n, 256), 256, 0, s>>>(out, a, b, n);
    after_launch("residual_forward");
}
void Trainer::gelu(float* out, const float* in, long long n) {
    gelu_k<<<grid_for(n, 256), 256, 0, s>>>(out, in, n);
    after_launch("gelu_forward");
}
void Trainer::gelu_bwd(float* dinp, const float* in, const float* dout, long long n) {
    gelu_bwd_k2<<<grid_for(n, 256), 256, 0, s>>>(dinp, in, dout, n);
    after_launch("gelu_backward");
}
void Trainer::res_bwd(float* d1, float* d2, const float* dout, long long n) {
    resbwd_k<<<grid_for(n, 256), 256, 0, s>>>(d1, d2, dout, n);
    after_launch("residual_backward");
}

}  // namespace vit

// ============================================================================ C ABI
struct vit_trainer {
    vit::Trainer t;
};
using vit::set_error;

extern "C" {
vit_trainer_t* vit_trainer_create(const vit_config_t* cfg, int batch, int precision, int device) {
    auto* h = new vit_trainer();
    if (!h->t.init(cfg, batch, precision, device)) {
        h->t.destroy();
        delete h;
        return nullptr;
    }
    return h;
}
void vit_trainer_destroy(vit_trainer_t* h) {
    if (!h) return;
    h->t.destroy();
    delete h;
}
long long vit_trainer_num_params(const vit_trainer_t* h) { return h->t.n_params; }
long long vit_trainer_device_bytes(const vit_trainer_t* h) { return (long long)h->t.dev_bytes; }
int vit_trainer_set_params(vit_trainer_t* h, const float* hp) {
    h->t.canon_to_device(hp, h->t.params);
    h->t.refresh_bf16();
    VIT_HIP(hipStreamSynchronize(h->t.s));
    return vit::has_error();
}
int vit_trainer_get_params(vit_trainer_t* h, float* hp) {
    h->t.device_to_canon(h->t.params, hp);
    return vit::has_error();
}
int vit_trainer_get_grads(vit_trainer_t* h, float* hg) {
    VIT_HIP(hipStreamSynchronize(h->t.s_comm));
    h->t.device_to_canon(h->t.grads, hg);
    return vit::has_error();
}
static bool labels_ok(const int* lab, int n, int nc) {
    for (int i = 0; i < n; i++)
        if (lab[i] < 0 || lab[i] >= nc) {
            set_error("label %d of the batch is %d, outside [0, %d)", i, lab[i], nc);
            return false;
        }
    return true;
}
int vit_trainer_set_batch(vit_trainer_t* h, const float* px, const int* lab) {
    auto& t = h->t;
    if (lab && !labels_ok(lab, t.B, t.NC)) return 1;
    VIT_HIP(hipMemcpyAsync(t.pixels, px, (size_t)t.B * 3 * t.cfg.img * t.cfg.img * 4, hipMemcpyHostToDevice, t.s));
    t.has_targets = lab != nullptr;
    if (lab) VIT_HIP(hipMemcpyAsync(t.labels, lab, (size_t)t.B * 4, hipMemcpyHostToDevice, t.s));
    VIT_HIP(hipStreamSynchronize(t.s));
    return vit::has_error();
}
int vit_trainer_set_batch_device(vit_trainer_t* h, const float* px, const int* lab) {
    auto& t = h->t;
    VIT_HIP(hipMemcpyAsync(t.pixels, px, (size_t)t.B * 3 * t.cfg.img * t.cfg.img * 4, hipMemcpyDeviceToDevice, t.s));
    t.has_targets = lab != nullptr;
    if (lab) VIT_HIP(hipMemcpyAsync(t.labels, lab, (size_t)t.B * 4, hipMemcpyDeviceToDevice, t.s));
    return vit::has_error();
}
int vit_trainer_forward(vit_trainer_t* h, int b_global) {
    auto& t = h->t;
    t.b_global = b_global > 0 ? b_global : t.B;
    if (t.lowp()) t.forward_bf16(); else t.forward_f32();
    return vit::has_error();
}
int vit_trainer_zero_grad(vit_trainer_t* h) {
    auto& t = h->t;
    // the previous step's all-reduce must be done with the arena before it is cleared
    if (t.comm) {
        VIT_HIP(hipEventRecord(t.comm_done, t.s_comm));
        VIT_HIP(hipStreamWaitEvent(t.s, t.comm_done, 0));
    }
    if (t.pre_side_on()) {  // on s2 beside the forward; the backward waits for it
        hipStream_t zs = t.pre_side_begin();
        VIT_HIP(hipMemsetAsync(t.grads, 0, t.arena_elems * 4, zs));
        t.pre_side_end();
    } else {
        VIT_HIP(hipMemsetAsync(t.grads, 0, t.arena_elems * 4, t.s));
    }
    return vit::has_error();
}
int vit_trainer_backward(vit_trainer_t* h) {
    auto& t = h->t;
    if (!t.has_targets) {
        set_error("vit_trainer_backward: the batch has no targets (forward-only batch)");
        return 1;
    }
    if (t.lowp()) t.backward_bf16(); else t.backward_f32();
    return vit::has_error();
}
int vit_trainer_step(vit_trainer_t* h, float lr) {
    h->t.step(lr);
    return vit::has_error();
}
int vit_trainer_train_step(vit_trainer_t* h, float lr, int b_global) {
    auto& t = h->t;
    vit_trainer_zero_grad(h);
    vit_trainer_forward(h, b_global);
    // the fused step knows lr before the backward: SGD per finished chunk (Trainer::early_sgd)
    t.early_on = t.early_sgd_on() && t.lowp() && !t.comm && t.two_streams && !t.timing && t.s2 && t.has_targets;
    t.early_lr = lr;
    vit_trainer_backward(h);
    t.early_done = t.early_on && !vit::has_error();
    t.early_on = false;
    vit_trainer_step(h, lr);
    return vit::has_error();
}
int vit_trainer_set_batch_jpeg(vit_trainer_t* h, vit_jpeg_loader_t* l, const float* mean3, const float* std3) {
    if (!h || !l || !mean3 || !std3) {
        set_error("vit_trainer_set_batch_jpeg: null argument");
        return 1;
    }
    return h->t.set_batch_jpeg(l, mean3, std3) ? 0 : 1;
}
int vit_trainer_set_batch_u8(vit_trainer_t* h, const unsigned char* images, const int* labels,
                             const float* mean3, const float* std3) {
    if (!h || !images || !mean3 || !std3) {
        set_error("vit_trainer_set_batch_u8: null argument");
        return 1;
    }
    if (labels && !labels_ok(labels, h->t.B, h->t.NC)) return 1;
    return h->t.set_batch_u8(images, labels, mean3, std3) ? 0 : 1;
}
int vit_trainer_step_adamw(vit_trainer_t* h, float lr, float beta1, float beta2, float eps,
                           float weight_decay) {
    h->t.step_adamw(lr, vit_adamw_t{beta1, beta2, eps, weight_decay});
    return vit::has_error();
}
int vit_trainer_get_adamw_state(vit_trainer_t* h, float* m, float* v, int* step) {
    auto& t = h->t;
    if (step) *step = t.adam_t;
    if (!t.adam_m) {
        set_error("vit_trainer_get_adamw_state: no AdamW step has run");
        return 1;
    }
    VIT_HIP(hipDeviceSynchronize());
    if (m) t.device_to_canon(t.adam_m, m);
    if (v) t.device_to_canon(t.adam_v, v);
    return vit::has_error();
}
int vit_trainer_eval(vit_trainer_t* h, int* host_pred, int* host_correct) {
    auto& t = h->t;
    if (host_correct) *host_correct = -1;
    t.b_global = t.B;
    if (t.lowp()) t.forward_bf16(); else t.forward_f32();
    VIT_HIP(hipMemsetAsync(t.preds + t.B, 0, 4, t.s));
    vit::argmax_rows_k<<<cdiv(t.B, 4), 256, 0, t.s>>>(t.preds, t.preds + t.B, t.logits,
                                                 t.has_targets ? t.labels : nullptr, t.B, t.NC);
    vit::after_launch("argmax_rows");
    std::vector<int> out(t.B + 1);
    VIT_HIP(hipMemcpyAsync(out.data(), t.preds, (size_t)(t.B + 1) * 4, hipMemcpyDeviceToHost, t.s));
    VIT_HIP(hipStreamSynchronize(t.s));
    if (vit::has_error()) return 1;
    if (host_pred) memcpy(host_pred, out.data(), (size_t)t.B * 4);
    if (host_correct && t.has_targets) *host_correct = out[t.B];
    return 0;
}
int vit_trainer_save_checkpoint(vit_trainer_t* h, const char* path) {
    auto& t = h->t;
    VIT_HIP(hipDeviceSynchronize());
    if (vit::has_error()) return 1;
    std::vector<float> p((size_t)t.n_params), m, v;
    t.device_to_canon(t.params, p.data());
    if (t.adam_m) {
        m.resize((size_t)t.n_params);
        v.resize((size_t)t.n_params);
        t.device_to_canon(t.adam_m, m.data());
        t.device_to_canon(t.adam_v, v.data());
    }
    if (vit::has_error()) return 1;
    return vit_checkpoint_write(path, &t.cfg, p.data(), t.adam_m ? m.data() : nullptr,
                                t.adam_m ? v.data() : nullptr, t.adam_t, &t.adam_hp);
}
int vit_trainer_load_checkpoint(vit_trainer_t* h, const char* path) {
    auto& t = h->t;
    vit_checkpoint_info_t info;
    if (vit_checkpoint_read_info(path, &info)) return 1;
    std::vector<float> p((size_t)t.n_params), m, v;
    if (info.has_opt) {
        m.resize((size_t)t.n_params);
        v.resize((size_t)t.n_params);
    }
    if (vit_checkpoint_read(path, &t.cfg, p.data(), info.has_opt ? m.data() : nullptr,
                            info.has_opt ? v.data() : nullptr))
        return 1;
    VIT_HIP(hipDeviceSynchronize());
    t.canon_to_device(p.data(), t.params);
    t.refresh_bf16();
    if (info.has_opt) {
        if (!t.ensure_adam()) return 1;
        t.canon_to_device(m.data(), t.adam_m);
        t.canon_to_device(v.data(), t.adam_v);
        t.adam_t = info.step;
        t.adam_hp = info.adamw;
    } else if (t.adam_m) {  // a parameters-only file restarts the optimizer
        VIT_HIP(hipMemsetAsync(t.adam_m, 0, t.arena_elems * 4, t.s));
        VIT_HIP(hipMemsetAsync(t.adam_v, 0, t.arena_elems * 4, t.s));
        t.adam_t = 0;
    }
    VIT_HIP(hipStreamSynchronize(t.s));
    return vit::has_error();
}
float vit_trainer_mean_loss(vit_trainer_t* h) {
    auto& t = h->t;
    if (!t.has_targets) return -1.0f;  // train_vit.rs:264-266
    std::vector<float> l(t.B);
    VIT_HIP(hipMemcpyAsync(l.data(), t.losses, t.B * 4, hipMemcpyDeviceToHost, t.s));
    VIT_HIP(hipStreamSynchronize(t.s));
    float m = 0.f;  // train_vit.rs:258-263
    for (float v : l) m += v;
    return m / (float)t.B;
}
int vit_trainer_get_logits(vit_trainer_t* h, float* out) {
    auto& t = h->t;
    VIT_HIP(hipMemcpyAsync(out, t.logits, (size_t)t.B * t.NC * 4, hipMemcpyDeviceToHost, t.s));
    VIT_HIP(hipStreamSynchronize(t.s));
    return vit::has_error();
}
int vit_trainer_sync(vit_trainer_t* h) {
    h->t.pre_side_wait();
    VIT_HIP(hipStreamSynchronize(h->t.s_comm));
    VIT_HIP(hipStreamSynchronize(h->t.s));
    return vit::has_error();
}
void* vit_trainer_stream(vit_trainer_t* h) { return (void*)h->t.s; }

int vit_layout_query(const vit_config_t* cfg, long long* tensor_off, long long* chunk_off, long long* arena_elems) {
    if (!cfg || cfg->num_layers < 1 || cfg->num_layers > VIT_MAX_LAYERS || cfg->patch < 1 || cfg->img < cfg->patch ||
        cfg->channels < 1 || cfg->num_classes < 1) {
        set_error("vit_layout_query: bad config");
        return -1;
    }
    const int L = cfg->num_layers, np = (cfg->img / cfg->patch) * (cfg->img / cfg->patch);
    long long canon[20], n_params = 0, co[VIT_MAX_LAYERS + 3], arena = 0;
    std::vector<long long> off;
    int n_chunks = 0;
    vit::compute_layout(cfg->channels, L, np + 1, cfg->in_ch * cfg->patch * cfg->patch, cfg->num_classes, canon,
                        n_params, off, co, n_chunks, arena);
    if (tensor_off) memcpy(tensor_off, off.data(), off.size() * sizeof(long long));
    if (chunk_off) memcpy(chunk_off, co, (size_t)(n_chunks + 1) * sizeof(long long));
    if (arena_elems) *arena_elems = arena;
    return n_chunks;
}
int vit_dp_unique_id_size(void) { return (int)sizeof(ncclUniqueId); }
int vit_dp_get_unique_id(char* out) {
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        set_error("ncclGetUniqueId: %s", ncclGetErrorString(r));
        return 1;
    }
    memcpy(out, &id, sizeof(id));
    return 0;
}
int vit_trainer_dp_init(vit_trainer_t* h, int rank, int world, const char* uid, int overlap) {
    auto& t = h->t;
    t.rank = rank;
    t.world = world;
    t.overlap = overlap;
    if (world < 1 || rank < 0 || rank >= world) {
        set_error("vit_trainer_dp_init: bad rank %d / world %d", rank, world);
        return 1;
    }
    ncclUniqueId id;
    memcpy(&id, uid, sizeof(id));
    VIT_HIP(hipSetDevice(t.device));
    ncclResult_t r = ncclCommInitRank(&t.comm, world, id, rank);
    if (r != ncclSuccess) {
        set_error("ncclCommInitRank(rank %d/%d): %s", rank, world, ncclGetErrorString(r));
        t.comm = nullptr;
        return 1;
    }
    return 0;
}
int vit_trainer_get_dp_snapshot(vit_trainer_t* h, float* host) {
    auto& t = h->t;
    if (!t.dp_probe_on) {
        set_error("vit_trainer_get_dp_snapshot: option dp_probe is off");
        return 1;
    }
    VIT_HIP(hipStreamSynchronize(t.s_comm));
    t.device_to_canon(t.dp_snap, host);
    return vit::has_error();
}
int vit_trainer_dp_ranks(vit_trainer_t* h) {
    if (!h->t.comm) return 0;
    int n = 0;
    ncclResult_t r = ncclCommCount(h->t.comm, &n);
    if (r != ncclSuccess) {
        set_error("ncclCommCount: %s", ncclGetErrorString(r));
        return -1;
    }
    return n;
}
int vit_trainer_set_concurrency(vit_trainer_t* h, int on) {
    auto& t = h->t;
    VIT_HIP(hipStreamSynchronize(t.s2));
    for (int k = 0; k < vit::Trainer::MAXMB; k++) if (t.ms[k]) VIT_HIP(hipStreamSynchronize(t.ms[k]));
    t.two_streams = on != 0;
    t.nmb = t.pick_nmb(t.mb_want);
    return vit::has_error();
}
int vit_trainer_set_option(vit_trainer_t* h, const char* name, int value) {
    auto& t = h->t;
    VIT_HIP(hipDeviceSynchronize());
    const std::string n = name ? name : "";
    if (n == "microbatch") {
        t.mb_want = value;
        t.nmb = t.pick_nmb(value);
    } else if (n == "dgrad_transposed") {
        t.dgrad_wt = value != 0;
    } else if (n == "fp8_ln_mx") {  // fp8: LayerNorm forward into the MX forms (default 1)
        t.ln_mx = value != 0;
    } else if (n == "fp8_ln_leftover") {  // fp8: LayerNorm -> MX forward, last partial round as rows (default 0)
        t.ln_left = value != 0;
    } else if (n == "early_sgd") {  // one GPU: SGD per finished gradient chunk inside train_step (default: fp8 mode only)
        t.early_sgd = value < 0 ? -1 : value != 0;
    } else if (n == "pre_side") {  // bf16 / fp8: gradient clear + transposed weights on s2 beside the forward (default 1)
        t.pre_side_wait();
        t.pre_side = value != 0;
    } else if (n == "patch_tail") {  // bf16 / fp8: patch embedding backward tail, see Trainer::patch_tail (default 1)
        t.patch_tail = value != 0;
    } else if (n == "head_splitk") {  // bf16 / fp8: the head GEMMs' split-K at ~4 K-steps per item (default 1)
        t.head_sk = value != 0;
    } else if (n == "fp8_lnb_mx") {  // fp8: the residual-gradient LayerNorm backwards write dres' MX forms (default 1)
        t.lnb_mx = value != 0;
    } else if (n == "dp_probe") {
        if (value && !t.dp_snap) {  // allocated once, kept until destroy
            t.dp_snap = t.alloc<float>(t.arena_elems);
            if (t.dp_snap) VIT_HIP(hipMemset(t.dp_snap, 0, t.arena_elems * 4));
        }
        t.dp_probe_on = value != 0 && t.dp_snap != nullptr;
    } else {
        set_error("vit_trainer_set_option: unknown option '%s'", n.c_str());
        return 1;
    }
    return vit::has_error();
}
int vit_trainer_set_timing(vit_trainer_t* h, int on) {
    h->t.timing = on != 0;
    return 0;
}
int vit_trainer_timing(vit_trainer_t* h, const char** names, double* ms, long long* calls,
                       double* flops, int max) {
    auto& t = h->t;
    t.collect();
    int n = 0;
    for (int c = 0; c < vit::TC_COUNT && n < max; c++) {
        if (!t.t_calls[c]) continue;
        names[n] = vit::kTimerNames[c];
        ms[n] = t.t_ms[c];
        calls[n] = t.t_calls[c];
        flops[n] = t.t_flops[c];
        n++;
    }
    return n;
}
void vit_trainer_timing_reset(vit_trainer_t* h) {
    auto& t = h->t;
    t.collect();
    for (int c = 0; c < vit::TC_COUNT; c++) {
        t.t_ms[c] = 0;
        t.t_calls[c] = 0;
        t.t_flops[c] = 0;
    }
}
}  // extern "C"
