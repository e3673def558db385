/*
 * oracle.c — CPU restatement of the reference ViT loops.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Every function cites the reference lines it restates.  Loop orders and the fp32 sequential
 * accumulation order are the reference's; the fixes of SURVEY.md §8a are marked Dn.
 */
#include "oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#if defined(ORACLE_F64)
#define R_EXP exp
#define R_LOG log
#define R_TANH tanh
#define R_COSH cosh
#define R_SQRT sqrt
#else
#define R_EXP expf
#define R_LOG logf
#define R_TANH tanhf
#define R_COSH coshf
#define R_SQRT sqrtf
#endif

typedef int64_t i64;

/* Threading (test infrastructure speed only): loops are split over OpenMP threads only along
 * indices whose outputs are disjoint, and every output element keeps the reference's sequential
 * accumulation order, so results are bitwise identical for any thread count.
 * ref_set_num_threads(1) gives the single-thread reference timing (bench.py cpu_baseline). */
void ref_set_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
int ref_get_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* train_vit.rs:376-382 */
void ref_residual_forward(real* out, const real* inp1, const real* inp2, int N) {
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < N; i++) out[i] = inp1[i] + inp2[i];
}

/* train_vit.rs:384-398 — out[bt,o] = b[o] + sum_i inp[bt,i] * W[o,i], sequential in i */
void ref_matmul_forward(real* out, const real* inp, const real* weight, const real* bias,
                        int B, int T, int C, int OC) {
#pragma omp parallel for schedule(static)
    for (i64 bt = 0; bt < (i64)B * T; bt++) {
        for (i64 o = 0; o < OC; o++) {
            real val = bias ? bias[o] : (real)0;
            const real* wrow = weight + o * C;
            const real* inp_bt = inp + bt * C;
            for (i64 i = 0; i < C; i++) val += inp_bt[i] * wrow[i];
            out[bt * OC + o] = val;
        }
    }
}

/* train_vit.rs:400-451 and attention.rs:1-57.
 * bth enumerates (b, t, h) with h fastest (train_vit.rs:406-407), so preatt/att are laid out
 * [B, T, NH, T] with row offset bth*T (D1: the reference's shadowed `t` used the position).
 * D2: every key of the row is normalised.  D3: ViT attention is non-causal (0..T); the causal
 * variant keeps the reference's 0..=t loop for a loop-structure KAT.  D16: -inf max init
 * (attention.rs:22), no expsum==0 guard (attention.rs:40). */
static void attention_forward_impl(real* out, real* preatt, real* att, const real* inp,
                                   int B, int T, int C, int NH, int causal) {
    const i64 C3 = (i64)C * 3;
    const int hs = C / NH;
    const real scale = (real)1.0 / R_SQRT((real)hs);
#pragma omp parallel for schedule(static)
    for (i64 bth = 0; bth < (i64)B * T * NH; bth++) {
        const i64 b = bth / ((i64)T * NH), t = (bth / NH) % T, h = bth % NH;
        const real* query_t = inp + (b * T + t) * C3 + h * hs;
        real* preatt_bth = preatt + bth * T;
        real* att_bth = att + bth * T;
        const i64 tend = causal ? t + 1 : T;

        real maxval = -INFINITY;
        for (i64 t2 = 0; t2 < tend; t2++) {
            const real* key_t2 = inp + (b * T + t2) * C3 + h * hs + C;
            real val = 0;
            for (int i = 0; i < hs; i++) val += query_t[i] * key_t2[i];
            val *= scale;
            if (val > maxval) maxval = val;
            preatt_bth[t2] = val;
        }
        real expsum = 0;
        for (i64 t2 = 0; t2 < tend; t2++) {
            real expv = R_EXP(preatt_bth[t2] - maxval);
            expsum += expv;
            att_bth[t2] = expv;
        }
        real expsum_inv = (real)1.0 / expsum;
        for (i64 t2 = 0; t2 < tend; t2++) att_bth[t2] *= expsum_inv; /* D2 */
        for (i64 t2 = tend; t2 < T; t2++) { preatt_bth[t2] = 0; att_bth[t2] = 0; }

        real* out_bth = out + (b * T + t) * C + h * hs;
        for (int i = 0; i < hs; i++) out_bth[i] = 0;
        for (i64 t2 = 0; t2 < tend; t2++) {
            const real* value_t2 = inp + (b * T + t2) * C3 + h * hs + (i64)C * 2;
            real a = att_bth[t2];
            for (int i = 0; i < hs; i++) out_bth[i] += a * value_t2[i];
        }
    }
}
void ref_attention_forward(real* out, real* preatt, real* att, const real* inp,
                           int B, int T, int C, int NH) {
    attention_forward_impl(out, preatt, att, inp, B, T, C, NH, 0);
}
void ref_attention_forward_causal(real* out, real* preatt, real* att, const real* inp,
                                  int B, int T, int C, int NH) {
    attention_forward_impl(out, preatt, att, inp, B, T, C, NH, 1);
}

/* train_vit.rs:453-480 */
void ref_layernorm_forward(real* out, real* mean, real* rstd, const real* inp,
                           const real* weight, const real* bias, int B, int T, int C) {
    const real eps = (real)1e-5;
#pragma omp parallel for schedule(static)
    for (i64 bt = 0; bt < (i64)B * T; bt++) {
        const real* x = inp + bt * C;
        real m = 0;
        for (int i = 0; i < C; i++) m += x[i];
        m /= (real)C;
        real v = 0;
        for (int i = 0; i < C; i++) {
            real xshift = x[i] - m;
            v += xshift * xshift;
        }
        v /= (real)C;
        real s = (real)1.0 / R_SQRT(v + eps);
        real* out_bt = out + bt * C;
        for (int i = 0; i < C; i++) {
            real n = s * (x[i] - m);
            real o = n * weight[i] + bias[i];
            out_bt[i] = o;
        }
        mean[bt] = m;
        rstd[bt] = s;
    }
}

static real gelu_s(void) { return R_SQRT((real)2.0 / (real)3.14159265358979323846); }

/* train_vit.rs:482-491 */
void ref_gelu_forward(real* out, const real* inp, int N) {
    const real s = gelu_s();
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < N; i++) {
        real x = inp[i];
        real cube = (real)0.044715 * x * x * x;
        out[i] = (real)0.5 * x * ((real)1.0 + R_TANH(s * (x + cube)));
    }
}

/* train_vit.rs:493-517 (max init -10000 kept, :499) */
void ref_softmax_forward(real* probs, const real* logits, int B, int T, int V) {
    for (i64 bt = 0; bt < (i64)B * T; bt++) {
        const real* logits_bt = logits + bt * V;
        real* probs_bt = probs + bt * V;
        real maxval = (real)-10000.0;
        for (int i = 0; i < V; i++)
            if (logits_bt[i] > maxval) maxval = logits_bt[i];
        real sum = 0;
        for (int i = 0; i < V; i++) {
            probs_bt[i] = R_EXP(logits_bt[i] - maxval);
            sum += probs_bt[i];
        }
        for (int i = 0; i < V; i++) probs_bt[i] /= sum;
    }
}

/* rusty_vit.rs:836-843, called train_vit.rs:256.  D6: loss = -log p[target] */
void ref_crossentropy_forward(real* losses, const real* probs, const int* targets,
                              int B, int T, int V) {
    for (i64 bt = 0; bt < (i64)B * T; bt++)
        losses[bt] = -R_LOG(probs[bt * V + targets[bt]]);
}

/* train_vit.rs:521-528 */
void ref_residual_backward(real* dinp1, real* dinp2, const real* dout, int N) {
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < N; i++) {
        dinp1[i] += dout[i];
        dinp2[i] += dout[i];
    }
}

/* train_vit.rs:530-557.  dinp may be NULL (skip dgrad: patch embedding has no pixel grad). */
void ref_matmul_backward(real* dinp, real* dweight, real* dbias, const real* dout,
                         const real* inp, const real* weight, int B, int T, int C, int OC) {
    const i64 BT = (i64)B * T;
    if (dinp) {
#pragma omp parallel for schedule(static)
        for (i64 bt = 0; bt < BT; bt++) {
            for (i64 o = 0; o < OC; o++) {
                const real d = dout[bt * OC + o];
                const real* wrow = weight + o * C;
                real* dinp_bt = dinp + bt * C;
                for (int i = 0; i < C; i++) dinp_bt[i] += wrow[i] * d;
            }
        }
    }
#pragma omp parallel for schedule(dynamic, 1)
    for (i64 o = 0; o < OC; o++) {
        for (i64 bt = 0; bt < BT; bt++) {
            const real d = dout[bt * OC + o];
            const real* inp_bt = inp + bt * C;
            real* dwrow = dweight + o * C;
            if (dbias) dbias[o] += d;
            for (int i = 0; i < C; i++) dwrow[i] += inp_bt[i] * d;
        }
    }
}

/* train_vit.rs:559-601, D1 (offsets by T), D3 (non-causal).  Keeps the reference's O(T^3)
 * softmax-Jacobian loop (:583-589).  dpreatt/datt are accumulated scratch, [B,T,NH,T]; when NULL
 * they are allocated (zeroed) internally. */
void ref_attention_backward(real* dinp, real* dpreatt, real* datt, const real* dout,
                            const real* inp, const real* att, int B, int T, int C, int NH) {
    const i64 C3 = (i64)C * 3;
    const int hs = C / NH;
    const real scale = (real)1.0 / R_SQRT((real)hs);
    const i64 n_scr = (i64)B * T * NH * T;
    real* own_dpre = NULL;
    real* own_datt = NULL;
    if (!dpreatt) dpreatt = own_dpre = (real*)calloc((size_t)n_scr, sizeof(real));
    if (!datt) datt = own_datt = (real*)calloc((size_t)n_scr, sizeof(real));

    /* (b, h) pairs in parallel: an iteration (b, t, h) touches only head h's columns of image b,
     * and inside a pair t ascends as in the reference's bth order */
#pragma omp parallel for schedule(dynamic, 1)
    for (i64 bh = 0; bh < (i64)B * NH; bh++)
    for (i64 t = 0; t < T; t++) {
        const i64 b = bh / NH, h = bh % NH, bth = (b * T + t) * NH + h;
        const real* att_bth = att + bth * T;
        real* datt_bth = datt + bth * T;
        real* dpreatt_bth = dpreatt + bth * T;
        real* dquery_t = dinp + (b * T + t) * C3 + h * hs;
        const real* query_t = inp + (b * T + t) * C3 + h * hs;
        const real* dout_bth = dout + (b * T + t) * C + h * hs;

        for (i64 t2 = 0; t2 < T; t2++) {
            const real* value_t2 = inp + (b * T + t2) * C3 + h * hs + (i64)C * 2;
            real* dvalue_t2 = dinp + (b * T + t2) * C3 + h * hs + (i64)C * 2;
            for (int i = 0; i < hs; i++) {
                datt_bth[t2] += value_t2[i] * dout_bth[i];
                dvalue_t2[i] += att_bth[t2] * dout_bth[i];
            }
        }
        for (i64 t2 = 0; t2 < T; t2++) {
            for (i64 t3 = 0; t3 < T; t3++) {
                real indicator = t2 == t3 ? (real)1.0 : (real)0.0;
                real local_derivative = att_bth[t2] * (indicator - att_bth[t3]);
                dpreatt_bth[t3] += local_derivative * datt_bth[t2];
            }
        }
        for (i64 t2 = 0; t2 < T; t2++) {
            const real* key_t2 = inp + (b * T + t2) * C3 + h * hs + C;
            real* dkey_t2 = dinp + (b * T + t2) * C3 + h * hs + C;
            for (int i = 0; i < hs; i++) {
                dquery_t[i] += key_t2[i] * dpreatt_bth[t2] * scale;
                dkey_t2[i] += query_t[i] * dpreatt_bth[t2] * scale;
            }
        }
    }
    free(own_dpre);
    free(own_datt);
}

/* train_vit.rs:603-637 (D5: (*inp_bt.add(i) - mean)) */
void ref_layernorm_backward(real* dinp, real* dweight, real* dbias, const real* dout,
                            const real* inp, const real* weight, const real* mean,
                            const real* rstd, int B, int T, int C) {
    /* dweight / dbias: each thread owns a column range and walks the rows in order (the
     * reference's per-element accumulation order); dinp: rows in parallel */
#pragma omp parallel
    {
#ifdef _OPENMP
        const int nth = omp_get_num_threads(), th = omp_get_thread_num();
#else
        const int nth = 1, th = 0;
#endif
        const int i0 = (int)((i64)C * th / nth), i1 = (int)((i64)C * (th + 1) / nth);
        for (i64 bt = 0; bt < (i64)B * T; bt++) {
            const real* dout_bt = dout + bt * C;
            const real* inp_bt = inp + bt * C;
            for (int i = i0; i < i1; i++) {
                real norm_bti = (inp_bt[i] - mean[bt]) * rstd[bt];
                dbias[i] += dout_bt[i];
                dweight[i] += norm_bti * dout_bt[i];
            }
        }
    }
#pragma omp parallel for schedule(static)
    for (i64 bt = 0; bt < (i64)B * T; bt++) {
        const real* dout_bt = dout + bt * C;
        const real* inp_bt = inp + bt * C;
        real* dinp_bt = dinp + bt * C;
        const real mean_bt = mean[bt];
        const real rstd_bt = rstd[bt];
        real dnorm_mean = 0;
        real dnorm_norm_mean = 0;
        for (int i = 0; i < C; i++) {
            real norm_bti = (inp_bt[i] - mean_bt) * rstd_bt;
            real dnorm_i = weight[i] * dout_bt[i];
            dnorm_mean += dnorm_i;
            dnorm_norm_mean += dnorm_i * norm_bti;
        }
        dnorm_mean /= (real)C;
        dnorm_norm_mean /= (real)C;
        for (int i = 0; i < C; i++) {
            real norm_bti = (inp_bt[i] - mean_bt) * rstd_bt;
            real dnorm_i = weight[i] * dout_bt[i];
            real dval = 0;
            dval += dnorm_i;
            dval -= dnorm_mean;
            dval -= norm_bti * dnorm_norm_mean;
            dval *= rstd_bt;
            dinp_bt[i] += dval;
        }
    }
}

/* train_vit.rs:639-653.  D4: sech^2 of the tanh argument itself (reference used cosh(2a)). */
void ref_gelu_backward(real* dinp, const real* inp, const real* dout, int N) {
    const real s = gelu_s();
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < N; i++) {
        real x = inp[i];
        real cube = (real)0.044715 * x * x * x;
        real tanh_arg = s * (x + cube);
        real tanh_out = R_TANH(tanh_arg);
        real coshf_out = R_COSH(tanh_arg); /* D4 */
        real sech_out = (real)1.0 / (coshf_out * coshf_out);
        real local_grad = (real)0.5 * ((real)1.0 + tanh_out) +
                          x * (real)0.5 * sech_out * s *
                              ((real)1.0 + (real)3.0 * (real)0.044715 * x * x);
        dinp[i] += local_grad * dout[i];
    }
}

/* undefined in the reference (called train_vit.rs:293); D6: dlogits += (p - 1[tgt]) * dloss */
void ref_crossentropy_softmax_backward(real* dlogits, const real* dlosses, const real* probs,
                                       const int* targets, int B, int T, int V) {
    for (i64 bt = 0; bt < (i64)B * T; bt++) {
        real* dlogits_bt = dlogits + bt * V;
        const real* probs_bt = probs + bt * V;
        const real dloss = dlosses[bt];
        const int ix = targets[bt];
        for (int i = 0; i < V; i++) {
            real p = probs_bt[i];
            real indicator = i == ix ? (real)1.0 : (real)0.0;
            dlogits_bt[i] += (p - indicator) * dloss;
        }
    }
}

/* D7: ViT patch embedding in place of encoder_forward (called train_vit.rs:196).
 * Row 0 of each image is the CLS token, rows 1..NP the patches in raster order; patch_w is
 * [C, IN_CH*P*P] with column (c*P + kh)*P + kw (Conv2d weight flatten order).  Each patch row
 * is a matmul_forward row (bias first, then the sequential dot product) plus wpe[t]. */
static void patch_row(real* dst, const real* pixels, int b, int p, int IMG, int P) {
    const int gw = IMG / P, ph = p / gw, pw = p % gw;
    int k = 0;
    for (int c = 0; c < 3; c++)
        for (int kh = 0; kh < P; kh++)
            for (int kw = 0; kw < P; kw++)
                dst[k++] = pixels[(((i64)b * 3 + c) * IMG + (i64)ph * P + kh) * IMG +
                                  (i64)pw * P + kw];
}

void ref_patch_embed_forward(real* encoded, const real* pixels, const real* patch_w,
                             const real* patch_b, const real* cls, const real* wpe,
                             int B, int IMG, int P, int C) {
    const int NP = (IMG / P) * (IMG / P), T = NP + 1, K = 3 * P * P;
#pragma omp parallel for schedule(static)
    for (int b = 0; b < B; b++) {
        real* row = (real*)malloc(sizeof(real) * (size_t)K);
        real* enc_b = encoded + (i64)b * T * C;
        for (int o = 0; o < C; o++) enc_b[o] = cls[o] + wpe[o];
        for (int p = 0; p < NP; p++) {
            patch_row(row, pixels, b, p, IMG, P);
            real* dst = enc_b + (i64)(1 + p) * C;
            for (int o = 0; o < C; o++) {
                real val = patch_b[o];
                const real* wrow = patch_w + (i64)o * K;
                for (int i = 0; i < K; i++) val += row[i] * wrow[i];
                dst[o] = val + wpe[(i64)(1 + p) * C + o];
            }
        }
        free(row);
    }
}

/* D7: encoder_backward (called train_vit.rs:371) for the patch embedding; no pixel gradient.
 * dpatch_w/dpatch_b follow matmul_backward's weight loop (o outer, rows middle, i inner). */
void ref_patch_embed_backward(real* dpatch_w, real* dpatch_b, real* dcls, real* dwpe,
                              const real* dencoded, const real* pixels,
                              int B, int IMG, int P, int C) {
    const int NP = (IMG / P) * (IMG / P), T = NP + 1, K = 3 * P * P;
    real* patches = (real*)malloc(sizeof(real) * (size_t)B * NP * K);
#pragma omp parallel for schedule(static)
    for (int b = 0; b < B; b++)
        for (int p = 0; p < NP; p++) patch_row(patches + ((i64)b * NP + p) * K, pixels, b, p, IMG, P);
#pragma omp parallel for schedule(dynamic, 1)
    for (int o = 0; o < C; o++) {
        for (int b = 0; b < B; b++) {
            for (int p = 0; p < NP; p++) {
                const real d = dencoded[((i64)b * T + 1 + p) * C + o];
                const real* prow = patches + ((i64)b * NP + p) * K;
                real* dwrow = dpatch_w + (i64)o * K;
                dpatch_b[o] += d;
                for (int i = 0; i < K; i++) dwrow[i] += prow[i] * d;
            }
        }
    }
    /* per element, images in ascending order (the reference's b-outer loop) */
#pragma omp parallel for schedule(static)
    for (int o = 0; o < C; o++)
        for (int b = 0; b < B; b++) dcls[o] += dencoded[(i64)b * T * C + o];
#pragma omp parallel for schedule(static)
    for (int t = 0; t < T; t++)
        for (int b = 0; b < B; b++)
            for (int o = 0; o < C; o++) dwpe[(i64)t * C + o] += dencoded[((i64)b * T + t) * C + o];
    free(patches);
}

/* train_vit.rs:737-743 */
void ref_sgd_step(real* params, const real* grads, long long n, real lr) {
    for (i64 i = 0; i < n; i++) params[i] -= lr * grads[i];
}

/* AdamW over the flat arena: the reference allocates m_memory / v_memory
 * (train_vit.rs:73-74, rusty_vit.rs:225-226) but its optimizer_step (train_vit.rs:737-743) is
 * plain SGD; this is the llm.c AdamW those buffers belong to, t = 1-based step.  Each line rounds
 * like the HIP kernel (no contraction): m, v, bias corrections, update with decoupled decay. */
void ref_adamw_step(real* params, const real* grads, real* m, real* v, long long n, real lr,
                    real beta1, real beta2, real eps, real weight_decay, int t) {
    const real bc1 = (real)1 - (real)pow((double)beta1, (double)t);
    const real bc2 = (real)1 - (real)pow((double)beta2, (double)t);
    for (i64 i = 0; i < n; i++) {
        const real g = grads[i];
        const real mi = beta1 * m[i] + ((real)1 - beta1) * g;
        const real vi = beta2 * v[i] + ((real)1 - beta2) * g * g;
        m[i] = mi;
        v[i] = vi;
        const real mh = mi / bc1, vh = vi / bc2;
        params[i] -= lr * (mh / (R_SQRT(vh) + eps) + weight_decay * params[i]);
    }
}

/* ------------------------------- model ------------------------------- */

long long ref_vit_param_sizes(const VitConfig* cfg, long long s[VIT_NUM_PARAM_TENSORS]) {
    const long long C = cfg->channels, L = cfg->num_layers, P = cfg->patch;
    const long long NP = (long long)(cfg->img / cfg->patch) * (cfg->img / cfg->patch);
    const long long T = NP + 1, K = (long long)cfg->in_ch * P * P, NC = cfg->num_classes;
    long long v[VIT_NUM_PARAM_TENSORS] = {
        C * K, C, C, T * C,                       /* patch_w patch_b cls wpe */
        L * C, L * C, L * 3 * C * C, L * 3 * C,   /* ln1w ln1b qkvw qkvb */
        L * C * C, L * C,                         /* attprojw attprojb */
        L * C, L * C, L * 4 * C * C, L * 4 * C,   /* ln2w ln2b fcw fcb */
        L * C * 4 * C, L * C,                     /* fcprojw fcprojb */
        C, C, NC * C, NC};                        /* lnfw lnfb head_w head_b */
    long long tot = 0;
    for (int i = 0; i < VIT_NUM_PARAM_TENSORS; i++) {
        s[i] = v[i];
        tot += v[i];
    }
    return tot;
}

void ref_vit_carve(const VitConfig* cfg, real* arena, VitParams* p) {
    long long s[VIT_NUM_PARAM_TENSORS];
    ref_vit_param_sizes(cfg, s);
    real** slots = (real**)p;
    for (int i = 0; i < VIT_NUM_PARAM_TENSORS; i++) {
        slots[i] = arena;
        arena += s[i];
    }
}

/* ActivationTensors (train_vit.rs:30-54), sized by B*T (D9); lnf/logits/probs/losses are the
 * CLS-row head (D15). */
typedef struct {
    real *encoded, *ln1, *ln1_mean, *ln1_rstd, *qkv, *atty, *preatt, *att, *attproj;
    real *residual2, *ln2, *ln2_mean, *ln2_rstd, *fch, *fch_gelu, *fcproj, *residual3;
    real *lnf, *lnf_mean, *lnf_rstd, *logits, *probs, *losses;
} Acts;

struct RefViT {
    VitConfig cfg;
    int B, T, NP;
    Acts a, g;
    real* a_mem;
    real* g_mem;
    long long n_acts;
    const real* pixels;
    int* targets;
    int B_global;
};

static long long carve_acts(const VitConfig* c, int B, int T, real* base, Acts* a) {
    const long long L = c->num_layers, C = c->channels, NH = c->num_heads, NC = c->num_classes;
    const long long BT = (long long)B * T;
    long long sz[23] = {BT * C,         L * BT * C, L * BT,     L * BT,     L * BT * 3 * C,
                        L * BT * C,     L * BT * NH * T,        L * BT * NH * T,
                        L * BT * C,     L * BT * C, L * BT * C, L * BT,     L * BT,
                        L * BT * 4 * C, L * BT * 4 * C,         L * BT * C, L * BT * C,
                        (long long)B * C, B,        B,          (long long)B * NC,
                        (long long)B * NC, B};
    long long tot = 0;
    real** slots = (real**)a;
    for (int i = 0; i < 23; i++) {
        slots[i] = base ? base + tot : NULL;
        tot += sz[i];
    }
    return tot;
}

RefViT* ref_vit_create(const VitConfig* cfg, int B) {
    RefViT* m = (RefViT*)calloc(1, sizeof(RefViT));
    m->cfg = *cfg;
    m->B = B;
    m->NP = (cfg->img / cfg->patch) * (cfg->img / cfg->patch);
    m->T = m->NP + 1;
    m->n_acts = carve_acts(cfg, B, m->T, NULL, &m->a);
    m->a_mem = (real*)calloc((size_t)m->n_acts, sizeof(real));
    m->g_mem = (real*)calloc((size_t)m->n_acts, sizeof(real));
    carve_acts(cfg, B, m->T, m->a_mem, &m->a);
    carve_acts(cfg, B, m->T, m->g_mem, &m->g);
    m->targets = (int*)calloc((size_t)B, sizeof(int));
    return m;
}

void ref_vit_destroy(RefViT* m) {
    if (!m) return;
    free(m->a_mem);
    free(m->g_mem);
    free(m->targets);
    free(m);
}

const real* ref_vit_logits(const RefViT* m) { return m->a.logits; }
const real* ref_vit_losses(const RefViT* m) { return m->a.losses; }
const real* ref_vit_probs(const RefViT* m) { return m->a.probs; }
const real* ref_vit_encoded(const RefViT* m) { return m->a.encoded; }

/* ViT::forward — train_vit.rs:188-268 */
real ref_vit_forward(RefViT* m, real* params, const real* pixels, const int* targets,
                     int B_global) {
    const VitConfig* c = &m->cfg;
    const int B = m->B, T = m->T, C = c->channels, L = c->num_layers, NH = c->num_heads;
    const int NC = c->num_classes;
    const i64 BTC = (i64)B * T * C, BT = (i64)B * T;
    VitParams p;
    ref_vit_carve(c, params, &p);
    Acts* a = &m->a;
    m->pixels = pixels;
    m->B_global = B_global;

    ref_patch_embed_forward(a->encoded, pixels, p.patch_w, p.patch_b, p.cls, p.wpe, B, c->img,
                            c->patch, C);
    real* residual = NULL;
    for (int l = 0; l < L; l++) {
        residual = l == 0 ? a->encoded : a->residual3 + (i64)(l - 1) * BTC;
        real* l_ln1w = p.ln1w + (i64)l * C;
        real* l_ln1b = p.ln1b + (i64)l * C;
        real* l_qkvw = p.qkvw + (i64)l * 3 * C * C;
        real* l_qkvb = p.qkvb + (i64)l * 3 * C;
        real* l_attprojw = p.attprojw + (i64)l * C * C;
        real* l_attprojb = p.attprojb + (i64)l * C;
        real* l_ln2w = p.ln2w + (i64)l * C;
        real* l_ln2b = p.ln2b + (i64)l * C;
        real* l_fcw = p.fcw + (i64)l * 4 * C * C;
        real* l_fcb = p.fcb + (i64)l * 4 * C;
        real* l_fcprojw = p.fcprojw + (i64)l * C * 4 * C;
        real* l_fcprojb = p.fcprojb + (i64)l * C;

        real* l_ln1 = a->ln1 + (i64)l * BTC;
        real* l_ln1_mean = a->ln1_mean + (i64)l * BT;
        real* l_ln1_rstd = a->ln1_rstd + (i64)l * BT;
        real* l_qkv = a->qkv + (i64)l * BTC * 3;
        real* l_atty = a->atty + (i64)l * BTC;
        real* l_preatt = a->preatt + (i64)l * BT * NH * T;
        real* l_att = a->att + (i64)l * BT * NH * T;
        real* l_attproj = a->attproj + (i64)l * BTC;
        real* l_residual2 = a->residual2 + (i64)l * BTC;
        real* l_ln2 = a->ln2 + (i64)l * BTC;
        real* l_ln2_mean = a->ln2_mean + (i64)l * BT;
        real* l_ln2_rstd = a->ln2_rstd + (i64)l * BT;
        real* l_fch = a->fch + (i64)l * BTC * 4;
        real* l_fch_gelu = a->fch_gelu + (i64)l * BTC * 4;
        real* l_fcproj = a->fcproj + (i64)l * BTC;
        real* l_residual3 = a->residual3 + (i64)l * BTC;

        ref_layernorm_forward(l_ln1, l_ln1_mean, l_ln1_rstd, residual, l_ln1w, l_ln1b, B, T, C);
        ref_matmul_forward(l_qkv, l_ln1, l_qkvw, l_qkvb, B, T, C, 3 * C);
        ref_attention_forward(l_atty, l_preatt, l_att, l_qkv, B, T, C, NH);
        ref_matmul_forward(l_attproj, l_atty, l_attprojw, l_attprojb, B, T, C, C);
        ref_residual_forward(l_residual2, residual, l_attproj, (int)BTC);
        ref_layernorm_forward(l_ln2, l_ln2_mean, l_ln2_rstd, l_residual2, l_ln2w, l_ln2b, B, T, C);
        ref_matmul_forward(l_fch, l_ln2, l_fcw, l_fcb, B, T, C, 4 * C);
        ref_gelu_forward(l_fch_gelu, l_fch, (int)(BTC * 4));
        ref_matmul_forward(l_fcproj, l_fch_gelu, l_fcprojw, l_fcprojb, B, T, 4 * C, C);
        ref_residual_forward(l_residual3, l_residual2, l_fcproj, (int)BTC);
    }
    /* D15: final LN + classifier head on the CLS row (row 0) of each image */
    residual = a->residual3 + (i64)(L - 1) * BTC;
    for (int b = 0; b < B; b++)
        ref_layernorm_forward(a->lnf + (i64)b * C, a->lnf_mean + b, a->lnf_rstd + b,
                              residual + (i64)b * T * C, p.lnfw, p.lnfb, 1, 1, C);
    ref_matmul_forward(a->logits, a->lnf, p.head_w, p.head_b, B, 1, C, NC);
    ref_softmax_forward(a->probs, a->logits, B, 1, NC);
    if (!targets) return (real)-1.0;
    memcpy(m->targets, targets, sizeof(int) * (size_t)B);
    ref_crossentropy_forward(a->losses, a->probs, m->targets, B, 1, NC);
    real mean_loss = 0;
    for (int i = 0; i < B; i++) mean_loss += a->losses[i];
    mean_loss /= (real)B;
    return mean_loss;
}

/* ViT::backward — train_vit.rs:271-373.  Accumulates into grads (caller zeroes them);
 * grads_acts are zeroed here (the elided zeroing of :272). */
void ref_vit_backward(RefViT* m, real* params, real* grads) {
    const VitConfig* c = &m->cfg;
    const int B = m->B, T = m->T, C = c->channels, L = c->num_layers, NH = c->num_heads;
    const int NC = c->num_classes;
    const i64 BTC = (i64)B * T * C, BT = (i64)B * T;
    VitParams p, g;
    ref_vit_carve(c, params, &p);
    ref_vit_carve(c, grads, &g);
    Acts* a = &m->a;
    Acts* ga = &m->g;
    memset(m->g_mem, 0, sizeof(real) * (size_t)m->n_acts);

    const real dloss_mean = (real)1.0 / (real)m->B_global; /* D15: 1/B_global */
    for (int i = 0; i < B; i++) ga->losses[i] = dloss_mean;
    ref_crossentropy_softmax_backward(ga->logits, ga->losses, a->probs, m->targets, B, 1, NC);
    ref_matmul_backward(ga->lnf, g.head_w, g.head_b, ga->logits, a->lnf, p.head_w, B, 1, C, NC);

    real* residual = a->residual3 + (i64)(L - 1) * BTC;
    real* dresidual = ga->residual3 + (i64)(L - 1) * BTC;
    for (int b = 0; b < B; b++)
        ref_layernorm_backward(dresidual + (i64)b * T * C, g.lnfw, g.lnfb, ga->lnf + (i64)b * C,
                               residual + (i64)b * T * C, p.lnfw, a->lnf_mean + b,
                               a->lnf_rstd + b, 1, 1, C);

    for (int l = L - 1; l >= 0; l--) {
        residual = l == 0 ? a->encoded : a->residual3 + (i64)(l - 1) * BTC;
        dresidual = l == 0 ? ga->encoded : ga->residual3 + (i64)(l - 1) * BTC;

        real* l_ln1w = p.ln1w + (i64)l * C;
        real* l_qkvw = p.qkvw + (i64)l * 3 * C * C;
        real* l_attprojw = p.attprojw + (i64)l * C * C;
        real* l_ln2w = p.ln2w + (i64)l * C;
        real* l_fcw = p.fcw + (i64)l * 4 * C * C;
        real* l_fcprojw = p.fcprojw + (i64)l * C * 4 * C;

        real* dl_ln1w = g.ln1w + (i64)l * C;
        real* dl_ln1b = g.ln1b + (i64)l * C;
        real* dl_qkvw = g.qkvw + (i64)l * 3 * C * C;
        real* dl_qkvb = g.qkvb + (i64)l * 3 * C;
        real* dl_attprojw = g.attprojw + (i64)l * C * C;
        real* dl_attprojb = g.attprojb + (i64)l * C;
        real* dl_ln2w = g.ln2w + (i64)l * C;
        real* dl_ln2b = g.ln2b + (i64)l * C;
        real* dl_fcw = g.fcw + (i64)l * 4 * C * C;
        real* dl_fcb = g.fcb + (i64)l * 4 * C;
        real* dl_fcprojw = g.fcprojw + (i64)l * C * 4 * C;
        real* dl_fcprojb = g.fcprojb + (i64)l * C;

        real* l_ln1 = a->ln1 + (i64)l * BTC;
        real* l_ln1_mean = a->ln1_mean + (i64)l * BT;
        real* l_ln1_rstd = a->ln1_rstd + (i64)l * BT;
        real* l_qkv = a->qkv + (i64)l * BTC * 3;
        real* l_atty = a->atty + (i64)l * BTC;
        real* l_att = a->att + (i64)l * BT * NH * T;
        real* l_residual2 = a->residual2 + (i64)l * BTC;
        real* l_ln2 = a->ln2 + (i64)l * BTC;
        real* l_ln2_mean = a->ln2_mean + (i64)l * BT;
        real* l_ln2_rstd = a->ln2_rstd + (i64)l * BT;
        real* l_fch = a->fch + (i64)l * BTC * 4;
        real* l_fch_gelu = a->fch_gelu + (i64)l * BTC * 4;

        real* dl_ln1 = ga->ln1 + (i64)l * BTC;
        real* dl_qkv = ga->qkv + (i64)l * BTC * 3;
        real* dl_atty = ga->atty + (i64)l * BTC;
        real* dl_preatt = ga->preatt + (i64)l * BT * NH * T;
        real* dl_att = ga->att + (i64)l * BT * NH * T;
        real* dl_attproj = ga->attproj + (i64)l * BTC;
        real* dl_residual2 = ga->residual2 + (i64)l * BTC;
        real* dl_ln2 = ga->ln2 + (i64)l * BTC;
        real* dl_fch = ga->fch + (i64)l * BTC * 4;
        real* dl_fch_gelu = ga->fch_gelu + (i64)l * BTC * 4;
        real* dl_fcproj = ga->fcproj + (i64)l * BTC;
        real* dl_residual3 = ga->residual3 + (i64)l * BTC;

        ref_residual_backward(dl_residual2, dl_fcproj, dl_residual3, (int)BTC);
        ref_matmul_backward(dl_fch_gelu, dl_fcprojw, dl_fcprojb, dl_fcproj, l_fch_gelu, l_fcprojw,
                            B, T, 4 * C, C);
        ref_gelu_backward(dl_fch, l_fch, dl_fch_gelu, (int)(BTC * 4));
        ref_matmul_backward(dl_ln2, dl_fcw, dl_fcb, dl_fch, l_ln2, l_fcw, B, T, C, 4 * C);
        ref_layernorm_backward(dl_residual2, dl_ln2w, dl_ln2b, dl_ln2, l_residual2, l_ln2w,
                               l_ln2_mean, l_ln2_rstd, B, T, C);
        ref_residual_backward(dresidual, dl_attproj, dl_residual2, (int)BTC);
        ref_matmul_backward(dl_atty, dl_attprojw, dl_attprojb, dl_attproj, l_atty, l_attprojw,
                            B, T, C, C);
        ref_attention_backward(dl_qkv, dl_preatt, dl_att, dl_atty, l_qkv, l_att, B, T, C, NH);
        ref_matmul_backward(dl_ln1, dl_qkvw, dl_qkvb, dl_qkv, l_ln1, l_qkvw, B, T, C, 3 * C);
        ref_layernorm_backward(dresidual, dl_ln1w, dl_ln1b, dl_ln1, residual, l_ln1w, l_ln1_mean,
                               l_ln1_rstd, B, T, C);
    }
    ref_patch_embed_backward(g.patch_w, g.patch_b, g.cls, g.wpe, ga->encoded, m->pixels, B,
                             c->img, c->patch, C);
}
