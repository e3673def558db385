/*
 * oracle.h — CPU restatement of the reference ViT training loops (TEST INFRASTRUCTURE).
 *
 * This is the parity checker, not the product.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product path (vit.rs_amd/, libvit_hip.so) never
 * links or calls anything here.
 *
 * What it restates: the layer ops and forward/backward orchestration of
 *   /root/reference/train_vit.rs:376-670  (ops, canonical c_int signatures)
 *   /root/reference/train_vit.rs:188-373  (ViT::forward / ViT::backward op order)
 *   /root/reference/attention.rs:1-57     (-inf max init variant of attention_forward)
 *   /root/reference/rusty_vit.rs:836-843  (crossentropy_forward placement)
 * with the defect fixes D1-D16 of SURVEY.md §8a (each applied fix is marked "Dn" at its line).
 * The reference is Rust, has no Cargo manifest and does not compile, so there
 * is no oracle/_ref build; parity is pinned by the reference's own known-answer tests
 * (tests/vit_tests.rs, corrected per D14), fp64 central finite differences of every backward op,
 * and an independent torch-CPU fp64 autograd cross-check whose outputs are committed under
 * tests/golden/ (see tests/golden/make_golden.py).
 *
 * Numerics: compiled with -O2 -ffp-contract=off (no FMA contraction, no fast-math) so that each
 * `a*b + c` rounds twice like the reference's Rust code, and every reduction runs in the
 * reference's sequential index order.  REAL is float for the parity oracle (liboracle_f32.so)
 * and double for the finite-difference / torch cross-check build (liboracle_f64.so).
 *
 * Dims are int like the reference's c_int; every offset is computed in 64-bit (D10).
 */
#ifndef VIT_ORACLE_H
#define VIT_ORACLE_H

#include <stddef.h>

#ifndef REAL
#define REAL float
#endif
typedef REAL real;

#ifdef __cplusplus
extern "C" {
#endif

/* ---- layer ops (reference names with a ref_ prefix; forward overwrites, backward accumulates) ---- */
void ref_residual_forward(real* out, const real* inp1, const real* inp2, int N);
void ref_matmul_forward(real* out, const real* inp, const real* weight, const real* bias,
                        int B, int T, int C, int OC);
void ref_attention_forward(real* out, real* preatt, real* att, const real* inp,
                           int B, int T, int C, int NH);
void ref_attention_forward_causal(real* out, real* preatt, real* att, const real* inp,
                                  int B, int T, int C, int NH);
void ref_layernorm_forward(real* out, real* mean, real* rstd, const real* inp,
                           const real* weight, const real* bias, int B, int T, int C);
void ref_gelu_forward(real* out, const real* inp, int N);
void ref_softmax_forward(real* probs, const real* logits, int B, int T, int V);
void ref_crossentropy_forward(real* losses, const real* probs, const int* targets,
                              int B, int T, int V);

void ref_residual_backward(real* dinp1, real* dinp2, const real* dout, int N);
void ref_matmul_backward(real* dinp, real* dweight, real* dbias, const real* dout,
                         const real* inp, const real* weight, int B, int T, int C, int OC);
void ref_attention_backward(real* dinp, real* dpreatt, real* datt, const real* dout,
                            const real* inp, const real* att, int B, int T, int C, int NH);
void ref_layernorm_backward(real* dinp, real* dweight, real* dbias, const real* dout,
                            const real* inp, const real* weight, const real* mean,
                            const real* rstd, int B, int T, int C);
void ref_gelu_backward(real* dinp, const real* inp, const real* dout, int N);
void ref_crossentropy_softmax_backward(real* dlogits, const real* dlosses, const real* probs,
                                       const int* targets, int B, int T, int V);

/* ViT replacement of the reference's undefined encoder_forward/backward (D7). */
void ref_patch_embed_forward(real* encoded, const real* pixels, const real* patch_w,
                             const real* patch_b, const real* cls, const real* wpe,
                             int B, int IMG, int P, int C);
void ref_patch_embed_backward(real* dpatch_w, real* dpatch_b, real* dcls, real* dwpe,
                              const real* dencoded, const real* pixels,
                              int B, int IMG, int P, int C);
/* optimizer_step (train_vit.rs:737-743): p -= lr * g */
void ref_sgd_step(real* params, const real* grads, long long n, real lr);
/* OpenMP thread count of the oracle (bitwise-identical results for any count; 1 = the
 * single-thread reference timing) */
void ref_set_num_threads(int n);
int ref_get_num_threads(void);
void ref_adamw_step(real* params, const real* grads, real* m, real* v, long long n, real lr,
                    real beta1, real beta2, real eps, real weight_decay, int t);

/* ---- model level (train_vit.rs:9-86 structs, :188-373 forward/backward) ---- */
typedef struct {
    int img, patch, in_ch, channels, num_layers, num_heads, num_classes;
} VitConfig;

#define VIT_NUM_PARAM_TENSORS 20
/* Canonical (reference, type-major) parameter order: the reference's 16 ParameterTensors
 * (train_vit.rs:10-27) with wte -> patch_w/patch_b/cls and the LM head -> head_w/head_b. */
typedef struct {
    real *patch_w, *patch_b, *cls, *wpe;
    real *ln1w, *ln1b, *qkvw, *qkvb, *attprojw, *attprojb;
    real *ln2w, *ln2b, *fcw, *fcb, *fcprojw, *fcprojb;
    real *lnfw, *lnfb, *head_w, *head_b;
} VitParams;

/* element counts of the 20 tensors in canonical order; returns the total */
long long ref_vit_param_sizes(const VitConfig* cfg, long long sizes[VIT_NUM_PARAM_TENSORS]);
/* carve a flat canonical arena into the pointer table (train_vit.rs:145-161) */
void ref_vit_carve(const VitConfig* cfg, real* arena, VitParams* out);

typedef struct RefViT RefViT;
RefViT* ref_vit_create(const VitConfig* cfg, int B);
void ref_vit_destroy(RefViT* m);
/* params/grads: flat canonical arenas owned by the caller */
real ref_vit_forward(RefViT* m, real* params, const real* pixels, const int* targets,
                     int B_global);
void ref_vit_backward(RefViT* m, real* params, real* grads);
/* read-only views of a few activations for parity tests */
const real* ref_vit_logits(const RefViT* m);
const real* ref_vit_losses(const RefViT* m);
const real* ref_vit_probs(const RefViT* m);
const real* ref_vit_encoded(const RefViT* m);

#ifdef __cplusplus
}
#endif
#endif
