/*
 * vit_trainer.h — C ABI of the native host trainer in libvit_hip.so.
 *
 * Mirrors the reference's model-level interface (/root/reference/train_vit.rs):
 *   struct ViT + build_from_checkpoint (:65-186)  -> vit_trainer_create + vit_trainer_set_params
 *   ViT::forward(inputs, targets, B, T) (:188)     -> vit_trainer_set_batch + vit_trainer_forward
 *   ViT::backward() (:271)                         -> vit_trainer_zero_grad + vit_trainer_backward
 *   optimizer_step(&mut ViT, lr) (:737)            -> vit_trainer_step
 *   mean_loss field (:85, :263)                    -> vit_trainer_mean_loss
 * Parameters cross this boundary in the reference's canonical type-major order (the 16
 * ParameterTensors of train_vit.rs:10-27 / param_sizes :115-131, with wte -> patch_w, patch_b,
 * cls and the tied LM head -> head_w, head_b; 20 tensors).  On the device the trainer keeps them
 * layer-major in reverse layer order so that backward finalises one contiguous gradient range per
 * layer (the unit of the overlapped RCCL all-reduce).
 *
 * Precision modes:
 *   VIT_FP32 (0): the reference op sequence on the GPU (the fp32 C-ABI ops of vit_ops.h,
 *                 materialised attention) — the parity path (<= 1e-4 rel vs the CPU oracle).
 *   VIT_BF16 (1): the fast path — bf16 MFMA GEMMs with fused epilogues, fused attention,
 *                 fp32 master weights / gradients / residual stream / LN statistics.
 *                 Head sizes 32/64/80/96/128 use the MFMA attention while T <= 320 (generic
 *                 VALU kernels beyond), and a patch whose 3*P*P is not a multiple of 8 runs the
 *                 patch embedding on the fp32 GEMM.
 *   VIT_FP8 (2):  BASELINE config 5 ("fp8 weights/activations"): VIT_BF16 with the forward and
 *                 input-gradient GEMMs of every layer (qkv, proj, fc, fcproj) on MXFP8 operands
 *                 (OCP e4m3 + one E8M0 scale per 32 k-elements, v_mfma_scale_f32_32x32x64_f8f6f4);
 *                 weights quantized from the fp32 master after every optimizer step, activations /
 *                 output gradients quantized as each GEMM consumes them.  Weight gradients,
 *                 attention, LayerNorm, the residual stream and the optimizer stay bf16 / fp32.
 *                 Needs C % 64 == 0.
 * All calls are asynchronous on the trainer's stream unless noted; functions returning int
 * return 0 on success (details via vit_last_error()).
 */
#ifndef VIT_TRAINER_H
#define VIT_TRAINER_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int img, patch, in_ch, channels, num_layers, num_heads, num_classes;
} vit_config_t;

enum { VIT_FP32 = 0, VIT_BF16 = 1, VIT_FP8 = 2 };
enum { VIT_NUM_PARAM_TENSORS = 20 };
enum { VIT_MAX_LAYERS = 64 };  /* num_layers range accepted by vit_trainer_create / vit_layout_query */

typedef struct vit_trainer vit_trainer_t;

vit_trainer_t* vit_trainer_create(const vit_config_t* cfg, int batch, int precision, int device);
void vit_trainer_destroy(vit_trainer_t* t);
long long vit_trainer_num_params(const vit_trainer_t* t);
/* bytes of device memory held by the trainer */
long long vit_trainer_device_bytes(const vit_trainer_t* t);
/* canonical (type-major) fp32 host arrays of vit_trainer_num_params() elements; synchronous */
int vit_trainer_set_params(vit_trainer_t* t, const float* host_params);
int vit_trainer_get_params(vit_trainer_t* t, float* host_params);
int vit_trainer_get_grads(vit_trainer_t* t, float* host_grads);
/* pixels [batch,3,img,img] fp32, labels [batch] int32 (host); synchronous upload.
 * labels NULL = a forward-only batch (the reference's targets == null branch, train_vit.rs:
 * 254-266): no loss, vit_trainer_mean_loss returns -1, vit_trainer_backward fails */
int vit_trainer_set_batch(vit_trainer_t* t, const float* host_pixels, const int* host_labels);
/* same from device pointers (stream-ordered device copy) */
int vit_trainer_set_batch_device(vit_trainer_t* t, const float* dev_pixels, const int* dev_labels);
/* forward; b_global = global batch of the data-parallel job (dloss = 1/b_global, D15) */
int vit_trainer_forward(vit_trainer_t* t, int b_global);
int vit_trainer_zero_grad(vit_trainer_t* t);
int vit_trainer_backward(vit_trainer_t* t);   /* also launches the overlapped all-reduce (DP) */
int vit_trainer_step(vit_trainer_t* t, float lr); /* waits for the all-reduce, then SGD */
/* AdamW: the update the reference's m_memory / v_memory (train_vit.rs:73-74)
 * were allocated for, which its SGD optimizer_step (:737) never runs.  t = number of AdamW steps
 * so far + 1 (kept by the trainer, saved in checkpoints); m, v are allocated and zeroed on the
 * first call.  Decoupled weight decay on every parameter:
 *   m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g g;  p -= lr (m/(1-b1^t) / (sqrt(v/(1-b2^t)) + eps) + wd p) */
int vit_trainer_step_adamw(vit_trainer_t* t, float lr, float beta1, float beta2, float eps,
                           float weight_decay);
/* canonical host copies of m, v (either may be NULL) and the step count; synchronous */
int vit_trainer_get_adamw_state(vit_trainer_t* t, float* m, float* v, int* step);
/* eval: forward of the current batch, then top-1 per image on the device.
 * host_pred [batch] (nullable) gets the predicted classes (first maximum, as numpy.argmax);
 * host_correct (nullable) gets the number equal to the labels, or -1 when the batch was set
 * without labels.  Synchronous. */
int vit_trainer_eval(vit_trainer_t* t, int* host_pred, int* host_correct);
/* zero_grad + forward + backward + step */
int vit_trainer_train_step(vit_trainer_t* t, float lr, int b_global);
/* synchronous readbacks; mean_loss = -1 for a batch without labels */
float vit_trainer_mean_loss(vit_trainer_t* t);
int vit_trainer_get_logits(vit_trainer_t* t, float* host_logits); /* [batch, num_classes] */
int vit_trainer_sync(vit_trainer_t* t);
void* vit_trainer_stream(vit_trainer_t* t);

/* device gradient-arena layout (host-only, no GPU needed): tensor_off [20 * num_layers] element
 * offsets of tensor ti (canonical order), layer l at [ti * num_layers + l] (unlayered tensors:
 * l = 0, the other entries 0); chunk_off [num_layers + 3] boundaries of the all-reduce chunks in
 * backward's completion order (0 = head + final LN, 1..L = layers L-1..0, L+1 = embedding);
 * arena_elems = arena size (with 64-element alignment padding).  Returns the chunk count (L + 2),
 * -1 on a bad config.  Any pointer may be NULL. */
int vit_layout_query(const vit_config_t* cfg, long long* tensor_off, long long* chunk_off,
                     long long* arena_elems);

/* ---- data parallelism over RCCL (one process per GPU) ---- */
int vit_dp_unique_id_size(void);
int vit_dp_get_unique_id(char* out);   /* rank 0 creates; broadcast the bytes out of band */
/* chunks: 0 = one all-reduce of the whole gradient arena after backward;
 *         1 = per-layer chunks on a side stream overlapped with backward (default) */
int vit_trainer_dp_init(vit_trainer_t* t, int rank, int world, const char* unique_id, int overlap);
/* ranks of the trainer's RCCL communicator (ncclCommCount); 0 before vit_trainer_dp_init */
int vit_trainer_dp_ranks(vit_trainer_t* t);

/* ---- stream concurrency (bf16 mode): on (default) = the batch runs as two micro-batch row halves
 *      on two streams and the weight-gradient GEMMs on a third; off = one stream, kernels one at a
 *      time (per-kernel roofline timing).  Call between steps. ---- */
int vit_trainer_set_concurrency(vit_trainer_t* t, int on);
/* ---- tuning options for A/B measurements in one process (call between steps):
 *      "microbatch" = number of micro-batch streams wanted (1 .. 4; the largest divisor of B),
 *      "dgrad_transposed" = 1 (default): dgrad GEMMs read the transposed weight copy,
 *      "fp8_ln_mx" = 1 (default): fp8 mode's LayerNorm forwards write the MX forms directly,
 *      "fp8_lnb_mx" = 1 (default): ... and its residual-gradient LayerNorm backwards those of dres,
 *      "head_splitk" = 1 (default): bf16 / fp8 modes split the classifier head's GEMMs at about
 *      four K-steps per work item (0: the fp32 engine's own split rule),
 *      "early_sgd" = -1 (default: on in fp8 mode, off in bf16; measured per dtype): one GPU, bf16 / fp8, concurrency on: vit_trainer_train_step
 *      updates each gradient chunk (head, layer L-1 .. 0, embedding) as soon as the backward has
 *      finished it, on a side stream beside the rest of the backward (same bits as one pass),
 *      "pre_side" = 1 (default): bf16 / fp8 modes with concurrency on clear the gradient arena
 *      (vit_trainer_zero_grad) and refresh the transposed weight copies on the weight-gradient
 *      stream beside the forward; the backward (and every host read) waits for them,
 *      "patch_tail" = 1 (default): bf16 / fp8 modes split the patch embedding's weight gradient for
 *      80 % of the GPU and run its small gradients on a second stream beside it (0: one stream, 45 %),
 *      "dp_probe" = 1: every gradient chunk is also copied, on the all-reduce stream right after
 *      its all-reduce, into a snapshot arena (read with vit_trainer_get_dp_snapshot) — a check
 *      that each overlapped chunk was final when it was reduced.
 *      Returns non-zero (and sets the error) for an unknown name. ---- */
int vit_trainer_set_option(vit_trainer_t* t, const char* name, int value);
/* canonical host copy of the dp_probe snapshot arena; synchronous */
int vit_trainer_get_dp_snapshot(vit_trainer_t* t, float* host);

/* ---- per-kernel-class timing with HIP events on the stream each kernel runs on ---- */
int vit_trainer_set_timing(vit_trainer_t* t, int on);
/* fills up to max entries; returns the number of classes. names point to static strings */
int vit_trainer_timing(vit_trainer_t* t, const char** names, double* total_ms, long long* calls,
                       double* flops, int max);
void vit_trainer_timing_reset(vit_trainer_t* t);

#ifdef __cplusplus
}
#endif
#endif
