/*
 * vit_checkpoint.h — ViT checkpoint files, host-only functions of libvit_hip.so.
 *
 * The reference's loader, ViT::build_from_checkpoint (/root/reference/train_vit.rs:89-186),
 * follows the llm.c convention: a 256-entry header at byte 0, the fp32 parameters in canonical
 * type-major order at byte 1024.  Its save_checkpoint / load_checkpoint (:715-735) write and read
 * only `wte`, with no header, and it reads the header into a byte array (D8), so the
 * reference has no complete format to stay compatible with.  This one keeps the convention and
 * completes it for the ViT tensors:
 *
 *   int32 header[256] (little endian) at byte 0
 *     [0] VIT_CKPT_MAGIC   [1] VIT_CKPT_VERSION
 *     [2] max_seq_len T = (img/patch)^2 + 1    (the reference's header[2])
 *     [3] num_classes     (the reference's vocab_size slot, header[3])
 *     [4] num_layers  [5] num_heads  [6] channels   (header[4..6], as the reference)
 *     [7] img  [8] patch  [9] in_ch
 *     [10] flags: bit 0 = AdamW state (m, v) follows the parameters
 *     [11] AdamW step t (number of completed AdamW updates)
 *     [12] / [13] num_params, low / high 32 bits
 *     [14..17] beta1, beta2, eps, weight_decay of the last AdamW update (IEEE fp32 bits)
 *     rest zero
 *   fp32 params[num_params] at byte 1024, in the 20-tensor canonical order of vit_trainer.h
 *   (patch_w, patch_b, cls, wpe, ln1w .. fcprojb (each [L, ...]), lnfw, lnfb, head_w, head_b)
 *   if flags & 1: fp32 m[num_params], then fp32 v[num_params], same order.
 *
 * All functions return 0 on success; on failure non-zero with the reason in vit_last_error().
 */
#ifndef VIT_CHECKPOINT_H
#define VIT_CHECKPOINT_H

#include "vit_trainer.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { VIT_CKPT_MAGIC = 20261016, VIT_CKPT_VERSION = 1, VIT_CKPT_HEADER_BYTES = 1024 };

typedef struct {
    float beta1, beta2, eps, weight_decay;
} vit_adamw_t;

typedef struct {
    vit_config_t cfg;
    long long num_params;
    int has_opt;        /* AdamW m / v present */
    int step;           /* AdamW t */
    vit_adamw_t adamw;
} vit_checkpoint_info_t;

/* canonical parameter count of a config (sum of the 20 tensor sizes) */
long long vit_config_num_params(const vit_config_t* cfg);
/* header only; validates magic, version, T == (img/patch)^2+1 and the file size */
int vit_checkpoint_read_info(const char* path, vit_checkpoint_info_t* info);
/* m, v: NULL for a parameters-only file (then step / adamw are ignored) */
int vit_checkpoint_write(const char* path, const vit_config_t* cfg, const float* params,
                         const float* m, const float* v, int step, const vit_adamw_t* adamw);
/* reads params (and m, v when non-NULL and present in the file) of num_params elements; fails if
 * the file's config differs from *cfg */
int vit_checkpoint_read(const char* path, const vit_config_t* cfg, float* params, float* m,
                        float* v);

/* ---- trainer-level save / resume (synchronous).  Save writes the AdamW state once an AdamW
 *      step has run; load restores params (and m, v, t when present) and refreshes the bf16
 *      shadows. ---- */
int vit_trainer_save_checkpoint(vit_trainer_t* t, const char* path);
int vit_trainer_load_checkpoint(vit_trainer_t* t, const char* path);

#ifdef __cplusplus
}
#endif
#endif
