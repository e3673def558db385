/*
 * vit_data.h — input pipeline of libvit_hip.so.
 *
 * The reference's forward takes an already-built input array (ViT::forward(inputs, targets, B, T),
 * /root/reference/train_vit.rs:188; encoder_forward :196) and has no data loader.  This is the
 * MI355X-side feed for real images:
 *
 *   vit_loader_*   native record loader: a raw uint8 image file [N, img, img, 3] (HWC, RGB) and a
 *                  raw int32 label file [N], memory-mapped; a per-epoch seeded shuffle; the batch
 *                  of each data-parallel rank; batches assembled by a background thread into a
 *                  ring of (pinned) host buffers.
 *   vit_trainer_set_batch_u8
 *                  copies one uint8 batch to the device on a copy stream (double-buffered device
 *                  staging, overlapping the previous step's kernels) and normalises it on the
 *                  device into the trainer's fp32 [B, 3, img, img] pixels:
 *                      pixel[b][c][y][x] = (u8[b][y][x][c] / 255 - mean[c]) / std[c]
 *                  (fp32, each operation correctly rounded, in that order).
 *
 * Shuffle: epoch e uses the permutation of Fisher-Yates (i = N-1 .. 1, swap(i, r_i mod (i+1)))
 * with r_i = splitmix64 counter stream of seed + e at position N-1-i (the generator of the
 * package's synthetic data, vit.rs_amd/data.py); shuffle = 0 keeps file order.  Step k of an
 * epoch gives rank r the records perm[(k*world + r)*batch .. +batch); the last partial global
 * batch is dropped, so every rank sees the same number of steps and disjoint records.
 */
#ifndef VIT_DATA_H
#define VIT_DATA_H

#include "vit_trainer.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vit_loader vit_loader_t;

/* pinned = 1: ring buffers in page-locked memory (hipHostMalloc; asynchronous DMA);
 * 0: malloc (no HIP call at all — usable without a GPU).  depth = ring slots (>= 2).
 * Returns NULL on error (vit_last_error). */
vit_loader_t* vit_loader_open(const char* images_path, const char* labels_path, int img,
                              int batch, unsigned long long seed, int rank, int world, int shuffle,
                              int pinned, int depth);
long long vit_loader_num_records(const vit_loader_t* l);
int vit_loader_steps_per_epoch(const vit_loader_t* l);
/* Blocks until the next batch is assembled.  images -> [batch, img, img, 3] uint8, labels ->
 * [batch] int32, valid until the next vit_loader_next / vit_loader_close.  epoch / step
 * (nullable) identify the batch.  Returns 0, or non-zero on error. */
int vit_loader_next(vit_loader_t* l, const unsigned char** images, const int** labels,
                    long long* epoch, int* step);
void vit_loader_close(vit_loader_t* l);

/* host pointers; labels NULL = forward-only batch.  Returns once the host buffers have been read
 * (they may be reused immediately); the device work is ordered before the next forward. */
int vit_trainer_set_batch_u8(vit_trainer_t* t, const unsigned char* images, const int* labels,
                             const float* mean3, const float* std3);

#ifdef __cplusplus
}
#endif
#endif
