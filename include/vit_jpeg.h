/*
 * vit_jpeg.h — JPEG input pipeline of libvit_hip.so ("image decode/normalise +
 * on-GPU prefetch").  The reference's forward takes an already-built input array
 * (ViT::forward(inputs, targets, B, T), /root/reference/train_vit.rs:188; encoder_forward :196)
 * and has no image decoder; this is the MI355X-side feed for real JPEG datasets.
 *
 * Hybrid decode: host threads do the serial part (markers, Huffman, DC prediction, restarts) and
 * hand each 8x8 block to the GPU as a 64-bit non-zero mask + its non-zero int16 coefficients; the
 * GPU dequantises, runs the IJG "islow" integer IDCT, upsamples chroma with libjpeg's "fancy"
 * triangle filter, converts YCbCr -> RGB with libjpeg's fixed-point tables, crops, flips and
 * resizes (bilinear, 1/256-pixel fixed point) to img x img, and — through the trainer —
 * normalises into the fp32 [B, 3, img, img] pixels.  Decoded pixels equal libjpeg-turbo's
 * (Pillow's decoder) bit for bit.  Supported: baseline / extended sequential Huffman DCT, 8-bit,
 * grayscale or YCbCr 4:4:4 / 4:2:2 / 4:2:0, restart intervals, multi-scan sequential files;
 * progressive, arithmetic-coded, lossless and CMYK files are rejected with an error.
 *
 * Dataset format ("packed JPEG records"): one file of concatenated JPEG files, an index of N+1
 * little-endian int64 byte offsets (record i = [off[i], off[i+1])), and N int32 labels.
 *
 * Shuffle and sharding are those of vit_loader (vit_data.h): epoch e's Fisher-Yates permutation
 * from splitmix64(seed + e); step k gives rank r the records perm[(k*world + r)*batch ..+batch).
 * Crop policy: augment = 0 -> the largest centred square (eval); augment = 1 -> random-resized
 * crop (area U[8 %, 100 %], log-aspect U[log 3/4, log 4/3], 10 tries, else the centred crop
 * clamped to that aspect range) and a horizontal flip with probability 1/2, drawn from
 * splitmix64(seed ^ splitmix64(0x6a70656755, e*N + record)) — reproducible per (epoch, record)
 * whatever the world size.
 */
#ifndef VIT_JPEG_H
#define VIT_JPEG_H

#include "vit_trainer.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vit_jpeg_loader vit_jpeg_loader_t;

/* Host only (no GPU): header probe.  kind 0 = grayscale, 1 = 4:4:4, 2 = 4:2:2, 3 = 4:2:0.
 * Returns 0, or non-zero with vit_last_error (unsupported or malformed file). */
int vit_jpeg_probe(const unsigned char* data, long long size, int* w, int* h, int* kind);
/* Host only: the quantised DCT coefficients of every block (int16, natural order, component-major,
 * each component's blocks row-major), for tests of the device half.  info (nullable, 208 ints):
 * w, h, kind, nc, then per component (3 slots) blocks wide, blocks high, valid width, valid
 * height, then 3 x 64 quantisation values (natural order).  coef may be NULL (info only). */
int vit_jpeg_coefficients(const unsigned char* data, long long size, short* coef, long long cap_blocks,
                          int* info);

/* threads = host entropy-decode threads; depth = ring slots (>= 2) decoded ahead by a background
 * producer.  Returns NULL on error (vit_last_error). */
vit_jpeg_loader_t* vit_jpeg_loader_open(const char* jpeg_path, const char* index_path, const char* labels_path,
                                        int batch, unsigned long long seed, int rank, int world, int shuffle,
                                        int augment, int depth, int threads);
long long vit_jpeg_loader_num_records(const vit_jpeg_loader_t* l);
int vit_jpeg_loader_steps_per_epoch(const vit_jpeg_loader_t* l);
/* Blocks until the next batch is entropy-decoded and makes it current.  labels -> [batch] int32
 * (valid until the next call); epoch / step nullable.  Non-zero if any record failed to decode. */
int vit_jpeg_loader_next(vit_jpeg_loader_t* l, const int** labels, long long* epoch, int* step);
/* The current batch's crop boxes: [batch][5] = x0, y0, width, height, flip. */
int vit_jpeg_loader_boxes(const vit_jpeg_loader_t* l, int* boxes);
/* GPU half on the context stream: the current batch -> dev_out [batch][img][img][3] uint8 (device
 * memory, HWC RGB).  Returns once the upload has read the host batch. */
int vit_jpeg_loader_decode_u8(vit_jpeg_loader_t* l, unsigned char* dev_out, int img);
/* Feed the trainer: the loader's current batch -> the trainer's normalised fp32 pixels and labels
 * (as vit_trainer_set_batch_u8: pixel = (u8 / 255 - mean[c]) / std[c]); decode on the trainer's
 * copy stream, ordered before the next forward. */
int vit_trainer_set_batch_jpeg(vit_trainer_t* t, vit_jpeg_loader_t* l, const float* mean3, const float* std3);
void vit_jpeg_loader_close(vit_jpeg_loader_t* l);

#ifdef __cplusplus
}
#endif
#endif
