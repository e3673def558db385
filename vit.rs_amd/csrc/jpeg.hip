// jpeg.hip — the device half of the hybrid JPEG decoder and the JPEG record loader
// (include/vit_jpeg.h, SURVEY.md §8f-3: real images for ViT::forward's input, train_vit.rs:188,
// encoder call :196).
//
// Host (jpeg_host.cpp, `threads` worker threads): markers + Huffman -> sparse quantised blocks.
// Device, two kernels per batch on one stream:
//   idct_k          one thread per 8x8 block: scatter the non-zero coefficients (zig-zag -> natural,
//                   x quantiser) into
//                   a column-interleaved LDS image, jpeg_idct_islow's two 1-D passes in int32,
//                   8 x 8 B row stores into the component plane (uint8, stride bw*8)
//   color_resize_k  one thread per output pixel of [n][img][img][3] uint8: the 2x2 source pixels
//                   of the bilinear tap (fixed point, 1/256 pixel), each one's chroma upsampled by
//                   the libjpeg "fancy" filter at that position and converted YCbCr -> RGB with the
//                   libjpeg fixed-point tables; crop box and horizontal flip from the descriptor
// The normalise into the trainer's fp32 [B][3][img][img] pixels is the uint8 path's kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <mutex>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../../include/vit_jpeg.h"
#include "jpeg_internal.h"

namespace vit {
void set_error(const char* fmt, ...);
bool has_error();
hipStream_t stream();
namespace jpg {

// one image of a batch as the kernels see it
struct ImgDesc {
    int w, h, kind, nc;
    int bw[MAXC], bh[MAXC], cw[MAXC], ch[MAXC];
    int nblk;            // blocks of the image (all components)
    int blk0[MAXC];      // first block of each component, batch-global
    long long pl[MAXC];  // byte offset of each component plane in the plane buffer (stride bw*8)
    int box[4];          // crop box in source pixels: x0, y0, width, height
    int flip, pad;
    uint16_t qt[MAXC][64];
};

// ------------------------------------------------------------------------------ islow IDCT
// jpeg_idct_islow (IJG libjpeg 6b jidctint.c, as libjpeg-turbo): CONST_BITS 13, PASS1_BITS 2
constexpr int CB = 13, P1 = 2;
constexpr int F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
              F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

// one 1-D pass over in[0..7] (stride 1) -> out[0..7], descaled by `sh`
__device__ __forceinline__ void idct8(const int (&in)[8], int (&out)[8], int sh) {
    int z2 = in[2], z3 = in[6];
    int z1 = (z2 + z3) * F0541;
    const int t2 = z1 + z3 * (-F1847);
    const int t3 = z1 + z2 * F0765;
    z2 = in[0];
    z3 = in[4];
    const int t0 = (z2 + z3) << CB;
    const int t1 = (z2 - z3) << CB;
    const int t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    int o0 = in[7], o1 = in[5], o2 = in[3], o3 = in[1];
    z1 = o0 + o3;
    z2 = o1 + o2;
    z3 = o0 + o2;
    int z4 = o1 + o3;
    const int z5 = (z3 + z4) * F1175;
    o0 *= F0298;
    o1 *= F2053;
    o2 *= F3072;
    o3 *= F1501;
    z1 *= -F0899;
    z2 *= -F2562;
    z3 *= -F1961;
    z4 *= -F0390;
    z3 += z5;
    z4 += z5;
    o0 += z1 + z3;
    o1 += z2 + z4;
    o2 += z2 + z3;
    o3 += z1 + z4;
    out[0] = descale(t10 + o3, sh);
    out[7] = descale(t10 - o3, sh);
    out[1] = descale(t11 + o2, sh);
    out[6] = descale(t11 - o2, sh);
    out[2] = descale(t12 + o1, sh);
    out[5] = descale(t12 - o1, sh);
    out[3] = descale(t13 + o0, sh);
    out[4] = descale(t13 - o0, sh);
}
// libjpeg's post-IDCT range limit: table[x & 1023] of (x + 128) clamped, with its wrap-around
__device__ __forceinline__ uint32_t range_limit(int x) {
    const int v = x & 1023;
    return v < 128 ? (uint32_t)(v + 128) : v < 512 ? 255u : v < 896 ? 0u : (uint32_t)(v - 896);
}

// zig-zag position -> natural index (the host emits each block's non-zero coefficients in zig-zag
// order, as the entropy decoder produces them)
__constant__ uint8_t kZigD[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                  35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                  58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

constexpr int IDCT_T = 64;  // threads (= blocks) per workgroup
__global__ __launch_bounds__(IDCT_T) void idct_k(uint8_t* __restrict__ planes, const ImgDesc* __restrict__ desc,
                                                 const uint64_t* __restrict__ masks,
                                                 const uint32_t* __restrict__ voff,
                                                 const int16_t* __restrict__ vals) {
    __shared__ int img[64 * IDCT_T];  // coefficient k of this workgroup's block t at [k][t]
    const ImgDesc& d = desc[blockIdx.y];
    const int t = threadIdx.x;
    const int b = blockIdx.x * IDCT_T + t;  // block within the image
    if (b >= d.nblk) return;
    int c = 0;
    while (c + 1 < d.nc && b >= d.blk0[c + 1] - d.blk0[0]) c++;
    const int lb = b - (d.blk0[c] - d.blk0[0]);
    const int gb = d.blk0[c] + lb;
#pragma unroll
    for (int k = 0; k < 64; k++) img[k * IDCT_T + t] = 0;
    uint64_t m = masks[gb];
    const int16_t* v = vals + voff[gb];
    const uint16_t* q = d.qt[c];
    while (m) {
        const int k = kZigD[__builtin_ctzll(m)];
        img[k * IDCT_T + t] = (int)*v++ * (int)q[k];
        m &= m - 1;
    }
    int ws[64];
#pragma unroll
    for (int col = 0; col < 8; col++) {  // pass 1: columns
        int in[8], out[8];
#pragma unroll
        for (int r = 0; r < 8; r++) in[r] = img[(r * 8 + col) * IDCT_T + t];
        idct8(in, out, CB - P1);
#pragma unroll
        for (int r = 0; r < 8; r++) ws[r * 8 + col] = out[r];
    }
    const int bx = lb % d.bw[c], by = lb / d.bw[c];
    const long long stride = (long long)d.bw[c] * 8;
    uint8_t* dst = planes + d.pl[c] + (long long)by * 8 * stride + bx * 8;
#pragma unroll
    for (int r = 0; r < 8; r++) {  // pass 2: rows, descale by CB + P1 + 3, range limit
        int in[8], out[8];
#pragma unroll
        for (int k = 0; k < 8; k++) in[k] = ws[r * 8 + k];
        idct8(in, out, CB + P1 + 3);
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            lo |= range_limit(out[k]) << (8 * k);
            hi |= range_limit(out[4 + k]) << (8 * k);
        }
        *reinterpret_cast<uint2*>(dst + r * stride) = make_uint2(lo, hi);
    }
}

// ------------------------------------------------------------------------------ colour + resize
// libjpeg jdcolor.c fixed point (SCALEBITS 16): FIX(x) = (int)(x * 65536 + 0.5)
constexpr int FIX_R = 91881, FIX_B = 116130, FIX_GR = 46802, FIX_GB = 22554;

__device__ __forceinline__ int clamp255(int x) { return x < 0 ? 0 : (x > 255 ? 255 : x); }

// the upsampled chroma sample of component plane p at full-resolution position (x, y)
__device__ __forceinline__ int chroma_at(const uint8_t* __restrict__ p, long long stride, int kind, int cwd, int chd,
                                         int x, int y) {
    if (kind == YCC444) return p[(long long)y * stride + x];
    const int c = x >> 1;
    if (kind == YCC422) {
        const uint8_t* row = p + (long long)y * stride;
        if (cwd <= 2) return row[c];  // libjpeg: fancy upsampling needs > 2 samples
        if ((x & 1) == 0) return c == 0 ? row[0] : (3 * row[c] + row[c - 1] + 1) >> 2;
        return c == cwd - 1 ? row[c] : (3 * row[c] + row[c + 1] + 2) >> 2;
    }
    // h2v2: vertical neighbour = the row above for even output rows, below for odd (edges replicate)
    const int r = y >> 1;
    if (cwd <= 2) return p[(long long)r * stride + c];
    const int rn = (y & 1) ? min(r + 1, chd - 1) : max(r - 1, 0);
    const uint8_t* r0 = p + (long long)r * stride;
    const uint8_t* r1 = p + (long long)rn * stride;
    auto cs = [&](int cc) { return 3 * (int)r0[cc] + (int)r1[cc]; };
    if ((x & 1) == 0) return c == 0 ? (4 * cs(0) + 8) >> 4 : (3 * cs(c) + cs(c - 1) + 8) >> 4;
    return c == cwd - 1 ? (4 * cs(c) + 7) >> 4 : (3 * cs(c) + cs(c + 1) + 7) >> 4;
}

__device__ __forceinline__ void rgb_at(const uint8_t* __restrict__ planes, const ImgDesc& d, int x, int y, int (&rgb)[3]) {
    const int Y = planes[d.pl[0] + (long long)y * d.bw[0] * 8 + x];
    if (d.kind == GRAY) {
        rgb[0] = rgb[1] = rgb[2] = Y;
        return;
    }
    const int cb = chroma_at(planes + d.pl[1], (long long)d.bw[1] * 8, d.kind, d.cw[1], d.ch[1], x, y) - 128;
    const int cr = chroma_at(planes + d.pl[2], (long long)d.bw[2] * 8, d.kind, d.cw[2], d.ch[2], x, y) - 128;
    rgb[0] = clamp255(Y + ((FIX_R * cr + 32768) >> 16));
    rgb[1] = clamp255(Y + ((-FIX_GB * cb + 32768 - FIX_GR * cr) >> 16));
    rgb[2] = clamp255(Y + ((FIX_B * cb + 32768) >> 16));
}

// bilinear tap of output coordinate o (of n) over box [b0, b0 + bl) of a len-sample axis, in
// 1/256 pixel: s = (o + 1/2) * bl / n - 1/2 + b0 (floor), taps clamped to the axis
__device__ __forceinline__ void tap(int o, int n, int b0, int bl, int len, int& i0, int& i1, int& f) {
    const long long s = (long long)(2 * o + 1) * bl * 128 / n - 128 + 256LL * b0;
    const int i = (int)(s >> 8);
    f = (int)(s & 255);
    i0 = min(max(i, 0), len - 1);
    i1 = min(max(i + 1, 0), len - 1);
}

__global__ __launch_bounds__(256) void color_resize_k(uint8_t* __restrict__ out, int img,
                                                      const uint8_t* __restrict__ planes,
                                                      const ImgDesc* __restrict__ desc) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= img * img) return;
    const ImgDesc& d = desc[blockIdx.y];
    const int oy = p / img, ox0 = p - oy * img;
    const int ox = d.flip ? img - 1 - ox0 : ox0;
    int x0, x1, fx, y0, y1, fy;
    tap(ox, img, d.box[0], d.box[2], d.w, x0, x1, fx);
    tap(oy, img, d.box[1], d.box[3], d.h, y0, y1, fy);
    int a[3], b[3], c[3], e[3];
    rgb_at(planes, d, x0, y0, a);
    rgb_at(planes, d, x1, y0, b);
    rgb_at(planes, d, x0, y1, c);
    rgb_at(planes, d, x1, y1, e);
    const int w00 = (256 - fx) * (256 - fy), w01 = fx * (256 - fy), w10 = (256 - fx) * fy, w11 = fx * fy;
    uint8_t* o = out + ((long long)blockIdx.y * img * img + p) * 3;
#pragma unroll
    for (int k = 0; k < 3; k++) o[k] = (uint8_t)((a[k] * w00 + b[k] * w01 + c[k] * w10 + e[k] * w11 + 32768) >> 16);
}

// ------------------------------------------------------------------------------ host batch
struct ImgOut {  // one image's host decode
    Frame f;
    Sparse sp;
    std::string err;
    bool ok = false;
};

template <typename T>
static T* align_up(char* base, size_t& off) {
    off = (off + 255) & ~(size_t)255;
    T* p = reinterpret_cast<T*>(base + off);
    return p;
}

// a batch ready for the device: descriptors + masks + value offsets + values in one pinned block
struct HostBatch {
    char* buf = nullptr;
    size_t cap = 0, used = 0;
    size_t o_desc = 0, o_mask = 0, o_voff = 0, o_vals = 0;
    int n = 0;
    long long nblk = 0, plane_bytes = 0;
    int max_blk = 0;
    std::vector<int> labels;
    std::vector<int> boxes;  // [n][5]
    std::vector<long long> img_bb, img_vb;  // first block / value of each image
    long long epoch = 0;
    int step = 0;
    int state = 0;  // 0 free, 1 ready, 2 handed out
    std::string err;

    bool pinned = false;
    void release() {
        if (buf) {
            if (pinned) (void)hipHostFree(buf);
            else free(buf);
        }
        buf = nullptr;
        cap = 0;
    }
    // page-locked when a GPU runtime is there (asynchronous DMA), else plain host memory
    bool reserve(size_t bytes) {
        if (bytes <= cap) return true;
        release();
        const size_t want = bytes + bytes / 4;
        pinned = hipHostMalloc((void**)&buf, want, hipHostMallocDefault) == hipSuccess;
        if (!pinned) {
            (void)hipGetLastError();
            buf = (char*)malloc(want);
        }
        if (!buf) return false;
        cap = want;
        return true;
    }
    ~HostBatch() { release(); }
};

// lay out hb for the decoded images: sizes, descriptors with their crop boxes, each image's
// first block / value (the sparse stream itself: copy_image)
static bool assemble(HostBatch& hb, std::vector<ImgOut>& outs, int n, const int* boxes) {
    long long nblk = 0, nval = 0, plane = 0;
    int max_blk = 0;
    for (int i = 0; i < n; i++) {
        if (!outs[i].ok) {
            hb.err = "image " + std::to_string(i) + ": " + outs[i].err;
            return false;
        }
        const long long b = outs[i].f.blocks();
        nblk += b;
        nval += outs[i].sp.nvals;
        max_blk = std::max<int>(max_blk, (int)b);
        for (int c = 0; c < outs[i].f.nc; c++) plane += (long long)outs[i].f.bw[c] * outs[i].f.bh[c] * 64;
    }
    if (nblk >= (1LL << 31) || nval >= (1LL << 32)) {
        hb.err = "batch too large";
        return false;
    }
    size_t off = 0;
    hb.o_desc = off;
    off += sizeof(ImgDesc) * (size_t)n;
    off = (off + 255) & ~(size_t)255;
    hb.o_mask = off;
    off += 8 * (size_t)nblk;
    off = (off + 255) & ~(size_t)255;
    hb.o_voff = off;
    off += 4 * (size_t)nblk;
    off = (off + 255) & ~(size_t)255;
    hb.o_vals = off;
    off += 2 * (size_t)std::max<long long>(nval, 1);
    if (!hb.reserve(off)) {
        hb.err = "pinned host allocation failed";
        return false;
    }
    hb.used = off;
    hb.n = n;
    hb.nblk = nblk;
    hb.plane_bytes = plane;
    hb.max_blk = max_blk;
    ImgDesc* desc = reinterpret_cast<ImgDesc*>(hb.buf + hb.o_desc);
    hb.img_bb.resize((size_t)n);
    hb.img_vb.resize((size_t)n);
    long long bb = 0, vb = 0, pb = 0;
    for (int i = 0; i < n; i++) {
        const Frame& f = outs[i].f;
        ImgDesc& d = desc[i];
        memset(&d, 0, sizeof(d));
        d.w = f.w; d.h = f.h; d.kind = f.kind; d.nc = f.nc;
        d.nblk = (int)f.blocks();
        long long cb = bb;
        for (int c = 0; c < f.nc; c++) {
            d.bw[c] = f.bw[c]; d.bh[c] = f.bh[c]; d.cw[c] = f.cw[c]; d.ch[c] = f.ch[c];
            d.blk0[c] = (int)cb;
            cb += (long long)f.bw[c] * f.bh[c];
            d.pl[c] = pb;
            pb += (long long)f.bw[c] * f.bh[c] * 64;
            memcpy(d.qt[c], f.qt[c], sizeof(d.qt[c]));
        }
        for (int k = 0; k < 4; k++) d.box[k] = boxes[5 * i + k];
        d.flip = boxes[5 * i + 4];
        hb.img_bb[(size_t)i] = bb;
        hb.img_vb[(size_t)i] = vb;
        bb += d.nblk;
        vb += outs[i].sp.nvals;
    }
    return true;
}
// the sparse stream of image i into its place (after assemble; independent per image: run on the
// worker pool)
static void copy_image(HostBatch& hb, const std::vector<ImgOut>& outs, int i) {
    uint64_t* masks = reinterpret_cast<uint64_t*>(hb.buf + hb.o_mask);
    uint32_t* voff = reinterpret_cast<uint32_t*>(hb.buf + hb.o_voff);
    int16_t* vals = reinterpret_cast<int16_t*>(hb.buf + hb.o_vals);
    const long long bb = hb.img_bb[(size_t)i], vb = hb.img_vb[(size_t)i];
    const Sparse& sp = outs[(size_t)i].sp;
    const long long nb = outs[(size_t)i].f.blocks();
    memcpy(masks + bb, sp.masks.data(), 8 * (size_t)nb);
    memcpy(vals + vb, sp.vals.data(), 2 * (size_t)sp.nvals);
    for (long long k = 0; k < nb; k++) voff[bb + k] = (uint32_t)(vb + sp.voff[(size_t)k]);
}

// decode one JPEG into out (host)
static void decode_one(const uint8_t* data, size_t size, ImgOut& out) {
    out.err.clear();
    out.ok = decode_sparse(data, size, out.f, out.sp, out.err);
}

// crop policy: 0 = the largest centred square; 1 = random-resized crop (area 8-100 %, aspect
// 3/4 - 4/3, 10 tries, then the centred crop clamped to that aspect range) + horizontal flip p=1/2
static uint64_t sm64(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static void crop_box(int W, int H, int augment, uint64_t seed, int* box) {
    if (!augment) {
        const int s = std::min(W, H);
        box[0] = (W - s) / 2; box[1] = (H - s) / 2; box[2] = s; box[3] = s; box[4] = 0;
        return;
    }
    uint64_t ctr = 0;
    auto u01 = [&]() { return (double)(sm64(seed, ctr++) >> 11) * (1.0 / 9007199254740992.0); };
    const double area = (double)W * H;
    for (int t = 0; t < 10; t++) {
        const double ta = area * (0.08 + 0.92 * u01());
        const double lr = std::log(3.0 / 4.0) + (std::log(4.0 / 3.0) - std::log(3.0 / 4.0)) * u01();
        const double ar = std::exp(lr);
        const int cw = (int)std::lround(std::sqrt(ta * ar)), ch = (int)std::lround(std::sqrt(ta / ar));
        if (cw > 0 && ch > 0 && cw <= W && ch <= H) {
            box[0] = (int)(sm64(seed, ctr++) % (uint64_t)(W - cw + 1));
            box[1] = (int)(sm64(seed, ctr++) % (uint64_t)(H - ch + 1));
            box[2] = cw; box[3] = ch;
            box[4] = (int)(sm64(seed, ctr++) & 1);
            return;
        }
    }
    const double r = (double)W / H;
    int cw = W, ch = H;
    if (r < 0.75) ch = std::max(1, (int)std::lround(W / 0.75));
    else if (r > 4.0 / 3.0) cw = std::max(1, (int)std::lround(H * 4.0 / 3.0));
    cw = std::min(cw, W);
    ch = std::min(ch, H);
    box[0] = (W - cw) / 2; box[1] = (H - ch) / 2; box[2] = cw; box[3] = ch;
    box[4] = (int)(sm64(seed, ctr++) & 1);
}

// device buffers of one consumer + the kernels
struct DeviceSide {
    char* dbuf = nullptr;
    size_t dcap = 0;
    uint8_t* planes = nullptr;
    size_t pcap = 0;
    hipEvent_t done = nullptr;      // the kernels of the previous batch (buffer reuse across streams)
    hipEvent_t uploaded = nullptr;  // the upload of the current batch (pinned host block reusable)

    bool grow(void** p, size_t& cap, size_t need) {
        if (need <= cap) return true;
        if (*p) {
            // only the previous batch's kernels read the old buffer: wait for them, not the device
            (void)hipEventSynchronize(done);
            (void)hipFree(*p);
        }
        *p = nullptr;
        cap = 0;
        const size_t want = need + need / 4;
        if (hipMalloc(p, want) != hipSuccess) {
            *p = nullptr;
            return false;
        }
        cap = want;
        return true;
    }
    // enqueue the upload and both kernels of hb on st; out [n][img][img][3] uint8 (device)
    bool run(const HostBatch& hb, uint8_t* out, int img, hipStream_t st) {
        if ((!done && hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) ||
            (!uploaded && hipEventCreateWithFlags(&uploaded, hipEventDisableTiming) != hipSuccess)) {
            set_error("jpeg: event creation failed");
            return false;
        }
        if (!grow((void**)&dbuf, dcap, hb.used) || !grow((void**)&planes, pcap, (size_t)std::max<long long>(hb.plane_bytes, 1))) {
            set_error("jpeg: device allocation failed");
            return false;
        }
        if (hipStreamWaitEvent(st, done, 0) != hipSuccess ||
            hipMemcpyAsync(dbuf, hb.buf, hb.used, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipEventRecord(uploaded, st) != hipSuccess) {
            set_error("jpeg: upload failed");
            return false;
        }
        const ImgDesc* desc = reinterpret_cast<const ImgDesc*>(dbuf + hb.o_desc);
        idct_k<<<dim3((hb.max_blk + IDCT_T - 1) / IDCT_T, hb.n), IDCT_T, 0, st>>>(
            planes, desc, reinterpret_cast<const uint64_t*>(dbuf + hb.o_mask),
            reinterpret_cast<const uint32_t*>(dbuf + hb.o_voff), reinterpret_cast<const int16_t*>(dbuf + hb.o_vals));
        color_resize_k<<<dim3((img * img + 255) / 256, hb.n), 256, 0, st>>>(out, img, planes, desc);
        if (hipGetLastError() != hipSuccess || hipEventRecord(done, st) != hipSuccess) {
            set_error("jpeg: kernel launch failed");
            return false;
        }
        // the pinned batch may be refilled once the upload has read it (the kernels keep running)
        (void)hipEventSynchronize(uploaded);
        return true;
    }
    ~DeviceSide() {
        if (done) (void)hipEventDestroy(done);
        if (uploaded) (void)hipEventDestroy(uploaded);
        if (dbuf) (void)hipFree(dbuf);
        if (planes) (void)hipFree(planes);
    }
};

struct Mapped {
    void* p = MAP_FAILED;
    size_t bytes = 0;
    bool open(const char* path) {
        int fd = ::open(path, O_RDONLY);
        if (fd < 0) return false;
        struct stat st;
        if (fstat(fd, &st) != 0 || st.st_size <= 0) {
            ::close(fd);
            return false;
        }
        bytes = (size_t)st.st_size;
        p = mmap(nullptr, bytes, PROT_READ, MAP_PRIVATE, fd, 0);
        ::close(fd);
        return p != MAP_FAILED;
    }
    ~Mapped() {
        if (p != MAP_FAILED) munmap(p, bytes);
    }
};

}  // namespace jpg
}  // namespace vit

using namespace vit::jpg;
using vit::set_error;

// ------------------------------------------------------------------------------ record loader
struct vit_jpeg_loader {
    Mapped data, index, labels;
    const long long* offs = nullptr;
    long long N = 0;
    int B = 0, rank = 0, world = 1, shuffle = 1, augment = 0, steps = 0, nthreads = 1;
    uint64_t seed = 0;
    std::vector<HostBatch> slots;
    std::mutex mu;
    std::condition_variable cv;
    bool stop = false;
    std::thread producer;
    size_t next_fill = 0, next_take = 0;
    long long out_slot = -1;
    std::vector<long long> perm;
    long long perm_epoch = -1;
    // worker pool for the entropy decode of one batch
    std::vector<std::thread> pool;
    std::mutex pmu;
    std::condition_variable pcv, pdone;
    long long job_gen = 0;
    std::atomic<int> job_next{0};
    std::atomic<bool> quit{false};
    int job_left = 0;
    const long long* job_recs = nullptr;
    HostBatch* job_hb = nullptr;
    bool job_copy = false;
    std::vector<ImgOut> outs;
    DeviceSide dev;

    void make_perm(long long epoch) {
        perm.resize((size_t)N);
        for (long long i = 0; i < N; i++) perm[(size_t)i] = i;
        if (shuffle) {
            const uint64_t s = seed + (uint64_t)epoch;
            for (long long i = N - 1; i >= 1; i--) {
                const uint64_t r = sm64(s, (uint64_t)(N - 1 - i));
                std::swap(perm[(size_t)i], perm[(size_t)(r % (uint64_t)(i + 1))]);
            }
        }
        perm_epoch = epoch;
    }
    void worker() {
        long long seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(pmu);
                pcv.wait(lk, [&] { return stop || job_gen != seen; });
                // a job published before the stop still runs to its end (quit makes it cheap), so
                // the producer waiting in pool_job always sees job_left reach 0
                if (job_gen == seen) return;
                seen = job_gen;
            }
            int done_here = 0;
            for (int i; (i = job_next.fetch_add(1)) < B;) {  // every index is counted, even on stop
                if (quit.load(std::memory_order_relaxed)) {
                    outs[(size_t)i].ok = false;
                    outs[(size_t)i].err = "loader closed";
                } else if (job_copy) {
                    copy_image(*job_hb, outs, i);
                } else {
                    const long long r = job_recs[i];
                    const uint8_t* base = (const uint8_t*)data.p;
                    decode_one(base + offs[r], (size_t)(offs[r + 1] - offs[r]), outs[(size_t)i]);
                }
                done_here++;
            }
            {
                std::lock_guard<std::mutex> lk(pmu);
                job_left -= done_here;
            }
            pdone.notify_all();
        }
    }
    // one job over the batch's B images on the pool: decode (recs) or copy into hb
    bool pool_job(const long long* recs, HostBatch* hb) {
        {
            std::lock_guard<std::mutex> lk(pmu);
            if (stop) return false;  // the workers may have left: publish nothing after a stop
            job_recs = recs;
            job_hb = hb;
            job_copy = hb != nullptr;
            job_next = 0;
            job_left = B;
            job_gen++;
        }
        pcv.notify_all();
        // the job's record list and outputs stay alive until every worker has left them
        std::unique_lock<std::mutex> lk(pmu);
        pdone.wait(lk, [&] { return job_left == 0; });
        return !quit.load();
    }
    void fill(HostBatch& hb, long long seq) {
        const long long epoch = seq / steps;
        const int step = (int)(seq % steps);
        if (epoch != perm_epoch) make_perm(epoch);
        const long long base = ((long long)step * world + rank) * B;
        std::vector<long long> recs((size_t)B);
        for (int b = 0; b < B; b++) recs[(size_t)b] = perm[(size_t)(base + b)];
        hb.err.clear();
        if (!pool_job(recs.data(), nullptr)) return;
        hb.labels.resize((size_t)B);
        hb.boxes.resize((size_t)B * 5);
        const int* lab = (const int*)labels.p;
        for (int b = 0; b < B; b++) {
            const long long r = recs[(size_t)b];
            hb.labels[(size_t)b] = lab[r];
            const ImgOut& o = outs[(size_t)b];
            if (o.ok)
                crop_box(o.f.w, o.f.h, augment, seed ^ sm64(0x6a70656755ULL, (uint64_t)(epoch * N + r)), &hb.boxes[(size_t)b * 5]);
        }
        if (assemble(hb, outs, B, hb.boxes.data())) pool_job(nullptr, &hb);
        hb.epoch = epoch;
        hb.step = step;
    }
    void run() {
        long long seq = 0;
        for (;;) {
            HostBatch* hb;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || slots[next_fill].state == 0; });
                if (stop) return;
                hb = &slots[next_fill];
            }
            fill(*hb, seq++);
            {
                std::lock_guard<std::mutex> lk(mu);
                hb->state = 1;
                next_fill = (next_fill + 1) % slots.size();
            }
            cv.notify_all();
        }
    }
    HostBatch* current() { return out_slot >= 0 ? &slots[(size_t)out_slot] : nullptr; }
    void shutdown() {
        quit = true;
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        {
            std::lock_guard<std::mutex> lk(pmu);
            stop = true;
        }
        cv.notify_all();
        pcv.notify_all();
        pdone.notify_all();
        if (producer.joinable()) producer.join();
        for (auto& t : pool)
            if (t.joinable()) t.join();
    }
};

namespace vit {
// trainer.hip: decode the loader's current batch into device uint8 [B][img][img][3] on st
// (expect_n >= 0: the destination holds exactly expect_n images; a loader batch of another size is
// rejected before anything is written or its labels read)
bool jpeg_loader_decode_to(vit_jpeg_loader_t* l, uint8_t* out, int img, hipStream_t st, const int** labels,
                           int expect_n) {
    HostBatch* hb = l->current();
    if (!hb) {
        set_error("jpeg loader: no current batch (call vit_jpeg_loader_next first)");
        return false;
    }
    if (expect_n >= 0 && hb->n != expect_n) {
        set_error("jpeg loader: batch of %d images, the trainer's batch is %d", hb->n, expect_n);
        return false;
    }
    if (!hb->err.empty()) {
        set_error("jpeg loader: %s", hb->err.c_str());
        return false;
    }
    if (labels) *labels = hb->labels.data();
    return l->dev.run(*hb, out, img, st);
}
}  // namespace vit

extern "C" {

int vit_jpeg_probe(const unsigned char* data, long long size, int* w, int* h, int* kind) {
    if (!data || size <= 0) {
        set_error("vit_jpeg_probe: empty input");
        return 1;
    }
    Frame f;
    std::string err;
    if (!parse_header(data, (size_t)size, f, err)) {
        set_error("vit_jpeg_probe: %s", err.c_str());
        return 1;
    }
    if (w) *w = f.w;
    if (h) *h = f.h;
    if (kind) *kind = f.kind;
    return 0;
}

int vit_jpeg_coefficients(const unsigned char* data, long long size, short* coef, long long cap_blocks,
                          int* info) {
    Frame f;
    std::string err;
    std::vector<int16_t> c;
    if (!data || size <= 0 || !decode_coefficients(data, (size_t)size, f, c, err)) {
        set_error("vit_jpeg_coefficients: %s", err.empty() ? "empty input" : err.c_str());
        return 1;
    }
    if (info) {  // w, h, kind, nc, then per component bw, bh, cw, ch, then 3 x 64 quant values
        int* o = info;
        *o++ = f.w; *o++ = f.h; *o++ = f.kind; *o++ = f.nc;
        for (int k = 0; k < MAXC; k++) {
            *o++ = k < f.nc ? f.bw[k] : 0; *o++ = k < f.nc ? f.bh[k] : 0;
            *o++ = k < f.nc ? f.cw[k] : 0; *o++ = k < f.nc ? f.ch[k] : 0;
        }
        for (int k = 0; k < MAXC; k++)
            for (int j = 0; j < 64; j++) *o++ = k < f.nc ? f.qt[k][j] : 0;
    }
    if (coef) {
        if (f.blocks() > cap_blocks) {
            set_error("vit_jpeg_coefficients: %lld blocks > capacity %lld", f.blocks(), cap_blocks);
            return 1;
        }
        memcpy(coef, c.data(), c.size() * sizeof(int16_t));
    }
    return 0;
}

vit_jpeg_loader_t* vit_jpeg_loader_open(const char* jpeg_path, const char* index_path, const char* labels_path,
                                        int batch, unsigned long long seed, int rank, int world, int shuffle,
                                        int augment, int depth, int threads) {
    if (!jpeg_path || !index_path || !labels_path || batch <= 0 || world < 1 || rank < 0 || rank >= world ||
        depth < 2 || threads < 1) {
        set_error("vit_jpeg_loader_open: bad arguments");
        return nullptr;
    }
    auto* l = new vit_jpeg_loader();
    if (!l->data.open(jpeg_path) || !l->index.open(index_path) || !l->labels.open(labels_path)) {
        set_error("vit_jpeg_loader_open: cannot map %s / %s / %s", jpeg_path, index_path, labels_path);
        delete l;
        return nullptr;
    }
    l->N = (long long)(l->labels.bytes / 4);
    l->offs = (const long long*)l->index.p;
    if (l->labels.bytes % 4 || l->index.bytes != 8 * (size_t)(l->N + 1)) {
        set_error("vit_jpeg_loader_open: index must hold N+1 int64 offsets for N int32 labels");
        delete l;
        return nullptr;
    }
    for (long long i = 0; i < l->N; i++)
        if (l->offs[i] < 0 || l->offs[i + 1] < l->offs[i] || (size_t)l->offs[i + 1] > l->data.bytes) {
            set_error("vit_jpeg_loader_open: offset %lld out of range", i);
            delete l;
            return nullptr;
        }
    l->B = batch;
    l->rank = rank;
    l->world = world;
    l->seed = seed;
    l->shuffle = shuffle != 0;
    l->augment = augment != 0;
    l->nthreads = threads;
    l->steps = (int)(l->N / ((long long)batch * world));
    if (l->steps < 1) {
        set_error("vit_jpeg_loader_open: %lld records < one global batch of %d x %d", l->N, batch, world);
        delete l;
        return nullptr;
    }
    l->slots = std::vector<HostBatch>((size_t)depth);
    l->outs.resize((size_t)batch);
    for (int t = 0; t < threads; t++) l->pool.emplace_back([l] { l->worker(); });
    l->producer = std::thread([l] { l->run(); });
    return l;
}

long long vit_jpeg_loader_num_records(const vit_jpeg_loader_t* l) { return l ? l->N : 0; }
int vit_jpeg_loader_steps_per_epoch(const vit_jpeg_loader_t* l) { return l ? l->steps : 0; }

int vit_jpeg_loader_next(vit_jpeg_loader_t* l, const int** labels, long long* epoch, int* step) {
    if (!l) {
        set_error("vit_jpeg_loader_next: null loader");
        return 1;
    }
    std::unique_lock<std::mutex> lk(l->mu);
    if (l->out_slot >= 0) {
        l->slots[(size_t)l->out_slot].state = 0;
        l->out_slot = -1;
        l->cv.notify_all();
    }
    l->cv.wait(lk, [&] { return l->slots[l->next_take].state == 1; });
    auto& s = l->slots[l->next_take];
    s.state = 2;
    l->out_slot = (long long)l->next_take;
    l->next_take = (l->next_take + 1) % l->slots.size();
    if (!s.err.empty()) {
        set_error("vit_jpeg_loader_next: %s", s.err.c_str());
        return 1;
    }
    if (labels) *labels = s.labels.data();
    if (epoch) *epoch = s.epoch;
    if (step) *step = s.step;
    return 0;
}

int vit_jpeg_loader_boxes(const vit_jpeg_loader_t* l, int* boxes) {
    if (!l || l->out_slot < 0 || !boxes) {
        set_error("vit_jpeg_loader_boxes: no current batch");
        return 1;
    }
    const HostBatch& s = l->slots[(size_t)l->out_slot];
    memcpy(boxes, s.boxes.data(), s.boxes.size() * sizeof(int));
    return 0;
}

int vit_jpeg_loader_decode_u8(vit_jpeg_loader_t* l, unsigned char* dev_out, int img) {
    if (!l || !dev_out || img <= 0) {
        set_error("vit_jpeg_loader_decode_u8: bad arguments");
        return 1;
    }
    return vit::jpeg_loader_decode_to(l, dev_out, img, vit::stream(), nullptr, -1) && !vit::has_error() ? 0 : 1;
}

void vit_jpeg_loader_close(vit_jpeg_loader_t* l) {
    if (!l) return;
    l->shutdown();
    delete l;
}

}  // extern "C"
