// attn_fused.h — fused bf16 MFMA attention (attention_forward / attention_backward,
// /root/reference/train_vit.rs:400-451, 559-601; attention.rs:1-57) for any head size HS in
// {32, 64, 80, 96, 128} and T up to what the LDS holds.  Fixes D1 (offsets by T), D2 (full
// normalisation), D3 (non-causal).  Instantiated per head size by attn_h*.hip (parallel builds).
//
// One workgroup per (b,h) holds the head's operands in LDS; scores never touch HBM.
//   forward : per 16-query tile, S^T = K.Q^T with v_mfma_f32_16x16x32_bf16 so each lane owns one
//             query column (lane&15) -> row max/sum need only two cross-lane shuffles; the fp32
//             score accumulators convert in place into the B operand of O^T = V^T.P^T (k = 4g+j |
//             16+4g+j on both operands), V read with ds_read_b64_tr_b16.  Writes O (bf16) and lse
//             (log2 domain) per query.
//   backward: two roles of one launch (kv: 32 keys per wave, dK^T, dV^T; q: 32 queries per wave,
//             dQ^T), P recomputed from lse, dS = P (dP - delta) with delta = rowsum(dO*O), the
//             O(T^2) form of the reference's O(T^3) softmax Jacobian loop (train_vit.rs:583-589).
// Head dims: the score products run k-steps of 32 over the head dim; when HS % 32 == 16 (HS 80,
// 96 is a multiple of 32) the last k-step's upper half (d = HS .. HS+15) is zero IN REGISTERS on
// both operands, so the images need no padding columns and nothing past column HS is read.  The
// output products tile the head dim by 16 (HS/16 tiles).  Rows >= T of every image are zero;
// the padded length TP is a multiple of 32.
#pragma once
#include "ops_internal.h"

namespace vit {
namespace fa {

// diagnostic builds only (tools/bench_attn.py on a -DVIT_ATTN_DIAG=n library; outputs wrong):
// bit 0 = the persistent backward issues no global loads inside its item loop, bit 1 = no dQ / dK / dV stores
#ifndef VIT_ATTN_DIAG
#define VIT_ATTN_DIAG 0
#endif
// bit 2: per-wave s_memtime stamps of the forward and both backward forms (blocks < 8, 16 records of
// 16 stamps per wave) into attn_trace, read with vit_attn_trace_read_h<HS> (tools/attn_trace.py)
#if VIT_ATTN_DIAG & 4
static __device__ unsigned long long attn_trace[8 * 16 * 16 * 16];
#define ATTN_STAMP(k)                                                                                   \
    do {                                                                                                \
        if (blockIdx.x < 8 && it < 16 && lane == 0)                                                     \
            attn_trace[((blockIdx.x * 16 + it) * 16 + w) * 16 + (k)] = __builtin_amdgcn_s_memtime();   \
    } while (0)
#else
#define ATTN_STAMP(k) \
    do {              \
    } while (0)
#endif

constexpr float LOG2E = 1.4426950408889634f;

template <int HS>
struct Geo {
    static_assert(HS % 16 == 0 && HS >= 32 && HS <= 128, "head size");
    static constexpr int KS = (HS + 31) / 32;      // 32-deep k-steps over the head dim
    static constexpr bool HALF = (HS % 32) != 0;   // last k-step: upper 16 are zero padding
    static constexpr int DT = HS / 16;             // 16-wide output tiles of the head dim
    static constexpr int CH = HS / 8;              // 16-B chunks per image row
    // row-read image stride: (SK/2) = 4*odd (mod 64) dwords -> 16 rows x 2 lane groups of b64
    // reads cover 64 distinct banks (HS + 8 satisfies it for every supported HS)
    static constexpr int SK = HS + 8;
    // transposed-read-only image stride: (SV/2) = 8*odd (mod 64) dwords -> the 8 rows x 32 B of a
    // ds_read_b64_tr_b16 lane group hit distinct banks
    static constexpr int SV = HS == 32 ? 48 : HS == 64 ? 80 : HS == 80 ? 80 : HS == 96 ? 112 : 144;
};

// 8 bf16 of rows r0+i for k-step s (k = 32s + 4g + j | 32s + 16 + 4g + j - 4)
template <int HS>
__device__ __forceinline__ bf16x8_t frag_row(const bf16_t* img, int stride, int r0, int s, int lane) {
    const int i = lane & 15, g = lane >> 4;
    const bf16_t* p = img + (r0 + i) * stride + 32 * s + 4 * g;
    const bf16x4_t lo = *reinterpret_cast<const bf16x4_t*>(p);
    bf16x4_t hi = {};
    if (!(Geo<HS>::HALF && s == Geo<HS>::KS - 1)) hi = *reinterpret_cast<const bf16x4_t*>(p + 16);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// The same fragments as two ds_read_b64 each.  hipcc merges the four 8-byte reads of a row block
// (k offsets 0, 16, 32, 48 of the HS = 64 row) into two ds_read2_b64: 8 LDS cycles each with 32-bank
// groups of 16 lanes, where rows i and i + 8 of the HS + 8 stride collide (16 cycles) — against 2
// cycles for a ds_read_b64 (64 banks, conflict-free at that stride: MI355X_MICROARCH.md §LDS).
// `RowBases` holds one address per (k-step, half) with the offsets hidden from the compiler, so
// no two reads share a base and a constant offset.
template <int HS>
struct RowBases {
    static constexpr int N = 2 * Geo<HS>::KS;
    const char* b[N];
    __device__ __forceinline__ RowBases(const bf16_t* img, int stride, int lane) {
        const int i = lane & 15, g = lane >> 4;
        const char* p = reinterpret_cast<const char*>(img + i * stride + 4 * g);
#pragma unroll
        for (int k = 0; k < N; k++) {
            int off = 32 * k;  // k = 2 s + half
            if (k > 0) asm volatile("" : "+v"(off));
            b[k] = p + off;
        }
    }
    // rows r0 + i, k-step s
    __device__ __forceinline__ bf16x8_t frag(int r0, int stride, int s) const {
        const bf16x4_t lo = *reinterpret_cast<const bf16x4_t*>(b[2 * s] + r0 * stride * 2);
        bf16x4_t hi = {};
        if (!(Geo<HS>::HALF && s == Geo<HS>::KS - 1)) hi = *reinterpret_cast<const bf16x4_t*>(b[2 * s + 1] + r0 * stride * 2);
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
};
// the same fragment straight from a [T][ld] global operand (rows >= T -> 0)
template <int HS>
__device__ __forceinline__ bf16x8_t frag_glb(const bf16_t* base, long long ld, int row, int T, int s, int lane) {
    const int g = lane >> 4;
    bf16x4_t lo = {}, hi = {};
    if (row < T) {
        const bf16_t* p = base + (long long)row * ld + 32 * s + 4 * g;
        lo = *reinterpret_cast<const bf16x4_t*>(p);
        if (!(Geo<HS>::HALF && s == Geo<HS>::KS - 1)) hi = *reinterpret_cast<const bf16x4_t*>(p + 16);
    }
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// transposed: k = rows kb + (4g+j | 16+4g+j-4), column c0 + i
__device__ __forceinline__ bf16x8_t frag_tr(const bf16_t* img, int stride, int kb, int c0, int lane) {
    const int i = lane & 15, g = lane >> 4;
    const bf16_t* p = img + (kb + 4 * g + (i >> 2)) * stride + c0 + 4 * (i & 3);
    const bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4_t, p));
    const bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4_t, p + 16 * stride));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// two 16-row accumulator tiles (rows 4g+r) -> one 32-deep operand with the shared permutation
__device__ __forceinline__ bf16x8_t pack_acc(f32x4_t a, f32x4_t b) {
    bf16x8_t r;
    r[0] = (__bf16)a[0]; r[1] = (__bf16)a[1]; r[2] = (__bf16)a[2]; r[3] = (__bf16)a[3];
    r[4] = (__bf16)b[0]; r[5] = (__bf16)b[1]; r[6] = (__bf16)b[2]; r[7] = (__bf16)b[3];
    return r;
}
// v_exp_f32 (2^x, ~1 ulp; results below 2^-126 flush to 0, irrelevant for probabilities that
// are rounded to bf16); exp2f adds a denormal range-reduction sequence around it
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
// sum over the 16 lanes of a DPP row, valid in lane 15 of the row (row_shr 1, 2, 4, 8; lanes
// shifted in from outside the row read 0)
__device__ __forceinline__ float row_sum16(float v) {
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xF, 0xF, false));
    return v;
}
__device__ __forceinline__ f32x4_t mfma(bf16x8_t a, bf16x8_t b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// rows of HS bf16 (HS/8 x 16 B each, rows >= T zero-filled) of NOP operands into their LDS images.
// Every global load of the thread is issued before its first LDS store, so the whole staging is
// one memory round trip.
template <int HS, int TP, int NTHR, int NOP>
__device__ __forceinline__ void load_images(bf16_t* const (&img)[NOP], const int (&stride)[NOP],
                                            const bf16_t* const (&src)[NOP],
                                            const long long (&ld)[NOP], int T) {
    constexpr int CH = Geo<HS>::CH;
    constexpr int PER = (TP * CH + NTHR - 1) / NTHR;
    uint4 v[NOP][PER];
#pragma unroll
    for (int o = 0; o < NOP; o++)
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int idx = j * NTHR + (int)threadIdx.x, t = idx / CH, c = idx - t * CH;
            v[o][j] = make_uint4(0, 0, 0, 0);
            if (idx < TP * CH && t < T) v[o][j] = *reinterpret_cast<const uint4*>(src[o] + (long long)t * ld[o] + c * 8);
        }
#pragma unroll
    for (int o = 0; o < NOP; o++)
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int idx = j * NTHR + (int)threadIdx.x, t = idx / CH, c = idx - t * CH;
            if (idx < TP * CH) *reinterpret_cast<uint4*>(img[o] + t * stride[o] + c * 8) = v[o][j];
        }
}
// sum of the 8 bf16 products of two 16-B pieces
__device__ __forceinline__ float dot8_bf16(uint4 a, uint4 b) {
    const uint32_t* a32 = reinterpret_cast<const uint32_t*>(&a);
    const uint32_t* b32 = reinterpret_cast<const uint32_t*>(&b);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 4; e++) {
        s += __uint_as_float(a32[e] << 16) * __uint_as_float(b32[e] << 16);
        s += __uint_as_float(a32[e] & 0xffff0000u) * __uint_as_float(b32[e] & 0xffff0000u);
    }
    return s;
}
// four accumulator values (x mul) as four bf16: (v0, v1) and (v2, v3) as two float2 -> bf16x2
// conversions, one v_cvt_pk_bf16_f32 each (hipcc vectorised the scalar pack_bf16x2 form as
// (v0, v2) / (v1, v3) products and then needed six and / shift / or ops to put the halves back);
// the same RNE rounding, bit-identical
typedef float f32x2v_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 pack4_bf16(f32x4_t v, float mul) {
    const f32x2v_t lo = f32x2v_t{v[0], v[1]} * mul, hi = f32x2v_t{v[2], v[3]} * mul;
    return make_uint2(__builtin_bit_cast(uint32_t, __builtin_convertvector(lo, bf16x2v_t)),
                      __builtin_bit_cast(uint32_t, __builtin_convertvector(hi, bf16x2v_t)));
}
__device__ __forceinline__ void store4(bf16_t* dst, f32x4_t v, float mul) {
    *reinterpret_cast<uint2*>(dst) = pack4_bf16(v, mul);
}

// raw buffer loads: offsets past num_records (bytes) return 0, so zero-padded rows need no branch
// (a "zero, then load if in range" pattern makes hipcc wait vmcnt(0) on the whole queue before the
// zeroing, which turned the backward's one-slice-ahead prefetch into a blocking load)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 buf_ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ float buf_ldf(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
typedef uint32_t v2u32_t __attribute__((ext_vector_type(2)));
// the fragment of frag_glb from a buffer resource over the [T][ld] operand (rows >= T read 0)
template <int HS>
__device__ __forceinline__ bf16x8_t frag_buf(__amdgpu_buffer_rsrc_t r, uint32_t ld_bytes, int row, int s, int lane) {
    const uint32_t off = (uint32_t)row * ld_bytes + 2u * (32 * s + 4 * (lane >> 4));
    const bf16x4_t lo = __builtin_bit_cast(bf16x4_t, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
    bf16x4_t hi = {};
    if (!(Geo<HS>::HALF && s == Geo<HS>::KS - 1))
        hi = __builtin_bit_cast(bf16x4_t, __builtin_amdgcn_raw_buffer_load_b64(r, off + 32, 0, 0));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Swizzled LDS images of the one-pass backward at head size 64 (rows of 128 B), conflict-free for
// every access (tools/lds_banks.py model, MI355X_MICROARCH.md §LDS):
//   Q / dO slices [32 q][64 d], stride 128 B, 16-B chunk index XOR gray(row): ds_read_b64 row
//     fragments, ds_read_b64_tr_b16 transposed fragments and the ds_write_b128 staging;
//   dS^T [key][32 q], stride 64 B, 8-B chunk index XOR gray(row): the ds_write_b64 of phase A and
//     the transposed reads of phase B.
// (the padded strides they replace cost 2x on the transposed slice reads and 4x on the dS^T writes)
__device__ __forceinline__ int gray8(int r) { return (r ^ (r >> 1)) & 7; }
__device__ __forceinline__ int sl_off(int row, int byte) { return row * 128 + ((((byte >> 4) ^ gray8(row)) << 4) | (byte & 15)); }
__device__ __forceinline__ int ds_off(int row, int byte) { return row * 64 + ((((byte >> 3) ^ gray8(row)) << 3) | (byte & 7)); }
__device__ __forceinline__ bf16x4_t lds4(const char* img, int off) { return *reinterpret_cast<const bf16x4_t*>(img + off); }
__device__ __forceinline__ bf16x4_t lds4tr(const char* img, int off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4_t, img + off));
}
// swizzled slice: row fragment (rows r0+i, k-step s) and transposed fragment (k rows kb.., cols c0+i)
__device__ __forceinline__ bf16x8_t frag_row_sw(const char* img, int r0, int s, int lane) {
    const int i = lane & 15, g = lane >> 4;
    return __builtin_shufflevector(lds4(img, sl_off(r0 + i, 64 * s + 8 * g)), lds4(img, sl_off(r0 + i, 64 * s + 32 + 8 * g)),
                                   0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8_t frag_tr_sw(const char* img, int kb, int c0, int lane) {
    const int i = lane & 15, g = lane >> 4, r = kb + 4 * g + (i >> 2), b = 2 * c0 + 8 * (i & 3);
    return __builtin_shufflevector(lds4tr(img, sl_off(r, b)), lds4tr(img, sl_off(r + 16, b)), 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8_t frag_tr_ds(const char* img, int kb, int c0, int lane) {
    const int i = lane & 15, g = lane >> 4, r = kb + 4 * g + (i >> 2), b = 2 * c0 + 8 * (i & 3);
    return __builtin_shufflevector(lds4tr(img, ds_off(r, b)), lds4tr(img, ds_off(r + 16, b)), 0, 1, 2, 3, 4, 5, 6, 7);
}

// ---------------------------------------------------------------------------------- forward
template <int HS, int NKT>  // key tiles of 16 covering TP = 16*NKT (a multiple of 32)
constexpr int fwd_lds_bytes() { return NKT * 16 * (Geo<HS>::SK + Geo<HS>::SV) * 2; }
// workgroups per CU the forward's LDS allows (launch bound)
template <int HS, int NKT>
constexpr int fwd_occ() { return fwd_lds_bytes<HS, NKT>() <= 80 * 1024 ? 2 : 1; }

#ifndef VIT_ATTN_FWD_BUF
#define VIT_ATTN_FWD_BUF 1  // K / V staging, Q loads and output / lse stores as buffer operations (no branches in the loop)
#endif
// NS: key tiles that hold a key (< T) -- the score MFMAs, the mask and the exponentials skip the
// all-padding tiles (NKT - NS of them, at most one: TP rounds T up to 32); P.V still runs NKT/2 pairs
template <int HS, int NKT, int NS = NKT>
__global__ __launch_bounds__(256, (fwd_occ<HS, NKT>())) void attn_fwd_k(bf16_t* __restrict__ out,
                                                                        float* __restrict__ lse,
                                                                        const bf16_t* __restrict__ qkv,
                                                                        int T, int C, int NH) {
    using G = Geo<HS>;
    constexpr int TP = NKT * 16;
    __shared__ __attribute__((aligned(16))) bf16_t Ks[TP * G::SK];
    __shared__ __attribute__((aligned(16))) bf16_t Vs[TP * G::SV];
    const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
    const long long C3 = 3LL * C;
    const bf16_t* base = qkv + (long long)b * T * C3 + h * HS;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
    [[maybe_unused]] int it = 15;  // ATTN_STAMP record
    ATTN_STAMP(0);
    // Q fragments of a 16-query tile straight from HBM (rows >= T -> 0); the next tile's are
    // requested while the current one computes, the first ones before the K/V staging
    // Branch-free Q loads and output stores (buffer operations: rows >= T read 0 / are dropped) let
    // hipcc count the loop's vmcnt: the next tile's Q loads are waited for, the previous tile's
    // stores stay in flight (with the "if (q < T)" stores and "row < T" loads it waited vmcnt(0))
    [[maybe_unused]] const auto rq = buf_rsrc(base, (uint32_t)(T * C3 * 2));
    [[maybe_unused]] const auto ro = buf_rsrc(out + (long long)b * T * C + h * HS, (uint32_t)(T * C * 2));
    [[maybe_unused]] const auto rl = buf_rsrc(lse + (long long)bh * T, (uint32_t)(T * 4));
    auto load_q = [&](int qt, bf16x8_t (&qf)[G::KS]) {
#pragma unroll
        for (int s = 0; s < G::KS; s++) {
            if constexpr (VIT_ATTN_FWD_BUF) qf[s] = frag_buf<HS>(rq, (uint32_t)(C3 * 2), qt * 16 + i, s, lane);
            else qf[s] = frag_glb<HS>(base, C3, qt * 16 + i, T, s, lane);
        }
    };
    const int nqt = (T + 15) / 16;
    bf16x8_t qn[G::KS];
    load_q(w, qn);
    if constexpr (VIT_ATTN_FWD_BUF) {
        // K | V rows through one resource from K's first column (every byte of rows >= T is past its
        // end, so those rows read 0 without a branch); all loads before the first LDS store
        const auto rkv = buf_rsrc(base + C, (uint32_t)(T * C3 * 2 - 2 * C));
        constexpr int CH = G::CH, PER = (TP * CH + 255) / 256;
        uint4 v[2][PER];
#pragma unroll
        for (int o = 0; o < 2; o++)
#pragma unroll
            for (int j = 0; j < PER; j++) {
                const int idx = j * 256 + (int)threadIdx.x, t = idx / CH, cc = idx - t * CH;
                v[o][j] = buf_ld16(rkv, (uint32_t)t * (uint32_t)(C3 * 2) + (uint32_t)(o * C * 2) + 16 * cc);
            }
#pragma unroll
        for (int o = 0; o < 2; o++)
#pragma unroll
            for (int j = 0; j < PER; j++) {
                const int idx = j * 256 + (int)threadIdx.x, t = idx / CH, cc = idx - t * CH;
                if ((TP * CH) % 256 == 0 || idx < TP * CH)
                    *reinterpret_cast<uint4*>((o ? Vs + t * G::SV : Ks + t * G::SK) + cc * 8) = v[o][j];
            }
    } else {
        bf16_t* const img[2] = {Ks, Vs};
        const int st[2] = {G::SK, G::SV};
        const bf16_t* const src[2] = {base + C, base + 2 * C};
        const long long ld[2] = {C3, C3};
        load_images<HS, TP, 256, 2>(img, st, src, ld, T);
    }
    ATTN_STAMP(1);
    __syncthreads();
    ATTN_STAMP(2);
    const float c = LOG2E / sqrtf((float)HS);
#ifndef VIT_ATTN_FWD_SPLIT
#define VIT_ATTN_FWD_SPLIT 1  // K row fragments as separate ds_read_b64 (RowBases); 0: hipcc merges them into ds_read2_b64
#endif
    const RowBases<HS> kb(Ks, G::SK, lane);
    for (int qt = w; qt < nqt; qt += 4) {
        const int q = qt * 16 + i;
        it = qt / 4;
        ATTN_STAMP(0);
        bf16x8_t qf[G::KS];
#pragma unroll
        for (int s = 0; s < G::KS; s++) qf[s] = qn[s];
        if (qt + 4 < nqt) load_q(qt + 4, qn);
        f32x4_t sacc[NKT];
#pragma unroll
        for (int kt = NS; kt < NKT; kt++) sacc[kt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kt = 0; kt < NS; kt++) {
            f32x4_t a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < G::KS; s++) {
                if constexpr (VIT_ATTN_FWD_SPLIT) a = mfma(kb.frag(kt * 16, G::SK, s), qf[s], a);
                else a = mfma(frag_row<HS>(Ks, G::SK, kt * 16, s, lane), qf[s], a);
            }
            sacc[kt] = a;
        }
        ATTN_STAMP(1);
        // lane (i,g) holds S^T[key = 16kt+4g+r][q]: the maximum of the raw scores (c > 0 commutes with
        // it), then p = 2^(s c - max c) as one FMA (a per-key-tile branch around the padded-key mask
        // measured slower: 107 vs 104 us, it splits the block the scheduler interleaves)
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < NS; kt++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                // padded keys lie in the last score tile (trimmed launch) or the last two (NKT = 2 ceil(T/32))
                const float x = kt < (NS < NKT ? NS - 1 : NKT - 2) || kt * 16 + 4 * g + r < T ? sacc[kt][r] : -INFINITY;
                sacc[kt][r] = x;
                mx = fmaxf(mx, x);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        mx *= c;
        float l = 0.f;
#ifndef VIT_ATTN_FWD_PK
#define VIT_ATTN_FWD_PK 1  // exponent arguments as packed fp32 (v_pk_fma_f32)
#endif
#ifndef VIT_ATTN_FWD_PAIRSUM
#define VIT_ATTN_FWD_PAIRSUM 1  // two row-sum chains + v_rcp / v_log (r06; fp8 curve re-recorded)
#endif
        if constexpr (VIT_ATTN_FWD_PK) {
            // r06: the row sum as two chains (even / odd score of each pair) and
            // 1 / l, log2 l on v_rcp_f32 / v_log_f32.  Both change the rounding of l / lse within every
            // oracle gate of the attention and model tests; the fp8 loss-curve fixture, a drift alarm,
            // was re-recorded under the rule in tests/golden/make_fp8_curve.py.
            typedef float f32x2_t __attribute__((ext_vector_type(2)));
            const f32x2_t c2 = {c, c}, m2 = {-mx, -mx};
            float l1 = 0.f;
#pragma unroll
            for (int kt = 0; kt < NS; kt++)
#pragma unroll
                for (int r = 0; r < 4; r += 2) {
                    const f32x2_t x = {sacc[kt][r], sacc[kt][r + 1]};
                    const f32x2_t y = __builtin_elementwise_fma(x, c2, m2);
                    sacc[kt][r] = fexp2(y.x);
                    sacc[kt][r + 1] = fexp2(y.y);
                    l += sacc[kt][r];
                    if constexpr (VIT_ATTN_FWD_PAIRSUM) l1 += sacc[kt][r + 1];
                    else l += sacc[kt][r + 1];
                }
            if constexpr (VIT_ATTN_FWD_PAIRSUM) l += l1;
        } else {
#pragma unroll
            for (int kt = 0; kt < NS; kt++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const float p = fexp2(fmaf(sacc[kt][r], c, -mx));
                    sacc[kt][r] = p;
                    l += p;
                }
        }
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
        ATTN_STAMP(2);
        f32x4_t o[G::DT];
#pragma unroll
        for (int dt = 0; dt < G::DT; dt++) o[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKT / 2; ks++) {
            const bf16x8_t pb = pack_acc(sacc[2 * ks], sacc[2 * ks + 1]);
#pragma unroll
            for (int dt = 0; dt < G::DT; dt++) o[dt] = mfma(frag_tr(Vs, G::SV, 32 * ks, 16 * dt, lane), pb, o[dt]);
        }
        ATTN_STAMP(3);
        if constexpr (VIT_ATTN_FWD_BUF) {
            // every lane stores: rows q >= T fall past the resources' ends; the four lanes of a query
            // write the same lse value
            const float inv = VIT_ATTN_FWD_PAIRSUM ? __builtin_amdgcn_rcpf(l) : 1.0f / l;
            const uint32_t off = (uint32_t)q * (uint32_t)(C * 2) + 8u * g;
#pragma unroll
            for (int dt = 0; dt < G::DT; dt++) {
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u32_t, pack4_bf16(o[dt], inv)), ro,
                                                      off + 32u * dt, 0, 0);
            }
            __builtin_amdgcn_raw_buffer_store_b32(
                __builtin_bit_cast(uint32_t, mx + (VIT_ATTN_FWD_PAIRSUM ? __builtin_amdgcn_logf(l) : log2f(l))), rl, 4u * q, 0, 0);
        } else if (q < T) {
            const float inv = 1.0f / l;
            bf16_t* dst = out + ((long long)b * T + q) * C + h * HS + 4 * g;
#pragma unroll
            for (int dt = 0; dt < G::DT; dt++) store4(dst + 16 * dt, o[dt], inv);
            if (g == 0) lse[(long long)bh * T + q] = mx + log2f(l);
        }
        ATTN_STAMP(4);
    }
    it = 15;
    ATTN_STAMP(3);
}

// --------------------------------------------------------------------------------- backward
// Two roles of one launch with 32-row register tiles (bwd_kv_body and bwd_q_body), a 256-thread
// workgroup per (b,h) and role.  Each fragment read from LDS feeds two 16-row MFMA tiles:
//   kv: wave owns 32 keys (K, V fragments in registers, dK^T / dV^T accumulators); per 32-query
//       chunk: S, dP (Q / dO rows from LDS), P = exp2(S c - lse), dS = P (dP - delta),
//       dV^T += dO^T P, dK^T += Q^T dS (transposed reads).
//   q:  wave owns 32 queries (Q, dO fragments in registers, dQ^T accumulators); per 32-key chunk:
//       S^T, dP^T (K / V rows from LDS), dQ^T += K^T dS^T.
// Rows >= T are zero-filled, so padded keys contribute nothing to dQ; padded queries have
// lse = +inf (P = 0).  P of padded keys is zeroed for the fused bias column sums.
template <int HS, int NKT>
constexpr int bwd_lds_bytes() {
    return 2 * NKT * 16 * Geo<HS>::SK * 2 + 2 * NKT * 16 * 4 + 4 * 2 * HS * 4;
}
template <int HS, int NKT>
constexpr int bwd_occ() { return bwd_lds_bytes<HS, NKT>() <= 80 * 1024 ? 2 : 1; }

template <int HS, int NKT>
__device__ __forceinline__ void bwd_kv_body(char* lds, int bh, bf16_t* __restrict__ dqkv,
                                            const bf16_t* __restrict__ dout,
                                            const bf16_t* __restrict__ qkv,
                                            const bf16_t* __restrict__ out,
                                            const float* __restrict__ lse, int T, int C, int NH,
                                            float* __restrict__ dsum) {
    using G = Geo<HS>;
    constexpr int TP = NKT * 16;  // padded length, multiple of 32
    constexpr int SK = G::SK, KS = G::KS, DT = G::DT;
    bf16_t* Qs = reinterpret_cast<bf16_t*>(lds);
    bf16_t* Ds = Qs + TP * SK;
    float* lse_s = reinterpret_cast<float*>(Ds + TP * SK);
    float* del_s = lse_s + TP;
    float (*csum_s)[2 * HS] = reinterpret_cast<float (*)[2 * HS]>(del_s + TP);
    const int b = bh / NH, h = bh % NH;
    const long long C3 = 3LL * C;
    const bf16_t* base = qkv + (long long)b * T * C3 + h * HS;
    const bf16_t* dbase = dout + (long long)b * T * C + h * HS;
    const bf16_t* obase = out + (long long)b * T * C + h * HS;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = lane & 15, g = lane >> 4;
    // K, V fragments of a 2 x 16-key tile straight from HBM (rows >= T -> 0); the wave's first
    // tile is requested before the Q/dO staging so its latency hides behind it
    auto load_kv = [&](int kt, bf16x8_t (&kf)[2][KS], bf16x8_t (&vf)[2][KS]) {
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
            const int key = kt * 32 + kk * 16 + i;
#pragma unroll
            for (int s = 0; s < KS; s++) {
                kf[kk][s] = frag_glb<HS>(base + C, C3, key, T, s, lane);
                vf[kk][s] = frag_glb<HS>(base + 2 * C, C3, key, T, s, lane);
            }
        }
    };
    bf16x8_t kf[2][KS], vf[2][KS];
    if (w < TP / 32) load_kv(w, kf, vf);
    {
        bf16_t* const img[2] = {Qs, Ds};
        const int st[2] = {SK, SK};
        const bf16_t* const src[2] = {base, dbase};
        const long long ld[2] = {C3, C};
        load_images<HS, TP, 256, 2>(img, st, src, ld, T);
    }
    __syncthreads();
    // delta = rowsum(dO * O) per query (O from HBM, dO from the image), lse staged
    for (int t = tid; t < TP; t += 256) {
        float dl = 0.f, ls = INFINITY;
        if (t < T) {
            ls = lse[(long long)bh * T + t];
            uint4 ov[G::CH];
#pragma unroll
            for (int cc = 0; cc < G::CH; cc++) ov[cc] = *reinterpret_cast<const uint4*>(obase + (long long)t * C + cc * 8);
#pragma unroll
            for (int cc = 0; cc < G::CH; cc++) {
                const uint4 dv = *reinterpret_cast<const uint4*>(Ds + t * SK + cc * 8);
                const uint32_t* o32 = reinterpret_cast<const uint32_t*>(&ov[cc]);
                const uint32_t* d32 = reinterpret_cast<const uint32_t*>(&dv);
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    dl += __uint_as_float(o32[e] << 16) * __uint_as_float(d32[e] << 16);
                    dl += __uint_as_float(o32[e] & 0xffff0000u) * __uint_as_float(d32[e] & 0xffff0000u);
                }
            }
        }
        lse_s[t] = ls;
        del_s[t] = dl;
    }
    __syncthreads();
    const float scale = 1.0f / sqrtf((float)HS);
    const float c = LOG2E * scale;
    f32x4_t ck[DT] = {}, cv[DT] = {};  // this lane's share of the dK / dV column sums
    for (int kt = w; kt < TP / 32; kt += 4) {
        const int key0 = kt * 32;
        if (kt != w) load_kv(kt, kf, vf);
        const bool kok[2] = {key0 + i < T, key0 + 16 + i < T};
        f32x4_t dv[2][DT], dk[2][DT];
#pragma unroll
        for (int kk = 0; kk < 2; kk++)
#pragma unroll
            for (int dt = 0; dt < DT; dt++) dv[kk][dt] = dk[kk][dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int qs = 0; qs < TP / 32; qs++) {
            f32x4_t P[2][2], dS[2][2];  // [kk][u]: lane (i,g) -> [q = 32qs+16u+4g+r][key = 16kk+i]
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int qt0 = qs * 32 + u * 16;
                bf16x8_t qr[KS], dr[KS];
#pragma unroll
                for (int s = 0; s < KS; s++) {
                    qr[s] = frag_row<HS>(Qs, SK, qt0, s, lane);
                    dr[s] = frag_row<HS>(Ds, SK, qt0, s, lane);
                }
                float lq[4], dq[4];
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    lq[r] = lse_s[qt0 + 4 * g + r];
                    dq[r] = del_s[qt0 + 4 * g + r];
                }
#pragma unroll
                for (int kk = 0; kk < 2; kk++) {
                    f32x4_t s_ = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int s = 0; s < KS; s++) {
                        s_ = mfma(qr[s], kf[kk][s], s_);
                        dp = mfma(dr[s], vf[kk][s], dp);
                    }
                    // padded keys (K, V rows zero) get P != 0 here; they only reach dK / dV rows
                    // that are neither stored nor summed
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const float pv = fexp2(s_[r] * c - lq[r]);
                        P[kk][u][r] = pv;
                        dS[kk][u][r] = pv * (dp[r] - dq[r]);
                    }
                }
            }
            bf16x8_t pb[2], db[2];
#pragma unroll
            for (int kk = 0; kk < 2; kk++) {
                pb[kk] = pack_acc(P[kk][0], P[kk][1]);
                db[kk] = pack_acc(dS[kk][0], dS[kk][1]);
            }
#pragma unroll
            for (int dt = 0; dt < DT; dt++) {
                const bf16x8_t td = frag_tr(Ds, SK, 32 * qs, 16 * dt, lane);
                const bf16x8_t tq = frag_tr(Qs, SK, 32 * qs, 16 * dt, lane);
#pragma unroll
                for (int kk = 0; kk < 2; kk++) {
                    dv[kk][dt] = mfma(td, pb[kk], dv[kk][dt]);
                    dk[kk][dt] = mfma(tq, db[kk], dk[kk][dt]);
                }
            }
        }
        // lane (i,g) of tile (kk,dt): key = key0 + 16kk + i, d = 16dt + 4g + r
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
            if (!kok[kk]) continue;
            bf16_t* dst = dqkv + ((long long)b * T + key0 + kk * 16 + i) * C3 + h * HS + 4 * g;
#pragma unroll
            for (int dt = 0; dt < DT; dt++) {
                store4(dst + C + 16 * dt, dk[kk][dt], scale);
                store4(dst + 2 * C + 16 * dt, dv[kk][dt], 1.0f);
            }
        }
        if (dsum) {
#pragma unroll
            for (int kk = 0; kk < 2; kk++) {
                if (!kok[kk]) continue;
#pragma unroll
                for (int dt = 0; dt < DT; dt++) {
                    ck[dt] += dk[kk][dt] * scale;
                    cv[dt] += dv[kk][dt];
                }
            }
        }
    }
    if (dsum) {  // per-(b,h) column sums of dK, dV -> dsum[bh][HS .. 3HS)
#pragma unroll
        for (int dt = 0; dt < DT; dt++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float tk = ck[dt][r], tv = cv[dt][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    tk += __shfl_xor(tk, o, 64);
                    tv += __shfl_xor(tv, o, 64);
                }
                if (i == 0) {
                    csum_s[w][16 * dt + 4 * g + r] = tk;
                    csum_s[w][HS + 16 * dt + 4 * g + r] = tv;
                }
            }
        __syncthreads();
        if (tid < 2 * HS)
            dsum[(long long)bh * 3 * HS + HS + tid] = csum_s[0][tid] + csum_s[1][tid] + csum_s[2][tid] + csum_s[3][tid];
    }
}

template <int HS, int NKT>
__device__ __forceinline__ void bwd_q_body(char* lds, int bh, bf16_t* __restrict__ dqkv,
                                           const bf16_t* __restrict__ dout,
                                           const bf16_t* __restrict__ qkv,
                                           const bf16_t* __restrict__ out,
                                           const float* __restrict__ lse, int T, int C, int NH,
                                           float* __restrict__ dsum) {
    using G = Geo<HS>;
    constexpr int TP = NKT * 16;
    constexpr int SK = G::SK, KS = G::KS, DT = G::DT;
    bf16_t* Ks = reinterpret_cast<bf16_t*>(lds);
    bf16_t* Vs = Ks + TP * SK;
    float (*csum_s)[HS] = reinterpret_cast<float (*)[HS]>(Vs + TP * SK);
    const int b = bh / NH, h = bh % NH;
    const bf16_t* obase = out + (long long)b * T * C + h * HS;
    const long long C3 = 3LL * C;
    const bf16_t* base = qkv + (long long)b * T * C3 + h * HS;
    const bf16_t* dbase = dout + (long long)b * T * C + h * HS;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = lane & 15, g = lane >> 4;
    // own 32-query tile: Q / dO fragments, lse, delta straight from HBM; the next tile's are
    // requested while the current one computes, the first ones before the K/V staging
    auto load_tile = [&](int qt, bf16x8_t (&qf)[2][KS], bf16x8_t (&df)[2][KS], float (&lq)[2], float (&dl)[2]) {
        const int q0 = qt * 32;
        float part[2] = {0.f, 0.f};
#pragma unroll
        for (int qq = 0; qq < 2; qq++) {
            const int q = q0 + qq * 16 + i;
#pragma unroll
            for (int s = 0; s < KS; s++) {
                qf[qq][s] = frag_glb<HS>(base, C3, q, T, s, lane);
                df[qq][s] = frag_glb<HS>(dbase, C, q, T, s, lane);
                const bf16x8_t of = frag_glb<HS>(obase, C, q, T, s, lane);
                // delta = rowsum(dO * O): this lane's share of the query's HS columns (the
                // zero padding of a half k-step adds nothing)
#pragma unroll
                for (int e = 0; e < 8; e++) part[qq] += (float)df[qq][s][e] * (float)of[e];
            }
            lq[qq] = q < T ? lse[(long long)bh * T + q] : INFINITY;
        }
#pragma unroll
        for (int qq = 0; qq < 2; qq++) {  // the 4 lanes of a query are lane, lane ^ 16, ^ 32
            float t = part[qq];
            t += __shfl_xor(t, 16, 64);
            t += __shfl_xor(t, 32, 64);
            dl[qq] = t;
        }
    };
    bf16x8_t qn[2][KS], dn[2][KS];
    float lqn[2], dln[2];
    if (w < TP / 32) load_tile(w, qn, dn, lqn, dln);
    {
        bf16_t* const img[2] = {Ks, Vs};
        const int st[2] = {SK, SK};
        const bf16_t* const src[2] = {base + C, base + 2 * C};
        const long long ld[2] = {C3, C3};
        load_images<HS, TP, 256, 2>(img, st, src, ld, T);
    }
    __syncthreads();
    const float scale = 1.0f / sqrtf((float)HS);
    const float c = LOG2E * scale;
    f32x4_t cq[DT] = {};
    for (int qt = w; qt < TP / 32; qt += 4) {
        const int q0 = qt * 32;
        bf16x8_t qf[2][KS], df[2][KS];
        float lq[2], dl[2];
#pragma unroll
        for (int qq = 0; qq < 2; qq++) {
            lq[qq] = lqn[qq];
            dl[qq] = dln[qq];
#pragma unroll
            for (int s = 0; s < KS; s++) {
                qf[qq][s] = qn[qq][s];
                df[qq][s] = dn[qq][s];
            }
        }
        if (qt + 4 < TP / 32) load_tile(qt + 4, qn, dn, lqn, dln);
        f32x4_t dq[2][DT];
#pragma unroll
        for (int qq = 0; qq < 2; qq++)
#pragma unroll
            for (int dt = 0; dt < DT; dt++) dq[qq][dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int ks = 0; ks < TP / 32; ks++) {
            f32x4_t dS[2][2];  // [qq][u]: lane (i,g) -> [key = 32ks+16u+4g+r][q = 16qq+i]
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int kt0 = ks * 32 + u * 16;
                bf16x8_t kr[KS], vr[KS];
#pragma unroll
                for (int s = 0; s < KS; s++) {
                    kr[s] = frag_row<HS>(Ks, SK, kt0, s, lane);
                    vr[s] = frag_row<HS>(Vs, SK, kt0, s, lane);
                }
#pragma unroll
                for (int qq = 0; qq < 2; qq++) {
                    f32x4_t s_ = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int s = 0; s < KS; s++) {
                        s_ = mfma(kr[s], qf[qq][s], s_);
                        dp = mfma(vr[s], df[qq][s], dp);
                    }
#pragma unroll
                    for (int r = 0; r < 4; r++) dS[qq][u][r] = fexp2(s_[r] * c - lq[qq]) * (dp[r] - dl[qq]);
                }
            }
            bf16x8_t db[2];
#pragma unroll
            for (int qq = 0; qq < 2; qq++) db[qq] = pack_acc(dS[qq][0], dS[qq][1]);
#pragma unroll
            for (int dt = 0; dt < DT; dt++) {
                const bf16x8_t tk = frag_tr(Ks, SK, 32 * ks, 16 * dt, lane);
#pragma unroll
                for (int qq = 0; qq < 2; qq++) dq[qq][dt] = mfma(tk, db[qq], dq[qq][dt]);
            }
        }
#pragma unroll
        for (int qq = 0; qq < 2; qq++) {
            const int q = q0 + qq * 16 + i;
            if (q >= T) continue;
            bf16_t* dst = dqkv + ((long long)b * T + q) * C3 + h * HS + 4 * g;
#pragma unroll
            for (int dt = 0; dt < DT; dt++) store4(dst + 16 * dt, dq[qq][dt], scale);
        }
        if (dsum) {  // padded queries: dS = exp2(-inf) * ... = 0
#pragma unroll
            for (int qq = 0; qq < 2; qq++)
#pragma unroll
                for (int dt = 0; dt < DT; dt++) cq[dt] += dq[qq][dt] * scale;
        }
    }
    if (dsum) {
#pragma unroll
        for (int dt = 0; dt < DT; dt++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float tq = cq[dt][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) tq += __shfl_xor(tq, o, 64);
                if (i == 0) csum_s[w][16 * dt + 4 * g + r] = tq;
            }
        __syncthreads();
        if (tid < HS) dsum[(long long)bh * 3 * HS + tid] = csum_s[0][tid] + csum_s[1][tid] + csum_s[2][tid] + csum_s[3][tid];
    }
}

// kv and q roles of one (b,h) in ONE launch: the two workgroups of a pair are dealt to the same
// XCD back to back (block ids 16k + x and 16k + 8 + x), so the second reads of Q, K, V, dO, O
// are served from that XCD's L2 instead of HBM.  Both roles compute delta themselves.
template <int HS, int NKT>
__global__ __launch_bounds__(256, (bwd_occ<HS, NKT>())) void attn_bwd_pair_k(
    bf16_t* __restrict__ dqkv, const bf16_t* __restrict__ dout, const bf16_t* __restrict__ qkv,
    const bf16_t* __restrict__ out, const float* __restrict__ lse, int T, int C, int NH, int BH,
    float* __restrict__ dsum) {
    __shared__ __attribute__((aligned(16))) char lds[bwd_lds_bytes<HS, NKT>()];
    const int x = blockIdx.x & 7, grp = blockIdx.x >> 3;
    const int role = grp & 1, bh = (grp >> 1) * 8 + x;
    if (bh >= BH) return;
    if (role == 0) bwd_kv_body<HS, NKT>(lds, bh, dqkv, dout, qkv, out, lse, T, C, NH, dsum);
    else bwd_q_body<HS, NKT>(lds, bh, dqkv, dout, qkv, out, lse, T, C, NH, dsum);
}

// ------------------------------------------------------------------ backward, one pass (default)
// One workgroup per (b,h) item, NW = TP/32 waves; wave w owns keys [32w, 32w+32): its K, V
// fragments (B operands of S and dP) and dK^T, dV^T accumulators stay in registers while the
// workgroup sweeps the queries in 32-row slices (Q / dO slices double-buffered in LDS, the next
// one prefetched into registers during the current one).  Per slice:
//   A: S, dP with the key on the lane; P = exp2(S c - lse), dS = P (dP - delta) — each score's
//      exp computed once; dV^T += dO^T P, dK^T += Q^T dS (transposed slice reads); dS^T (bf16)
//      into LDS [key][query];                                                      barrier
//   B: dQ^T = K^T . dS^T for the slice's 2·HS/16 output tiles, spread over the waves (K image
//      and dS^T both read transposed); stores.                                    barrier
// = the five products of the flash backward (train_vit.rs:559-601 with the O(T^2) softmax
// Jacobian form) with no recomputation: per 32x32 block 5 x (HS/16 or 2·KS) MFMAs instead of
// the paired roles' 7.  dQ needs no cross-workgroup sum: the workgroup holds every key.
// Two forms: attn_bwdp_k (persistent: one workgroup per CU walks the items and fetches the next
// item's K / V rows and the next slice's Q / dO / O rows under the current slice's MFMA work) and
// attn_bwd1_k (one workgroup per item, blocking prologue) where the persistent LDS does not fit.
constexpr int BWD_SDS = 48;          // dS^T [key][query] row stride: (SDS/2) = 8*odd dwords (tr reads)
constexpr int ATTN_PART_ROWS = 16;   // column-sum partial rows per (b,h) a backward kernel may write
// slice-image and dS^T row strides (elements): the swizzled images at head size 64 (sl_off, ds_off)
// VIT_ATTN_SW_SLICE: swizzled 128-B slice rows (conflict-free transposed reads, more address
// registers) vs the padded stride; the dS^T swizzle is always on at head size 64
#ifndef VIT_ATTN_SW_SLICE
#define VIT_ATTN_SW_SLICE 1
#endif

template <int HS>
constexpr bool sw_slice() { return HS == 64 && VIT_ATTN_SW_SLICE; }
#ifndef VIT_ATTN_SW_DS
#define VIT_ATTN_SW_DS 1
#endif
template <int HS>
constexpr bool sw_ds() { return HS == 64 && VIT_ATTN_SW_DS; }
template <int HS>
constexpr int slice_stride() { return sw_slice<HS>() ? 64 : Geo<HS>::SK; }
template <int HS>
constexpr int sds_stride() { return sw_ds<HS>() ? 32 : BWD_SDS; }
// element (row j, column d) of a slice image as fp32
template <int HS>
__device__ __forceinline__ float slice_at(const bf16_t* img, int j, int d) {
    if constexpr (sw_slice<HS>()) return bf2f(*reinterpret_cast<const bf16_t*>(reinterpret_cast<const char*>(img) + sl_off(j, 2 * d)));
    else return bf2f(img[j * Geo<HS>::SK + d]);
}
// dims 8p .. 8p+7 of slice row j (one 16-B read; the swizzle moves whole 16-B chunks)
template <int HS>
__device__ __forceinline__ uint4 slice_chunk8(const bf16_t* img, int j, int p) {
    if constexpr (sw_slice<HS>()) return *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(img) + sl_off(j, 16 * p));
    else return *reinterpret_cast<const uint4*>(img + j * Geo<HS>::SK + 8 * p);
}
// 16-B piece cc of slice row t into a slice image
template <int HS>
__device__ __forceinline__ void slice_put(bf16_t* img, int t, int cc, uint4 v) {
    if constexpr (sw_slice<HS>()) *reinterpret_cast<uint4*>(reinterpret_cast<char*>(img) + sl_off(t, 16 * cc)) = v;
    else *reinterpret_cast<uint4*>(img + t * Geo<HS>::SK + cc * 8) = v;
}

template <int HS, int KK = 2>
struct BwdRegs {  // per-wave state of the one-pass backward: the wave owns KK 16-key tiles
    bf16x8_t kf[KK][Geo<HS>::KS], vf[KK][Geo<HS>::KS];  // K, V rows of the wave's keys (B operands)
    f32x4_t dv[KK][Geo<HS>::DT], dk[KK][Geo<HS>::DT];   // [kk][dt]: lane (i,g) -> [d = 16dt+4g+r][key = 16kk+i]
    // per-key sums of dS over the queries: the dQ column sums (qkv-bias gradient) follow as
    // sum_q dQ[q][d] = scale * sum_key (sum_q dS[q][key]) K[key][d], with K in registers
    float sds[KK];
    __device__ __forceinline__ void zero() {
#pragma unroll
        for (int kk = 0; kk < KK; kk++) {
#pragma unroll
            for (int dt = 0; dt < Geo<HS>::DT; dt++) dv[kk][dt] = dk[kk][dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            sds[kk] = 0.f;
        }
    }
};

// phase A of one 32-query slice for the wave's keys: Qc / Dc slice images (stride SK), lq / dl the
// slice's lse / delta, dSk = dS^T rows of the wave's first key
// MASK: for operands whose rows past T are copies of row T-1 (not zero), the probabilities
// of padded queries (q >= T) and keys (key >= T) are masked to 0 (nq / nk: valid queries / keys
// counted from the slice's and the wave's first one)
#ifndef VIT_ATTN_AHOIST
#define VIT_ATTN_AHOIST 0  // phase A: all reads / score MFMAs first, 1-3: transposed reads all / half / none hoisted (0: per 16-query half; 1-3 spill at ViT-B/16)
#endif
template <int HS, int KK = 2, bool MASK = false>
__device__ __forceinline__ void bwd_slice_a(BwdRegs<HS, KK>& R, const bf16_t* Qc, const bf16_t* Dc, const float* lq_s,
                                            const float* dl_s, bf16_t* dSk, float c, int lane, int nq = 0,
                                            int nk = 0) {
    using G = Geo<HS>;
    constexpr int KS = G::KS, DT = G::DT, SK = G::SK;
    constexpr bool SW = sw_slice<HS>(), SWD = sw_ds<HS>();  // swizzled slice / dS^T images (sl_off / ds_off)
    const int i = lane & 15, g = lane >> 4;
    f32x4_t P[KK][2], dS[KK][2];  // [kk][u]: lane (i,g) -> [q = 16u+4g+r][key = 16kk+i]
    bf16x8_t pb[KK], db[KK];
    auto tr_frags = [&](int dt, bf16x8_t& td, bf16x8_t& tq) {
        if constexpr (SW) {
            td = frag_tr_sw(reinterpret_cast<const char*>(Dc), 0, 16 * dt, lane);
            tq = frag_tr_sw(reinterpret_cast<const char*>(Qc), 0, 16 * dt, lane);
        } else {
            td = frag_tr(Dc, SK, 0, 16 * dt, lane);
            tq = frag_tr(Qc, SK, 0, 16 * dt, lane);
        }
    };
#if VIT_ATTN_AHOIST
    // Every LDS read first (both 16-query halves' row fragments, lse / delta), then all 16 score
    // MFMAs, then the transposed fragments of the dV / dK products, requested before the
    // exponentials so they land under them.  Same products and sums in the same order as the
    // per-half form below (bit-identical); it waited on each half's reads and on the transposed
    // reads right in front of the MFMAs that consume them.
    bf16x8_t qr[2][KS], dr[2][KS];
    float lq[2][4], dq[2][4];
#pragma unroll
    for (int u = 0; u < 2; u++) {
#pragma unroll
        for (int s = 0; s < KS; s++) {
            if constexpr (SW) {
                qr[u][s] = frag_row_sw(reinterpret_cast<const char*>(Qc), 16 * u, s, lane);
                dr[u][s] = frag_row_sw(reinterpret_cast<const char*>(Dc), 16 * u, s, lane);
            } else {
                qr[u][s] = frag_row<HS>(Qc, SK, 16 * u, s, lane);
                dr[u][s] = frag_row<HS>(Dc, SK, 16 * u, s, lane);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            lq[u][r] = lq_s[16 * u + 4 * g + r];
            dq[u][r] = dl_s[16 * u + 4 * g + r];
        }
    }
    f32x4_t sa[KK][2], pa[KK][2];
#pragma unroll
    for (int u = 0; u < 2; u++)
#pragma unroll
        for (int kk = 0; kk < KK; kk++) {
            f32x4_t s_ = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < KS; s++) {
                s_ = mfma(qr[u][s], R.kf[kk][s], s_);
                dp = mfma(dr[u][s], R.vf[kk][s], dp);
            }
            sa[kk][u] = s_;
            pa[kk][u] = dp;
        }
    // VIT_ATTN_AHOIST 1: all DT transposed pairs before the exponentials; 2: the first TRH of them
    constexpr int TRH = VIT_ATTN_AHOIST == 1 ? DT : VIT_ATTN_AHOIST == 2 ? (DT + 1) / 2 : 0;
    bf16x8_t td[DT], tq[DT];
#pragma unroll
    for (int dt = 0; dt < TRH; dt++) tr_frags(dt, td[dt], tq[dt]);
#pragma unroll
    for (int u = 0; u < 2; u++)
#pragma unroll
        for (int kk = 0; kk < KK; kk++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float pv = fexp2(sa[kk][u][r] * c - lq[u][r]);
                if constexpr (MASK) pv = (16 * u + 4 * g + r < nq && 16 * kk + i < nk) ? pv : 0.f;
                P[kk][u][r] = pv;
                dS[kk][u][r] = pv * (pa[kk][u][r] - dq[u][r]);
                R.sds[kk] += dS[kk][u][r];
            }
#pragma unroll
    for (int kk = 0; kk < KK; kk++) {
        pb[kk] = pack_acc(P[kk][0], P[kk][1]);
        db[kk] = pack_acc(dS[kk][0], dS[kk][1]);
    }
#pragma unroll
    for (int dt = TRH; dt < DT; dt++) tr_frags(dt, td[dt], tq[dt]);
#pragma unroll
    for (int dt = 0; dt < DT; dt++)
#pragma unroll
        for (int kk = 0; kk < KK; kk++) {
            R.dv[kk][dt] = mfma(td[dt], pb[kk], R.dv[kk][dt]);
            R.dk[kk][dt] = mfma(tq[dt], db[kk], R.dk[kk][dt]);
        }
#else
#pragma unroll
    for (int u = 0; u < 2; u++) {
        bf16x8_t qr[KS], dr[KS];
#pragma unroll
        for (int s = 0; s < KS; s++) {
            if constexpr (SW) {
                qr[s] = frag_row_sw(reinterpret_cast<const char*>(Qc), 16 * u, s, lane);
                dr[s] = frag_row_sw(reinterpret_cast<const char*>(Dc), 16 * u, s, lane);
            } else {
                qr[s] = frag_row<HS>(Qc, SK, 16 * u, s, lane);
                dr[s] = frag_row<HS>(Dc, SK, 16 * u, s, lane);
            }
        }
        float lq[4], dq[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            lq[r] = lq_s[16 * u + 4 * g + r];
            dq[r] = dl_s[16 * u + 4 * g + r];
        }
#pragma unroll
        for (int kk = 0; kk < KK; kk++) {
            f32x4_t s_ = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < KS; s++) {
                s_ = mfma(qr[s], R.kf[kk][s], s_);
                dp = mfma(dr[s], R.vf[kk][s], dp);
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float pv = fexp2(s_[r] * c - lq[r]);
                if constexpr (MASK) pv = (16 * u + 4 * g + r < nq && 16 * kk + i < nk) ? pv : 0.f;
                P[kk][u][r] = pv;
                dS[kk][u][r] = pv * (dp[r] - dq[r]);
                R.sds[kk] += dS[kk][u][r];
            }
        }
    }
#pragma unroll
    for (int kk = 0; kk < KK; kk++) {
        pb[kk] = pack_acc(P[kk][0], P[kk][1]);
        db[kk] = pack_acc(dS[kk][0], dS[kk][1]);
    }
#pragma unroll
    for (int dt = 0; dt < DT; dt++) {
        bf16x8_t td, tq;
        tr_frags(dt, td, tq);
#pragma unroll
        for (int kk = 0; kk < KK; kk++) {
            R.dv[kk][dt] = mfma(td, pb[kk], R.dv[kk][dt]);
            R.dk[kk][dt] = mfma(tq, db[kk], R.dk[kk][dt]);
        }
    }
#endif
    // dS^T -> LDS [key][query] (bf16, the MFMA operand's values): 4 consecutive queries per lane
    // and tile.  Without MASK, padded keys carry P != 0 (their K, V rows are zero): their dS is
    // finite and multiplies the zero K rows in dQ.  dSk = the wave's first key row.
#pragma unroll
    for (int kk = 0; kk < KK; kk++)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const bf16x4_t h4 = u ? __builtin_shufflevector(db[kk], db[kk], 4, 5, 6, 7)
                                  : __builtin_shufflevector(db[kk], db[kk], 0, 1, 2, 3);
            if constexpr (SWD)
                *reinterpret_cast<bf16x4_t*>(reinterpret_cast<char*>(dSk) + ds_off(16 * kk + i, 32 * u + 8 * g)) = h4;
            else
                *reinterpret_cast<bf16x4_t*>(dSk + (16 * kk + i) * BWD_SDS + 16 * u + 4 * g) = h4;
        }
}

// phase B: dQ^T tiles (dt, u) of the slice at q0, spread over the NW waves; dq = dqkv Q rows of the item
// xk_ds / xk_k (XK): dS[q][T-1] per query of the slice and K[T-1] (fp32) of a key the kernel does not
// own on the MFMA path (the XK side path): its rank-1 term dS[q][T-1] K[T-1] joins the dQ
// accumulators before the store
#ifndef VIT_ATTN_BLA
#define VIT_ATTN_BLA 2  // phase B operand lookahead (blocks); 0: reads in front of each MFMA
#endif
template <int HS, int NSL, int NW, bool XK = false>
__device__ __forceinline__ void bwd_slice_b(const bf16_t* Ks, const bf16_t* dSs, bf16_t* dq, long long C3, int q0,
                                            int T, float scale, int w, int lane, const float* xk_ds = nullptr,
                                            const float* xk_k = nullptr) {
    constexpr int DT = Geo<HS>::DT, SV = Geo<HS>::SV;
    constexpr bool SW = sw_ds<HS>();
    const int i = lane & 15, g = lane >> 4;
    // 2*DT output tiles over the NW waves; waves w and w+4 share a SIMD, so with NW = 7 and 8 tiles
    // the tile past the first seven goes to wave 3 (alone on its SIMD) rather than wave 0
    auto tile = [&](int jj) {
        const int dt = jj >> 1, u = jj & 1;
        // two accumulation chains (even / odd key blocks) halve the dependent-MFMA latency
        f32x4_t acc = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        auto fa = [&](int ks) { return frag_tr(Ks, SV, 32 * ks, 16 * dt, lane); };
        auto fb = [&](int ks) {
            if constexpr (SW) return frag_tr_ds(reinterpret_cast<const char*>(dSs), 32 * ks, 16 * u, lane);
            else return frag_tr(dSs, BWD_SDS, 32 * ks, 16 * u, lane);
        };
#if VIT_ATTN_BLA
        // operands of block ks + BLA requested before block ks's MFMA (the unpipelined form waited for
        // each block's four reads right in front of its MFMA: an LDS round trip per MFMA)
        constexpr int LA = VIT_ATTN_BLA < NSL ? VIT_ATTN_BLA : NSL;
        bf16x8_t ra[LA], rb[LA];
#pragma unroll
        for (int k = 0; k < LA; k++) {
            ra[k] = fa(k);
            rb[k] = fb(k);
        }
#pragma unroll
        for (int ks = 0; ks < NSL; ks++) {
            const bf16x8_t a = ra[ks % LA], b = rb[ks % LA];
            if (ks + LA < NSL) {
                ra[ks % LA] = fa(ks + LA);
                rb[ks % LA] = fb(ks + LA);
            }
            if (ks & 1) acc1 = mfma(a, b, acc1);
            else acc = mfma(a, b, acc);
        }
#else
#pragma unroll
        for (int ks = 0; ks < NSL; ks++) {
            const bf16x8_t a = fa(ks), b = fb(ks);
            if (ks & 1) acc1 = mfma(a, b, acc1);
            else acc = mfma(a, b, acc);
        }
#endif
        acc += acc1;
        // lane (i,g): d = 16dt + 4g + r, q = q0 + 16u + i (padded queries: dS = 0)
        const int q = q0 + 16 * u + i;
        if constexpr (XK) {
            const float e = xk_ds[16 * u + i];
#pragma unroll
            for (int r = 0; r < 4; r++) acc[r] += e * xk_k[16 * dt + 4 * g + r];
        }
        if constexpr (VIT_ATTN_DIAG & 2) asm volatile("" ::"v"(acc));
        else if (q < T) store4(dq + (long long)q * C3 + 16 * dt + 4 * g, acc, scale);
    };
    constexpr bool BAL = NW == 7 && 2 * DT == 8;  // one loop body (two inlined copies spill)
    const int jlast = BAL ? (w == 3 ? 7 : w) : 2 * DT - 1, jstep = BAL ? 4 : NW;
    for (int j = w; j <= jlast; j += jstep) tile(j);
}

// Σ over the 16 lanes of a DPP row of v[0..15], transposed: lane i of the row gets Σ_lanes v[i].
// Butterfly over the partners i ^ 15 (row_mirror), i ^ 7 (row_half_mirror), i ^ 2, i ^ 1 (quad_perm),
// each step keeping the half of the values selected by bit 3, 2, 1, 0 of i: 15 DPP adds instead of
// the 64 of sixteen row_sum16 reductions, and every lane ends up holding a result.
template <int CTRL>
__device__ __forceinline__ float dpp_c(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_transpose_sum16(const float (&v)[16], int i) {
    const bool b3 = i & 8, b2 = i & 4, b1 = i & 2, b0 = i & 1;
    float w[8], x[4], y[2];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = (b3 ? v[k + 8] : v[k]) + dpp_c<0x140>(b3 ? v[k] : v[k + 8]);
#pragma unroll
    for (int k = 0; k < 4; k++) x[k] = (b2 ? w[k + 4] : w[k]) + dpp_c<0x141>(b2 ? w[k] : w[k + 4]);
#pragma unroll
    for (int k = 0; k < 2; k++) y[k] = (b1 ? x[k + 2] : x[k]) + dpp_c<0x4E>(b1 ? x[k] : x[k + 2]);
    return (b0 ? y[1] : y[0]) + dpp_c<0xB1>(b0 ? y[0] : y[1]);
}

// end of an item: dK, dV of the wave's keys; the wave's column sums of dQ | dK | dV into its own
// partial row part[3 HS] (attn_colsum_reduce_k sums the rows: no barrier, no LDS).  The sums go
// through row_transpose_sum16, sixteen columns per reduction, each lane storing one column (at head
// size 64 three dword stores of 256 contiguous bytes); the row_sum16 form (4 DPP adds per column, the
// sum in lane 15, 4-B stores by 4 lanes) measured 5.3k + 1k cycles per item at ViT-B/16, 7.1k at
// ViT-H/14 (tools/attn_trace.py)
template <int HS, int KK = 2>
__device__ __forceinline__ void bwd_item_end(BwdRegs<HS, KK>& R, bf16_t* dq, long long C, int key0, int T, float scale,
                                             float* part, int lane, int it = 99) {
    constexpr int KS = Geo<HS>::KS, DT = Geo<HS>::DT;
    const int i = lane & 15, g = lane >> 4;
    [[maybe_unused]] const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // ATTN_STAMP
    const long long C3 = 3 * C;
#pragma unroll
    for (int kk = 0; kk < KK; kk++) {
        const int key = key0 + 16 * kk + i;
        if (key >= T || (VIT_ATTN_DIAG & 2)) continue;
        bf16_t* dst = dq + (long long)key * C3 + 4 * g;
#pragma unroll
        for (int dt = 0; dt < DT; dt++) {
            store4(dst + C + 16 * dt, R.dk[kk][dt], scale);
            store4(dst + 2 * C + 16 * dt, R.dv[kk][dt], 1.0f);
        }
    }
    ATTN_STAMP(8);
    if (!part) return;
    // dQ: lane (i,g) sums over the 4 g-groups' queries, then over its key column i
    float sd[KK];
#pragma unroll
    for (int kk = 0; kk < KK; kk++) {
        sd[kk] = R.sds[kk] + __shfl_xor(R.sds[kk], 16, 64);
        sd[kk] += __shfl_xor(sd[kk], 32, 64);
    }
    // per-lane values: dK / dV index 4 dt + r (d = 16 dt + 4 g + r); dQ index 8 s + j over the valid
    // (s, j) of the k-steps (the last one of HS % 32 == 16 has j < 4 only)
    constexpr int NKV = 4 * DT, NQ = 8 * KS - (Geo<HS>::HALF ? 4 : 0);
    constexpr int PKV = (NKV + 15) / 16 * 16, PQ = (NQ + 15) / 16 * 16;  // padded to whole reductions
    float vk[PKV], vv[PKV], vq[PQ];
#pragma unroll
    for (int k = 0; k < PKV; k++) vk[k] = vv[k] = 0.f;
#pragma unroll
    for (int k = 0; k < PQ; k++) vq[k] = 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; dt++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
#pragma unroll
            for (int kk = 0; kk < KK; kk++)
                if (key0 + 16 * kk + i < T) {
                    vk[4 * dt + r] += R.dk[kk][dt][r] * scale;
                    vv[4 * dt + r] += R.dv[kk][dt][r];
                }
        }
#pragma unroll
    for (int k = 0; k < NQ; k++) {
        const int s = k >> 3, j = k & 7;
        float t = 0.f;
#pragma unroll
        for (int kk = 0; kk < KK; kk++) t += sd[kk] * (float)R.kf[kk][s][j];
        vq[k] = t;
    }
    auto dq_col = [&](int k) {
        const int s = k >> 3, j = k & 7;
        return 32 * s + (j < 4 ? 4 * g + j : 16 + 4 * g + j - 4);
    };
    // sixteen values at a time: lane i of each DPP row gets the sum of value base + i
#pragma unroll
    for (int base = 0; base < PKV; base += 16) {
        float tk[16], tv[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            tk[k] = vk[base + k];
            tv[k] = vv[base + k];
        }
        const float sk = row_transpose_sum16(tk, i), sv = row_transpose_sum16(tv, i);
        const int k = base + i;
        if (k < NKV) {
            const int d = 16 * (k >> 2) + 4 * g + (k & 3);
            part[HS + d] = sk;
            part[2 * HS + d] = sv;
        }
    }
    ATTN_STAMP(9);
#pragma unroll
    for (int base = 0; base < PQ; base += 16) {
        float tq[16];
#pragma unroll
        for (int k = 0; k < 16; k++) tq[k] = vq[base + k];
        const float sq = row_transpose_sum16(tq, i);
        const int k = base + i;
        if (k < NQ) part[dq_col(k)] = sq * scale;
    }
    ATTN_STAMP(10);
}

// XK: T = TP + 1 (ViT-H/14, ViT-L/14 at 224^2: T = 257 = 8 x 32 + 1): the waves own keys 0 .. TP-1
// on the MFMA path, the queries run in TP/32 + 1 slices, and the last key is handled beside them on
// the VALU: per slice, 16 lanes per query form s = Q K[T-1] and dP = dO V[T-1] from the slice images
// (DPP row sums), dS = P (dP - delta) joins phase B's dQ as a rank-1 term, and 2 HS threads
// accumulate dK[T-1] = sum_q dS Q and dV[T-1] = sum_q P dO over the slices (fixed order)
template <int HS, int NKT, bool XK = false>
struct Bwd1 {
    static constexpr int TP = NKT * 16, NW = NKT / 2, NT = NW * 64, NSL = TP / 32;
    static constexpr int TPQ = TP + (XK ? 32 : 0), NSLQ = TPQ / 32;  // padded queries, query slices
    static constexpr int SK = slice_stride<HS>();  // Q / dO slices: row and transposed reads
    static constexpr int SV = Geo<HS>::SV;   // K image: transposed reads only
    static constexpr int SDS = sds_stride<HS>();
    static constexpr int K_OFF = 0;
    static constexpr int Q_OFF = K_OFF + TP * SV * 2;
    static constexpr int D_OFF = Q_OFF + 2 * 32 * SK * 2;
    static constexpr int S_OFF = D_OFF + 2 * 32 * SK * 2;
    static constexpr int L_OFF = S_OFF + TP * SDS * 2;
    static constexpr int X_OFF = L_OFF + 2 * TPQ * 4;  // XK: the slice's dS, P of key T-1; K, V rows of it
    static constexpr int BYTES = X_OFF + (XK ? (64 + 2 * HS) * 4 : 0);
    static constexpr int PER = (32 * Geo<HS>::CH + NT - 1) / NT;  // 16-B pieces per thread per slice operand
};
// LDS, and registers: up to 8 waves (2 per SIMD, 256 VGPRs) for HS <= 80; 4 waves for HS 96/128
// (more waves -> 3 per SIMD -> 168 VGPRs, which the 32-key accumulators do not fit)
template <int HS, int NKT>
constexpr bool bwd1_fits() {
    return Bwd1<HS, NKT>::BYTES <= 160 * 1024 && (NKT / 2 <= 4 || (NKT / 2 <= 8 && HS <= 80)) &&
           NKT / 2 <= ATTN_PART_ROWS;
}
// the XK form at NKT key tiles: the same register rule, LDS with the extra query slice
template <int HS, int NKT>
constexpr bool bwd1_fits_xk() {
    return Bwd1<HS, NKT, true>::BYTES <= 160 * 1024 && (NKT / 2 <= 4 || (NKT / 2 <= 8 && HS <= 80)) &&
           NKT / 2 + 1 <= ATTN_PART_ROWS && NKT / 2 * 64 >= 2 * HS;  // a thread per dK / dV output of the last key
}

template <int HS, int NKT, bool XK = false>
__global__ __launch_bounds__(NKT / 2 * 64, 1) void attn_bwd1_k(bf16_t* __restrict__ dqkv,
                                                               const bf16_t* __restrict__ dout,
                                                               const bf16_t* __restrict__ qkv,
                                                               const bf16_t* __restrict__ out,
                                                               const float* __restrict__ lse, int T,
                                                               int C, int NH, float* __restrict__ dsum) {
    using G = Geo<HS>;
    using Z = Bwd1<HS, NKT, XK>;
    constexpr int TP = Z::TP, NW = Z::NW, NT = Z::NT, NSL = Z::NSL, SK = Z::SK, SV = Z::SV;
    constexpr int TPQ = Z::TPQ, NSLQ = Z::NSLQ;
    constexpr int KS = G::KS, CH = G::CH, PER = Z::PER;
    __shared__ __attribute__((aligned(16))) char lds[Z::BYTES];
    bf16_t* Ks = reinterpret_cast<bf16_t*>(lds + Z::K_OFF);
    bf16_t* Qs = reinterpret_cast<bf16_t*>(lds + Z::Q_OFF);
    bf16_t* Ds = reinterpret_cast<bf16_t*>(lds + Z::D_OFF);
    bf16_t* dSs = reinterpret_cast<bf16_t*>(lds + Z::S_OFF);
    float* lse_s = reinterpret_cast<float*>(lds + Z::L_OFF);
    float* del_s = lse_s + TPQ;
    float* xds_s = reinterpret_cast<float*>(lds + Z::X_OFF);  // XK only: dS, P of key T-1 (32 each), K, V rows
    float* xp_s = xds_s + 32;
    float* xk_s = xp_s + 32;
    float* xv_s = xk_s + HS;
    const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
    const long long C3 = 3LL * C;
    const bf16_t* base = qkv + (long long)b * T * C3 + h * HS;
    const bf16_t* dbase = dout + (long long)b * T * C + h * HS;
    const bf16_t* obase = out + (long long)b * T * C + h * HS;
    bf16_t* dq = dqkv + (long long)b * T * C3 + h * HS;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = lane & 15;
    const int key0 = w * 32;
    [[maybe_unused]] int it = 15;  // ATTN_STAMP record: kernel-level stamps in record 15, slice sl in record sl
    ATTN_STAMP(0);
    BwdRegs<HS> R;
    // the wave's V fragments (rows >= T -> 0), requested first so their latency hides
#pragma unroll
    for (int kk = 0; kk < 2; kk++)
#pragma unroll
        for (int s = 0; s < KS; s++) R.vf[kk][s] = frag_glb<HS>(base + 2 * C, C3, key0 + 16 * kk + i, T, s, lane);
    // one slice (32 rows) of Q and dO: PER 16-B pieces per thread and operand
    uint4 pq[PER], pd[PER];
#ifndef VIT_ATTN_BWD1_BUF
#define VIT_ATTN_BWD1_BUF 1
#endif
#if VIT_ATTN_BWD1_BUF
    // buffer loads (rows >= T read 0, no "zero, then load if in range" merge), lanes past the last
    // piece repeating one (put_slice skips them), and only the waves that own a piece
    const auto rq_s = buf_rsrc(base, (uint32_t)(T * C3 * 2)), rd_s = buf_rsrc(dbase, (uint32_t)(T * C * 2));
    const bool slice_wave = __builtin_amdgcn_readfirstlane(w) * 64 < 32 * CH;  // a piece in the wave's first lane
    auto fetch_slice = [&](int q0) {
        if (!slice_wave) return;
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int idx = (j * NT + tid) % (32 * CH), t = idx / CH, c = idx - t * CH;
            const uint32_t r = (uint32_t)(q0 + t);
            pq[j] = buf_ld16(rq_s, r * (uint32_t)(C3 * 2) + 16 * c);
            pd[j] = buf_ld16(rd_s, r * (uint32_t)(C * 2) + 16 * c);
        }
    };
#else
    auto fetch_slice = [&](int q0) {
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int idx = j * NT + tid, t = idx / CH, c = idx - t * CH;
            pq[j] = pd[j] = make_uint4(0, 0, 0, 0);
            if (idx < 32 * CH && q0 + t < T) {
                pq[j] = *reinterpret_cast<const uint4*>(base + (long long)(q0 + t) * C3 + c * 8);
                pd[j] = *reinterpret_cast<const uint4*>(dbase + (long long)(q0 + t) * C + c * 8);
            }
        }
    };
#endif
    auto put_slice = [&](int buf) {
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int idx = j * NT + tid, t = idx / CH, c = idx - t * CH;
            if (idx < 32 * CH) {
                slice_put<HS>(Qs + buf * 32 * SK, t, c, pq[j]);
                slice_put<HS>(Ds + buf * 32 * SK, t, c, pd[j]);
            }
        }
    };
    fetch_slice(0);
    // lse and delta = rowsum(dO * O) for every query (padded queries: lse = +inf -> P = 0).  With one
    // query per thread their rows are requested here, before the K image's, so the prologue is one
    // memory round trip, not two (rows past T are clamped to row T-1 and their results dropped: no
    // branch around the loads)
#ifndef VIT_ATTN_BWD1_EARLY
#define VIT_ATTN_BWD1_EARLY 1
#endif
    constexpr bool EARLY = VIT_ATTN_BWD1_EARLY && TPQ <= NT;
    uint4 ov[EARLY ? CH : 1], dv[EARLY ? CH : 1];
    float ls_e = INFINITY;
    if constexpr (EARLY) {
        const int t = min(tid, T - 1);
#pragma unroll
        for (int cc = 0; cc < CH; cc++) {
            ov[cc] = *reinterpret_cast<const uint4*>(obase + (long long)t * C + cc * 8);
            dv[cc] = *reinterpret_cast<const uint4*>(dbase + (long long)t * C + cc * 8);
        }
        ls_e = lse[(long long)bh * T + t];
    }
    {
        bf16_t* const img[1] = {Ks};
        const int st[1] = {SV};
        const bf16_t* const src[1] = {base + C};
        const long long ld[1] = {C3};
        load_images<HS, TP, NT, 1>(img, st, src, ld, T);
    }
    put_slice(0);
    if constexpr (EARLY) {
        if (tid < TPQ) {
            float dl = 0.f;
#pragma unroll
            for (int cc = 0; cc < CH; cc++) dl += dot8_bf16(ov[cc], dv[cc]);
            lse_s[tid] = tid < T ? ls_e : INFINITY;
            del_s[tid] = tid < T ? dl : 0.f;
        }
    } else {
        for (int t = tid; t < TPQ; t += NT) {
            float dl = 0.f, ls = INFINITY;
            if (t < T) {
                ls = lse[(long long)bh * T + t];
#pragma unroll
                for (int cc = 0; cc < CH; cc++)
                    dl += dot8_bf16(*reinterpret_cast<const uint4*>(obase + (long long)t * C + cc * 8),
                                    *reinterpret_cast<const uint4*>(dbase + (long long)t * C + cc * 8));
            }
            lse_s[t] = ls;
            del_s[t] = dl;
        }
    }
    if constexpr (XK) {
        for (int d = tid; d < HS; d += NT) {
            xk_s[d] = bf2f(base[C + (long long)(T - 1) * C3 + d]);
            xv_s[d] = bf2f(base[2 * C + (long long)(T - 1) * C3 + d]);
        }
    }
    __syncthreads();
    // the wave's K fragments from the image (one global read of K per item, not two)
#pragma unroll
    for (int kk = 0; kk < 2; kk++)
#pragma unroll
        for (int s = 0; s < KS; s++) R.kf[kk][s] = frag_row<HS>(Ks, SV, key0 + 16 * kk, s, lane);
    float xacc = 0.f, xsds = 0.f;  // XK: this thread's dK / dV element of key T-1; sum of its dS
    [[maybe_unused]] const int xo = tid - (NT - 2 * HS);  // XK: that element's index (>= 0: the last 2 HS threads)
    // XK: the 8 dims 8p .. 8p+7 (p = tid & 15 < HS / 8) of key T-1's K and V rows, in registers for
    // the item: each query's s = q . k and dP = do . v is 16 lanes x one 16-B slice read
    float xkr[8], xvr[8];
    if constexpr (XK) {
        const int p8 = (tid & 15) * 8;
#pragma unroll
        for (int e = 0; e < 8; e++) {
            xkr[e] = p8 < HS ? xk_s[p8 + e] : 0.f;
            xvr[e] = p8 < HS ? xv_s[p8 + e] : 0.f;
        }
    }
    const float scale = 1.0f / sqrtf((float)HS);
    const float c = LOG2E * scale;
    R.zero();
    ATTN_STAMP(1);
#pragma unroll 1
    for (int sl = 0; sl < NSLQ; sl++) {
        const int q0 = sl * 32, cur = sl & 1;
        it = sl;
        ATTN_STAMP(0);
        if (sl + 1 < NSLQ) fetch_slice(q0 + 32);  // lands in registers during phase A
        bwd_slice_a<HS>(R, Qs + cur * 32 * SK, Ds + cur * 32 * SK, lse_s + q0, del_s + q0, dSs + key0 * Z::SDS, c, lane);
        ATTN_STAMP(1);
        if constexpr (XK) {  // key T-1 against the slice's 32 queries: 16 lanes per query
            const bf16_t* Qc = Qs + cur * 32 * SK;
            const bf16_t* Dc = Ds + cur * 32 * SK;
            for (int idx = tid; idx < 512; idx += NT) {
                const int j = idx >> 4, part = idx & 15;  // part == tid & 15 (NT % 16 == 0)
                float sq = 0.f, dp = 0.f;
                if (part * 8 < HS) {
                    const uint4 qv = slice_chunk8<HS>(Qc, j, part), dv = slice_chunk8<HS>(Dc, j, part);
                    const uint32_t qw[4] = {qv.x, qv.y, qv.z, qv.w}, dw[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        sq += __uint_as_float(qw[e] << 16) * xkr[2 * e] + __uint_as_float(qw[e] & 0xffff0000u) * xkr[2 * e + 1];
                        dp += __uint_as_float(dw[e] << 16) * xvr[2 * e] + __uint_as_float(dw[e] & 0xffff0000u) * xvr[2 * e + 1];
                    }
                }
                sq = row_sum16(sq);
                dp = row_sum16(dp);
                if (part == 15) {
                    const float p = q0 + j < T ? fexp2(sq * c - lse_s[q0 + j]) : 0.f;
                    xds_s[j] = p * (dp - del_s[q0 + j]);
                    xp_s[j] = p;
                }
            }
        }
        __syncthreads();
        ATTN_STAMP(2);
        if constexpr (XK) {
            // the last 2 HS threads (waves 5-7 at 8 waves): waves 0-4 carry put_slice's pieces and
            // waves 0-1 phase B's two extra dQ tiles, so these run beside them instead of after them
            if (xo >= 0) {
                const bf16_t* img = (xo < HS ? Qs : Ds) + cur * 32 * SK;
                const float* wv = xo < HS ? xds_s : xp_s;
                const int d = xo < HS ? xo : xo - HS;
#pragma unroll 8
                for (int j = 0; j < 32; j++) {
                    xacc += wv[j] * slice_at<HS>(img, j, d);
                    xsds += xds_s[j];
                }
            }
        }
        if (sl + 1 < NSLQ) put_slice(cur ^ 1);  // its buffer was last read in the previous slice
#ifndef VIT_ATTN_BWD1_VMWAIT
#define VIT_ATTN_BWD1_VMWAIT 1
#endif
        // every wave, every slice: the fetch's loads are complete here (put_slice waited for them on the
        // owning waves; the others issued none).  Without a wait hipcc sees on every path, it kept
        // the loads possibly pending on the non-owner path and waited vmcnt(0) before the next
        // fetch — after phase B's dQ stores, so every slice waited for its own stores to complete
        if constexpr (VIT_ATTN_BWD1_VMWAIT) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) only
        ATTN_STAMP(3);
        bwd_slice_b<HS, NSL, NW, XK>(Ks, dSs, dq, C3, q0, T, scale, w, lane, xds_s, xk_s);
        ATTN_STAMP(4);
        __syncthreads();
        ATTN_STAMP(5);
    }
    it = 15;
    ATTN_STAMP(6);
    // per-wave column-sum rows: dsum[((b NWR + w) NH + h)][3 HS], NWR = NW (+ 1: the last key's row, XK)
    constexpr int NWR = NW + (XK ? 1 : 0);
    bwd_item_end<HS>(R, dq, C, key0, T, scale,
                     dsum ? dsum + ((long long)(b * NWR + w) * NH + h) * 3 * HS : nullptr, lane, it);
    ATTN_STAMP(7);
    if constexpr (XK) {  // key T-1's dK, dV and its column-sum row (index NW of the item)
        if (xo >= 0) {
            const int o = xo, d = o < HS ? o : o - HS;
            const float v = o < HS ? xacc * scale : xacc;
            dq[(long long)(T - 1) * C3 + (o < HS ? C : 2 * C) + d] = f2bf(v);
            if (dsum) {
                float* row = dsum + ((long long)(b * NWR + NW) * NH + h) * 3 * HS;
                row[(o < HS ? HS : 2 * HS) + d] = v;
                if (o < HS) row[d] = scale * xsds * xk_s[d];
            }
        }
    }
}

template <int HS, int NKT, int KK = 2>
// VIT_ATTN_SKEW: the persistent backward runs phase B of slice s-1 right after phase A of slice s
// (dS^T double-buffered), one barrier per slice instead of two, so the two phases' MFMA, VALU and
// LDS work share one barrier interval
#ifndef VIT_ATTN_SKEW
#define VIT_ATTN_SKEW 1
#endif

struct Bwdp {
    using G = Geo<HS>;
    static constexpr int TP = NKT * 16, NW = NKT / KK, NT = NW * 64, NSL = TP / 32, CH = G::CH;
    static constexpr int SK = G::SK, SV = G::SV, SL = slice_stride<HS>(), SDS = sds_stride<HS>();
    static constexpr int K_OFF = 0;                          // K images [2][TP][SV]: current / next item
    static constexpr int V_OFF = K_OFF + 2 * TP * SV * 2;    // next item's V rows [TP][SK]
    static constexpr int Q_OFF = V_OFF + TP * SK * 2;        // Q slices [2][32][SL]
    static constexpr int D_OFF = Q_OFF + 2 * 32 * SL * 2;    // dO slices [2][32][SL]
    static constexpr int NDS = VIT_ATTN_SKEW ? 2 : 1;       // dS^T buffers
    static constexpr int S_OFF = D_OFF + 2 * 32 * SL * 2;    // dS^T [NDS][TP][SDS]
    static constexpr int L_OFF = S_OFF + NDS * TP * SDS * 2; // lse [2][TP] (item parity)
    static constexpr int E_OFF = L_OFF + 2 * TP * 4;         // delta [2][32] (slice parity)
    static constexpr int BYTES = E_OFF + 2 * 32 * 4;
    static constexpr int PER = (32 * CH + NT - 1) / NT;      // 16-B pieces per thread, slice operand
    static constexpr int PERS = (2 * 32 * CH + NT - 1) / NT; // next item's K + V rows, per slice
};
// the delta reduction runs over CH consecutive lanes (a power of two dividing 64).  KK = 2: 32 keys
// per wave, up to 8 waves (bwd1's register rule).  KK = 1 (16 keys per wave, twice the waves and
// the LDS reads, <= 128 VGPRs) measured 377 vs 296 us at ViT-B/16 (spills; LDS-bound): not launched.
template <int HS, int NKT, int KK = 2>
constexpr bool bwdp_fits() {
    using Z = Bwdp<HS, NKT, KK>;
    return Z::BYTES <= 160 * 1024 && (64 % Geo<HS>::CH) == 0 && HS <= 64 && Z::NW <= ATTN_PART_ROWS &&
           NKT % KK == 0 && (KK == 2 ? bwd1_fits<HS, NKT>() : KK == 4 ? (HS == 64 && Z::NW <= 4) : Z::NW <= 16);
}

template <int HS, int NKT, int KK>
__global__ __launch_bounds__(NKT / KK * 64, 1) void attn_bwdp_k(bf16_t* __restrict__ dqkv,
                                                               const bf16_t* __restrict__ dout,
                                                               const bf16_t* __restrict__ qkv,
                                                               const bf16_t* __restrict__ out,
                                                               const float* __restrict__ lse, int T,
                                                               int C, int NH, int BH, float* __restrict__ dsum,
                                                               int stagger) {
    using G = Geo<HS>;
    using Z = Bwdp<HS, NKT, KK>;
    // stagger (100 MHz ticks, VIT_ATTN_STAGGER): every other CU of each XCD starts that much later, so
    // the CUs' items do not all end (dK / dV store burst) at the same moment.  Measured (VERDICT r05
    // item 3, B/16, two rounds): 0: 239.5 / 245.0 us, 400: 245.8 / 240.6, 870 (half an item): 248.0 /
    // 248.0, 1300: 253.3 / 247.3 -- no gain (profiles/r06_attn_bwd_stagger.txt), so 0
    if (stagger > 0 && ((blockIdx.x >> 3) & 1)) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)stagger) __builtin_amdgcn_s_sleep(8);
    }
    constexpr int TP = Z::TP, NW = Z::NW, NT = Z::NT, NSL = Z::NSL, SK = Z::SK, SV = Z::SV, SL = Z::SL;
    static_assert((32 * G::CH) % 64 == 0 && NT % 64 == 0, "slice pieces are whole waves");
    constexpr int KS = G::KS, CH = G::CH, PER = Z::PER, PERS = Z::PERS;
    __shared__ __attribute__((aligned(16))) char lds[Z::BYTES];
    bf16_t* Kimg = reinterpret_cast<bf16_t*>(lds + Z::K_OFF);
    bf16_t* Vst = reinterpret_cast<bf16_t*>(lds + Z::V_OFF);
    bf16_t* Qs = reinterpret_cast<bf16_t*>(lds + Z::Q_OFF);
    bf16_t* Ds = reinterpret_cast<bf16_t*>(lds + Z::D_OFF);
    bf16_t* dSs = reinterpret_cast<bf16_t*>(lds + Z::S_OFF);
    float* lse_s = reinterpret_cast<float*>(lds + Z::L_OFF);
    float* del_s = reinterpret_cast<float*>(lds + Z::E_OFF);
    const long long C3 = 3LL * C;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int key0 = w * 16 * KK;
    // the waves that own a slice piece (PER = 1: the first 32 CH / 64); the others would fetch and
    // store duplicates (VIT_ATTN_SLICE_ALL=1: every wave does, the pre-r05 form)
#ifndef VIT_ATTN_SLICE_ALL
#define VIT_ATTN_SLICE_ALL 0
#endif
    constexpr bool SPLIT_SLICE = !VIT_ATTN_SLICE_ALL && Bwdp<HS, NKT, KK>::PER == 1 && (32 * G::CH) % 64 == 0;
    const bool slice_wave = !SPLIT_SLICE || w < 32 * G::CH / 64;
    const float scale = 1.0f / sqrtf((float)HS);
    const float c = LOG2E * scale;
    auto qkv_of = [&](int bh) { return qkv + (long long)(bh / NH) * T * C3 + (bh % NH) * HS; };
    auto row_of = [&](const bf16_t* p, int bh) { return p + (long long)(bh / NH) * T * C + (bh % NH) * HS; };
    // slice rows (Q, dO, O) of item bh at q0 -> registers; into LDS with delta = rowsum(dO * O)
    uint4 pq[PER], pd[PER], po[PER];
    // Buffer loads: rows >= T read 0 without a branch.  No branch around any prefetch either: lanes
    // past the last piece repeat a piece (same bytes to the same LDS address), so the compiler sees
    // every prefetch register consumed on every path and never drains vmcnt to re-use one.
    struct Src { __amdgpu_buffer_rsrc_t q, d, o, kv, l; };  // an item's buffer descriptors
    auto src_of = [&](int bh) {
        Src r;
        r.q = buf_rsrc(qkv_of(bh), (uint32_t)(T * C3 * 2));
        r.d = buf_rsrc(row_of(dout, bh), (uint32_t)(T * C * 2));
        r.o = buf_rsrc(row_of(out, bh), (uint32_t)(T * C * 2));
        // K | V columns from K's first column: every byte of rows >= T is past the end
        r.kv = buf_rsrc(qkv_of(bh) + C, (uint32_t)(T * C3 * 2 - 2 * C));
        r.l = buf_rsrc(lse + (long long)bh * T, (uint32_t)(T * 4));
        return r;
    };
    auto fetch_slice = [&](const Src& sr, int q0) {
        const auto rq = sr.q, rd = sr.d, ro = sr.o;
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int idx = (j * NT + tid) % (32 * CH), t = idx / CH, cc = idx - t * CH;
            const uint32_t r = (uint32_t)(q0 + t);
            pq[j] = buf_ld16(rq, r * (uint32_t)(C3 * 2) + 16 * cc);
            pd[j] = buf_ld16(rd, r * (uint32_t)(C * 2) + 16 * cc);
            po[j] = buf_ld16(ro, r * (uint32_t)(C * 2) + 16 * cc);
        }
    };
    auto put_slice = [&](int buf) {
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int idx = (j * NT + tid) % (32 * CH), t = idx / CH, cc = idx - t * CH;
            float dl = dot8_bf16(po[j], pd[j]);  // the CH lanes of row t are consecutive
#pragma unroll
            for (int o = 1; o < CH; o <<= 1) dl += __shfl_xor(dl, o, 64);
            slice_put<HS>(Qs + buf * 32 * SL, t, cc, pq[j]);
            slice_put<HS>(Ds + buf * 32 * SL, t, cc, pd[j]);
            if (cc == 0) del_s[buf * 32 + t] = dl;
        }
    };
    // next item's K and V rows [32 rb, 32 rb + 32) -> registers; into its K image / the V rows
    uint4 ps[PERS];
    float lse_n = INFINITY;
    auto fetch_side = [&](const Src& sr, int rb) {
        const auto rk = sr.kv;
#pragma unroll
        for (int j = 0; j < PERS; j++) {
            const int idx = (j * NT + tid) % (64 * CH), op = idx >= 32 * CH, rem = idx - op * 32 * CH, t = rem / CH,
                      cc = rem - t * CH, row = 32 * rb + t;
            ps[j] = buf_ld16(rk, (uint32_t)row * (uint32_t)(C3 * 2) + (uint32_t)(op * C * 2) + 16 * cc);
        }
    };
    auto put_side = [&](int kbuf, int rb) {
#pragma unroll
        for (int j = 0; j < PERS; j++) {
            const int idx = (j * NT + tid) % (64 * CH), op = idx >= 32 * CH, rem = idx - op * 32 * CH, t = rem / CH,
                      cc = rem - t * CH, row = 32 * rb + t;
            bf16_t* dst = op ? Vst + row * SK : Kimg + kbuf * TP * SV + row * SV;
            *reinterpret_cast<uint4*>(dst + cc * 8) = ps[j];
        }
    };
    auto load_kv = [&](BwdRegs<HS, KK>& R, int kbuf) {  // the wave's fragments from the staged rows
#pragma unroll
        for (int kk = 0; kk < KK; kk++)
#pragma unroll
            for (int s = 0; s < KS; s++) {
                R.kf[kk][s] = frag_row<HS>(Kimg + kbuf * TP * SV, SV, key0 + 16 * kk, s, lane);
                R.vf[kk][s] = frag_row<HS>(Vst, SK, key0 + 16 * kk, s, lane);
            }
    };
    int bh = blockIdx.x;
    if (bh >= BH) return;
    // (measured, not kept: s_setprio 1 for waves 4-6, 263.6 vs 254.5 us — their phase A sped up by what
    // waves 0-2's slowed down; waves 4-6 running phase B before phase A, 262 us: the SIMD's issue is
    // shared, not idle)
    // prologue (first item): K image, V rows, lse, slice 0 — one blocking round trip
    fetch_slice(src_of(bh), 0);
    {
        bf16_t* const img[2] = {Kimg, Vst};
        const int st[2] = {SV, SK};
        const bf16_t* const src[2] = {qkv_of(bh) + C, qkv_of(bh) + 2 * C};
        const long long ld[2] = {C3, C3};
        load_images<HS, TP, NT, 2>(img, st, src, ld, T);
    }
    for (int t = tid; t < TP; t += NT) lse_s[t] = t < T ? lse[(long long)bh * T + t] : INFINITY;
    put_slice(0);
    if constexpr ((VIT_ATTN_DIAG & 1) != 0) fetch_side(src_of(bh), 0);
    __syncthreads();
    BwdRegs<HS, KK> R;
    load_kv(R, 0);
    int kb = 0, it = 0;
#pragma unroll 1
    for (int n = 0; bh < BH; n++, bh += gridDim.x) {
        const int bhn = bh + gridDim.x;
        const bool has_next = bhn < BH;
        const int bhc = has_next ? bhn : bh;  // the next item, or this one again after the last
        const Src s_cur = src_of(bh), s_nxt = src_of(bhc);
        bf16_t* dq = dqkv + (long long)(bh / NH) * T * C3 + (bh % NH) * HS;
        const float* lse_cur = lse_s + (n & 1) * TP;
        R.zero();
#pragma unroll 1
        for (int sl = 0; sl < NSL; sl++, it++) {
            const int cur = it & 1, q0 = sl * 32;
            ATTN_STAMP(0);
            // one step ahead: the next slice (this item's or the next item's first), the next
            // item's K / V row block sl and, with its first block, its lse
            // (unconditional: past the last item / slice a valid item is re-read into buffers no one
            // reads again, so the compiler sees every prefetch register consumed on every path and
            // does not drain vmcnt before re-using them)
            if constexpr (!(VIT_ATTN_DIAG & 1)) {
                if (slice_wave) {
                    if (sl + 1 < NSL) fetch_slice(s_cur, q0 + 32);
                    else fetch_slice(s_nxt, 0);
                }
                fetch_side(s_nxt, sl);
                // unconditional load (past T: 0); padded keys get +inf when it is put
                if (sl == 0) lse_n = buf_ldf(s_nxt.l, 4 * tid);
            }
            if constexpr (VIT_ATTN_SKEW) {
                // A(sl) -> dS^T buffer sl&1; B(sl-1) from buffer (sl-1)&1 (complete since the last
                // barrier); the slice buffers cur^1 were last read by A(sl-1), before that barrier
                bf16_t* dS_a = dSs + (sl & 1) * TP * Z::SDS;
                bwd_slice_a<HS, KK>(R, Qs + cur * 32 * SL, Ds + cur * 32 * SL, lse_cur + q0, del_s + cur * 32,
                                    dS_a + key0 * Z::SDS, c, lane);
                ATTN_STAMP(1);
                if (sl > 0)
                    bwd_slice_b<HS, NSL, NW>(Kimg + kb * TP * SV, dSs + ((sl - 1) & 1) * TP * Z::SDS, dq, C3,
                                             q0 - 32, T, scale, w, lane);
                ATTN_STAMP(2);
                if (slice_wave) put_slice(cur ^ 1);
                if (sl == 0 && tid < TP) lse_s[((n + 1) & 1) * TP + tid] = tid < T ? lse_n : INFINITY;
                ATTN_STAMP(3);
                __syncthreads();
                ATTN_STAMP(4);
                // the next item's K image / V rows: after the barrier, so every wave has finished
                // this item's load_kv reads of the V rows (item start) before any block is replaced
                put_side(kb ^ 1, sl);
                ATTN_STAMP(5);
            } else {
                bwd_slice_a<HS, KK>(R, Qs + cur * 32 * SL, Ds + cur * 32 * SL, lse_cur + q0, del_s + cur * 32,
                                    dSs + key0 * Z::SDS, c, lane);
                __syncthreads();
                // buffers written here were last read before the barrier above (slice buffer cur^1 by
                // the previous slice, the idle K image by the previous item, the V rows by load_kv)
                put_slice(cur ^ 1);
                put_side(kb ^ 1, sl);
                if (sl == 0 && tid < TP) lse_s[((n + 1) & 1) * TP + tid] = tid < T ? lse_n : INFINITY;
                bwd_slice_b<HS, NSL, NW>(Kimg + kb * TP * SV, dSs, dq, C3, q0, T, scale, w, lane);
                __syncthreads();
            }
        }
        if constexpr (VIT_ATTN_SKEW) {  // the item's last phase B; the barrier also publishes the last put_side
            bwd_slice_b<HS, NSL, NW>(Kimg + kb * TP * SV, dSs + ((NSL - 1) & 1) * TP * Z::SDS, dq, C3,
                                     (NSL - 1) * 32, T, scale, w, lane);
            __syncthreads();
        }
        ATTN_STAMP(6);
        bwd_item_end<HS, KK>(R, dq, C, key0, T, scale,
                             dsum ? dsum + ((long long)((bh / NH) * NW + w) * NH + bh % NH) * 3 * HS : nullptr, lane,
                             it);
        ATTN_STAMP(7);
        if (has_next) {
            kb ^= 1;
            load_kv(R, kb);  // every block was put before the item's last barrier
        }
    }
}

// largest padded length (multiple of 32) whose forward AND backward images fit the 160 KiB LDS
template <int HS>
constexpr int max_tp() {
    int tp = 32;
    while (tp + 32 <= 320 && (tp + 32) * (Geo<HS>::SK + Geo<HS>::SV) * 2 <= 160 * 1024 &&
           2 * (tp + 32) * Geo<HS>::SK * 2 + 2 * (tp + 32) * 4 + 8 * HS * 4 <= 160 * 1024)
        tp += 32;
    return tp;
}

// launchers over the key-tile count (NKT = 2, 4, ..., 2*max_tp/32)
template <int HS, int NKT>
bool launch_fwd(bf16_t* out, float* lse, const bf16_t* qkv, int B, int T, int C, int NH, hipStream_t s) {
    if (T > NKT * 16 || T <= (NKT - 2) * 16) return false;  // the kernel masks keys in its last score tile only
#ifndef VIT_ATTN_FWD_TRIM
#define VIT_ATTN_FWD_TRIM 1
#endif
    if (VIT_ATTN_FWD_TRIM && (NKT - 1) * 16 >= T)
        attn_fwd_k<HS, NKT, NKT - 1><<<B * NH, 256, 0, s>>>(out, lse, qkv, T, C, NH);
    else
        attn_fwd_k<HS, NKT><<<B * NH, 256, 0, s>>>(out, lse, qkv, T, C, NH);
    count_hit(VIT_HIT_ATTN_FWD_MFMA);
    return true;
}
int attn_bwd_variant();  // attention.hip: VIT_ATTN_BWD = pair | one | (default) persistent (A/B)
int attn_cu_count();     // attention.hip: compute units of the current device
// returns the column-sum partial rows written per (b,h) (attn_colsum_reduce_k sums B x rows)
template <int HS, int NKT>
int launch_bwd(bf16_t* dqkv, const bf16_t* dout, const bf16_t* qkv, const bf16_t* out, const float* lse, int B,
               int T, int C, int NH, float* part, hipStream_t s) {
    const int v = attn_bwd_variant(), BH = B * NH;
    // "p4": the persistent one-pass kernel with 64 keys per wave (4 waves, one per SIMD, up to 512
    // registers each; keys padded to a multiple of 64): measured slower than the default 32 keys per
    // wave (338 vs 289 us at ViT-B/16 B=256: one wave per SIMD hides no latency)
    constexpr int NK4 = (NKT + 7) / 8 * 8;
    if constexpr (bwdp_fits<HS, NK4, 4>()) {
        if (v == 4) {
            attn_bwdp_k<HS, NK4, 4><<<std::min(BH, attn_cu_count()), NK4 / 4 * 64, 0, s>>>(dqkv, dout, qkv, out, lse,
                                                                                          T, C, NH, BH, part, 0);
            count_hit(VIT_HIT_ATTN_BWD_PERSISTENT);
            return NK4 / 4;
        }
    }
    if constexpr (bwdp_fits<HS, NKT, 2>()) {
        if (v == 0) {
            static const int stagger = [] {
                const char* e = getenv("VIT_ATTN_STAGGER");
                return e ? atoi(e) : 0;
            }();
            attn_bwdp_k<HS, NKT, 2><<<std::min(BH, attn_cu_count()), NKT / 2 * 64, 0, s>>>(dqkv, dout, qkv, out, lse,
                                                                                         T, C, NH, BH, part, stagger);
            count_hit(VIT_HIT_ATTN_BWD_PERSISTENT);
            return NKT / 2;
        }
    }
    if constexpr (bwd1_fits<HS, NKT>()) {
        if (v != 2) {
            attn_bwd1_k<HS, NKT><<<BH, NKT / 2 * 64, 0, s>>>(dqkv, dout, qkv, out, lse, T, C, NH, part);
            count_hit(VIT_HIT_ATTN_BWD_ONEPASS);
            return NKT / 2;
        }
    }
    // T = 32k + 1 (ViT-H/14, ViT-L/14 at 224^2: T = 257): the one-pass kernel over the first T-1 keys
    // (NKT - 2 tiles) and all queries, the last key on its VALU side path (XK)
    if constexpr (NKT > 2 && bwd1_fits_xk<HS, NKT - 2>()) {
        if (v != 2 && T == (NKT - 2) * 16 + 1) {
            constexpr int NW = (NKT - 2) / 2;
            attn_bwd1_k<HS, NKT - 2, true><<<BH, NW * 64, 0, s>>>(dqkv, dout, qkv, out, lse, T, C, NH, part);
            count_hit(VIT_HIT_ATTN_BWD_XKEY);
            return NW + 1;
        }
    }
    attn_bwd_pair_k<HS, NKT><<<2 * cdiv(BH, 8) * 8, 256, 0, s>>>(dqkv, dout, qkv, out, lse, T, C, NH, BH, part);
    count_hit(VIT_HIT_ATTN_BWD_PAIR);
    return 1;
}
template <int HS, int NKT = 2>
bool dispatch_fwd(int nkt, bf16_t* out, float* lse, const bf16_t* qkv, int B, int T, int C, int NH,
                  hipStream_t s) {
    if constexpr (NKT * 16 > max_tp<HS>()) {
        return false;
    } else {
        if (nkt == NKT) return launch_fwd<HS, NKT>(out, lse, qkv, B, T, C, NH, s);
        return dispatch_fwd<HS, NKT + 2>(nkt, out, lse, qkv, B, T, C, NH, s);
    }
}
template <int HS, int NKT = 2>
int dispatch_bwd(int nkt, bf16_t* dqkv, const bf16_t* dout, const bf16_t* qkv, const bf16_t* out,
                 const float* lse, int B, int T, int C, int NH, float* part, hipStream_t s) {
    if constexpr (NKT * 16 > max_tp<HS>()) {
        return 0;
    } else {
        if (nkt == NKT) return launch_bwd<HS, NKT>(dqkv, dout, qkv, out, lse, B, T, C, NH, part, s);
        return dispatch_bwd<HS, NKT + 2>(nkt, dqkv, dout, qkv, out, lse, B, T, C, NH, part, s);
    }
}

}  // namespace fa

// per-head-size entry points (attn_h*.hip); false = shape outside the instantiated range
#define VIT_FA_DECLARE(HS)                                                                         \
    bool fa_forward_h##HS(bf16_t* out, float* lse, const bf16_t* qkv, int B, int T, int C, int NH, \
                          hipStream_t s);                                                          \
    int fa_backward_h##HS(bf16_t* dqkv, const bf16_t* dout, const bf16_t* qkv, const bf16_t* out, \
                          const float* lse, int B, int T, int C, int NH, float* part, hipStream_t s); \
    int fa_max_t_h##HS();
VIT_FA_DECLARE(32)
VIT_FA_DECLARE(64)
VIT_FA_DECLARE(80)
VIT_FA_DECLARE(96)
VIT_FA_DECLARE(128)

#define VIT_FA_DEFINE(HS)                                                                           \
    bool fa_forward_h##HS(bf16_t* out, float* lse, const bf16_t* qkv, int B, int T, int C, int NH,  \
                          hipStream_t s) {                                                          \
        return fa::dispatch_fwd<HS>(cdiv(T, 32) * 2, out, lse, qkv, B, T, C, NH, s);                \
    }                                                                                               \
    int fa_backward_h##HS(bf16_t* dqkv, const bf16_t* dout, const bf16_t* qkv, const bf16_t* out,   \
                          const float* lse, int B, int T, int C, int NH, float* part, hipStream_t s) { \
        return fa::dispatch_bwd<HS>(cdiv(T, 32) * 2, dqkv, dout, qkv, out, lse, B, T, C, NH, part, s); \
    }                                                                                               \
    int fa_max_t_h##HS() { return fa::max_tp<HS>(); }

}  // namespace vit
