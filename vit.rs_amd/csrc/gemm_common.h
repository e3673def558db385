// gemm_common.h — launch parameters, XCD / split-K tile mapping and the fused epilogues shared
// by the bf16 GEMM engines (gemm.hip) and the fp8 engine (gemm_fp8.hip).
#pragma once
#include "gemm.h"

namespace vit {

struct GemmParams {
    const void* A;
    const void* B;
    void* C;
    void* C2;
    const void* aux;
    const float* bias;
    float* dbias;
    float* colsum_out;  // partial rows [cdiv(M,128)][N] of the aux epilogues' column sums (stored)
    long long lda, ldb, ldc, ldaux;
    int M, N, K;
    int kchunk;  // K range per split (multiple of the K tile)
    int no_epi;  // diagnostic (gemm_bf16_set_debug): skip the epilogue, keep the accumulators live
    int dbg;     // diagnostic flags (gemm_bf16_set_debug & 0xF0): 16 = persistent engine drains its
                 // epilogue stores (vmcnt(0)) before the next tile's main loop
    int stagger;  // two-per-CU engines: first-round delay (100 MHz ticks) of the CU's second workgroup
    unsigned long long* trace;  // diagnostic: [workgroup][4] start, main-loop end, end, hw id
    int tiles;   // output tiles of the launch (the grid is tiles x K-splits)
    int gm;      // persistent engine tile order: groups of gm row panels, column-major inside a group
                 // (0: row-major; VIT_GEMM_GM)
    uint8_t* mx_q;  // fused MX output (GemmArgs::mx_q / mx_s); mx_rg = padded rows / 32
    uint8_t* mx_s;
    int mx_rg;
    uint8_t* mxc_q;  // fused column-wise MX output (GemmArgs::mxc_*); mxc_rg = padded N / 32
    uint8_t* mxc_s;
    long long mxc_ld;
    int mxc_off, mxc_rg;
    // persistent engine with a split tail (variant 10): the last, partly filled round's tiles run as
    // tsplit K-ranges of kchunk each into fp32 partial tiles tpart[tile][part][256][256]; tfull = the
    // tiles of the full rounds (gemm_tail_fix_k finishes the tail tiles)
    int tsplit, tfull;
    float* tpart;
};

// E8M0 scale byte of an MX block: X + 127 with X = ceil(log2(amax / 448)) (no element overflows
// e4m3's 448), clamped to [0, 254]; 127 (scale 1) for an all-zero block
__device__ __forceinline__ int mx_scale_byte(float amax) {
    if (!(amax > 0.f)) return 127;
    const uint32_t u = __float_as_uint(amax);
    const int e = (int)((u >> 23) & 0xff), mant = (int)(u & 0x7fffff);
    int s = e - 8 + (mant > 0x600000 ? 1 : 0);
    return s < 0 ? 0 : (s > 254 ? 254 : s);
}
// the MX copy of 8 bf16 output values (packed as stored) at row m, columns n..n+7: the 4 lanes of
// a 32-column block (lane bits 0-1 in the staged layout) share one scale
__device__ __forceinline__ void mx_out8(const GemmParams& p, int m, int n, uint32_t w0, uint32_t w1, uint32_t w2,
                                        uint32_t w3, int lane) {
    const uint32_t w[4] = {w0, w1, w2, w3};
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; e++) {
        v[2 * e] = __uint_as_float(w[e] << 16);
        v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
    }
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 8; j++) amax = fmaxf(amax, fabsf(v[j]));
    amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
    amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
    const int sb = mx_scale_byte(amax);
    if ((lane & 3) == 0) {
        const int kb = n >> 5;
        p.mx_s[((long long)(kb >> 1) * p.mx_rg + (m >> 5)) * 64 + (kb & 1) * 32 + (m & 31)] = (uint8_t)sb;
    }
    const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);  // 2^(127 - sb), exact
    int t0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, 0, false);
    t0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, t0, true);
    int t1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, 0, false);
    t1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, t1, true);
    *reinterpret_cast<uint2*>(p.mx_q + (long long)m * p.N + n) = make_uint2((uint32_t)t0, (uint32_t)t1);
}

// the 8 bf16 values (packed as stored) back into the wave's staging rows as fp32, for the
// column-wise MX pass (mx_cols_pass)
__device__ __forceinline__ void stage_back8(float* w, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<f4*>(w) = f4{__uint_as_float(w0 << 16), __uint_as_float(w0 & 0xffff0000u),
                                   __uint_as_float(w1 << 16), __uint_as_float(w1 & 0xffff0000u)};
    *reinterpret_cast<f4*>(w + 4) = f4{__uint_as_float(w2 << 16), __uint_as_float(w2 & 0xffff0000u),
                                       __uint_as_float(w3 << 16), __uint_as_float(w3 & 0xffff0000u)};
}

// host: the partial-row buffer of an aux epilogue's column sums (colsum_part or the thread
// workspace; nullptr when the GEMM sums no columns) and the fixed-order add into colsum_out
float* colsum_rows_begin(const GemmArgs& a);
void colsum_rows_end(const GemmArgs& a, float* rows, hipStream_t s);
// host, split-K of the one-workgroup-per-CU engines (gemm.hip): the split count for `tiles` output
// tiles over nk K-steps; the fp32 slab workspace of `split` partial planes (a.ws or the thread
// workspace; nullptr + error when neither fits); C += sum of the slabs in a fixed order
int choose_split_waves(int tiles, int nk);
float* slab_buffer(const GemmArgs& a, int split);
void slab_reduce(const GemmArgs& a, float* slab, int split, hipStream_t s);

// (tile, K-split) of this workgroup.  Workgroups are dealt round-robin over the 8 XCDs in
// linear-id order (x fastest), so the XCD-aware remap runs over the whole (split, tile) grid: the
// ~1/8 of the grid on one XCD is a contiguous range of the same K-split's tiles, which share
// their A and B K-slices in that XCD's L2 (split-K wgrad launches have tiles x splits blocks).
__device__ __forceinline__ void split_remap(int tiles, int& tile, int& split) {
    const int nwg = gridDim.x * gridDim.y;
    const int l = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, nwg);
    split = l / tiles;
    tile = l - split * tiles;
}
__device__ __forceinline__ int split_index(int tiles) {
    int t, s;
    split_remap(tiles, t, s);
    return s;
}

// epilogue 16-B global access
typedef unsigned int epi_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void epi_st16(const GemmParams&, void* q, epi_u32x4 v) {
    *reinterpret_cast<epi_u32x4*>(q) = v;
}
__device__ __forceinline__ epi_u32x4 epi_ld16(const GemmParams&, const void* q) {
    return *reinterpret_cast<const epi_u32x4*>(q);
}

// Two workgroups per CU (g4 engines): workgroups b and b + 256 of a launch share a CU
// (tools/probe_placement.hip), and every tile takes the same time, so without help the two start,
// reach their epilogues and finish together, round after round.  Delaying the second workgroup of
// each CU in the first round by about half a tile keeps the pair half a tile apart for the whole
// launch (a finishing workgroup's successor starts at once), so one's epilogue runs beside the
// other's main loop.
// one_per_cu (256x256 engine): delay every other CU of each XCD in the first round instead (the
// CUs then reach their epilogues' store bursts at different times)
__device__ __forceinline__ void first_round_stagger(int ticks, bool one_per_cu = false) {
    if (ticks <= 0) return;
    const int lin = blockIdx.y * gridDim.x + blockIdx.x;
    if (one_per_cu ? (lin >= 256 || !((lin >> 3) & 1)) : (lin < 256 || lin >= 512)) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)ticks) __builtin_amdgcn_s_sleep(8);
}

// diagnostic timestamps (gemm_bf16_set_trace): record of 16 u64 per workgroup, written by lane 0
// of a wave with vector stores: 0 start, 1 main-loop end, 2 end (wave 0), 3 hardware id, 4 + w end
// of wave w (k = 2 writes both), 12 first K-step's operands landed (wave 0)
constexpr int TRACE_WORDS = 16;
__device__ __forceinline__ void trace_stamp(const GemmParams& p, int k) {
    if (!p.trace || (threadIdx.x & 63) != 0) return;
    const int w = threadIdx.x >> 6;
    if (w != 0 && k != 2) return;
    const long long rec = ((long long)blockIdx.y * gridDim.x + blockIdx.x) * TRACE_WORDS;
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    if (k == 2) {
        p.trace[rec + 4 + w] = t;
        if (w != 0) return;
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        p.trace[rec + 3] = ((unsigned long long)xcc << 32) | hw;
    }
    p.trace[rec + k] = t;
}

// diagnostic: time the main loop alone (the accumulators stay live so nothing is eliminated)
template <int NA, int NB>
__device__ __forceinline__ bool skip_epilogue(const GemmParams& p, f32x4_t (&acc)[NA][NB]) {
    if (!(p.no_epi & 1)) return false;
#pragma unroll
    for (int a = 0; a < NA; a++)
#pragma unroll
        for (int b = 0; b < NB; b++) asm volatile("" ::"v"(acc[a][b]));
    return true;
}

// epilogue for one lane's C[m][n..n+3] (n % 4 == 0, m < M, n < N).  EPI_F32_ATOMIC never reaches
// a kernel: the launchers turn it into K-split slabs + a fixed-order reduce (or EPI_F32_ACC)
template <int EPI>
__device__ __forceinline__ void epilogue(const GemmParams& p, int m, int n, f32x4_t& v) {
    static_assert(EPI != EPI_F32_ATOMIC, "split-K partials go through slabs");
    if constexpr (epi_bias(EPI)) {
        if (p.bias) {
            const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
            v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
        }
    }
    const long long off = (long long)m * p.ldc + n;
    if constexpr (EPI == EPI_F32_STORE) {
        *reinterpret_cast<float4*>((float*)p.C + off) = make_float4(v[0], v[1], v[2], v[3]);
    } else if constexpr (EPI == EPI_F32_ACC) {
        float4* q = reinterpret_cast<float4*>((float*)p.C + off);
        float4 o = *q;
        o.x += v[0]; o.y += v[1]; o.z += v[2]; o.w += v[3];
        *q = o;
    } else if constexpr (EPI == EPI_BF16_STORE) {
        *reinterpret_cast<uint2*>((bf16_t*)p.C + off) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    } else if constexpr (EPI == EPI_BF16_GELU) {
        *reinterpret_cast<uint2*>((bf16_t*)p.C + off) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        *reinterpret_cast<uint2*>((bf16_t*)p.C2 + off) =
            make_uint2(pack_bf16x2(gelu_fast_f(v[0]), gelu_fast_f(v[1])),
                       pack_bf16x2(gelu_fast_f(v[2]), gelu_fast_f(v[3])));
    } else if constexpr (EPI == EPI_F32_RESID) {
        const float4 r = *reinterpret_cast<const float4*>((const float*)p.aux +
                                                          (long long)m * p.ldaux + n);
        *reinterpret_cast<float4*>((float*)p.C + off) =
            make_float4(v[0] + r.x, v[1] + r.y, v[2] + r.z, v[3] + r.w);
    } else if constexpr (EPI == EPI_F32_SLAB) {
        float* slab = (float*)p.C + (long long)split_index(p.tiles) * p.M * p.ldc;
        *reinterpret_cast<float4*>(slab + off) = make_float4(v[0], v[1], v[2], v[3]);
    } else if constexpr (EPI == EPI_BF16_GELU_D) {
        float g[4], d[4];
#pragma unroll
        for (int j = 0; j < 4; j++) gelu_pair_fast_f(v[j], g[j], d[j]);
        *reinterpret_cast<uint2*>((bf16_t*)p.C + off) = make_uint2(pack_bf16x2(d[0], d[1]), pack_bf16x2(d[2], d[3]));
        *reinterpret_cast<uint2*>((bf16_t*)p.C2 + off) = make_uint2(pack_bf16x2(g[0], g[1]), pack_bf16x2(g[2], g[3]));
    } else if constexpr (epi_aux16(EPI)) {
#pragma clang fp contract(off)  // the products are rounded before the callers' column sums
        const uint2 h = *reinterpret_cast<const uint2*>((const bf16_t*)p.aux +
                                                        (long long)m * p.ldaux + n);
        const float x0 = __uint_as_float(h.x << 16), x1 = __uint_as_float(h.x & 0xffff0000u);
        const float x2 = __uint_as_float(h.y << 16), x3 = __uint_as_float(h.y & 0xffff0000u);
        if constexpr (EPI == EPI_BF16_DGELU) {
            v[0] *= gelu_grad_fast_f(x0); v[1] *= gelu_grad_fast_f(x1);
            v[2] *= gelu_grad_fast_f(x2); v[3] *= gelu_grad_fast_f(x3);
        } else {
            v[0] *= x0; v[1] *= x1; v[2] *= x2; v[3] *= x3;
        }
        *reinterpret_cast<uint2*>((bf16_t*)p.C + off) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    }
}

// ------------------------------------------------------------- row-contiguous (staged) epilogue
// Columns n..n+7 of row m (n % 8 == 0), v = raw accumulators: one 16-B (bf16) or 2 x 16-B (fp32)
// access per lane and operand, so a wave instruction covers whole 128-B lines.  cs accumulates
// the column sums of the DGELU output (fused bias gradient).
template <int EPI, bool MX = true>
__device__ __forceinline__ void epilogue8(const GemmParams& p, int m, int n, float (&v)[8],
                                          float (&cs)[8], int lane = 0, float* wb = nullptr) {
    if constexpr (epi_bias(EPI)) {
        if (p.bias) {
            const float4 b0 = *reinterpret_cast<const float4*>(p.bias + n);
            const float4 b1 = *reinterpret_cast<const float4*>(p.bias + n + 4);
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
    }
    const long long off = (long long)m * p.ldc + n;
    auto st_f32 = [&](float* q) {
        reinterpret_cast<float4*>(q)[0] = make_float4(v[0], v[1], v[2], v[3]);
        reinterpret_cast<float4*>(q)[1] = make_float4(v[4], v[5], v[6], v[7]);
    };
    auto pack8 = [&](const float (&w)[8]) {
        return make_uint4(pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]), pack_bf16x2(w[4], w[5]),
                          pack_bf16x2(w[6], w[7]));
    };
    if constexpr (EPI == EPI_F32_STORE) {
        st_f32((float*)p.C + off);
    } else if constexpr (EPI == EPI_F32_ACC) {
        float* q = (float*)p.C + off;
        const float4 o0 = reinterpret_cast<const float4*>(q)[0];
        const float4 o1 = reinterpret_cast<const float4*>(q)[1];
        v[0] += o0.x; v[1] += o0.y; v[2] += o0.z; v[3] += o0.w;
        v[4] += o1.x; v[5] += o1.y; v[6] += o1.z; v[7] += o1.w;
        st_f32(q);
    } else if constexpr (EPI == EPI_F32_SLAB) {
        st_f32((float*)p.C + (long long)split_index(p.tiles) * p.M * p.ldc + off);
    } else if constexpr (EPI == EPI_BF16_STORE) {
        *reinterpret_cast<uint4*>((bf16_t*)p.C + off) = pack8(v);
    } else if constexpr (EPI == EPI_BF16_GELU) {
        float gv[8];
#pragma unroll
        for (int j = 0; j < 8; j++) gv[j] = gelu_fast_f(v[j]);
        *reinterpret_cast<uint4*>((bf16_t*)p.C + off) = pack8(v);
        const uint4 g8 = pack8(gv);
        if (p.C2) *reinterpret_cast<uint4*>((bf16_t*)p.C2 + off) = g8;
        if constexpr (MX) {
            if (p.mx_q) mx_out8(p, m, n, g8.x, g8.y, g8.z, g8.w, lane);
            if (wb) stage_back8(wb, g8.x, g8.y, g8.z, g8.w);
        }
    } else if constexpr (EPI == EPI_F32_RESID) {
        const float* r = (const float*)p.aux + (long long)m * p.ldaux + n;
        const float4 r0 = reinterpret_cast<const float4*>(r)[0];
        const float4 r1 = reinterpret_cast<const float4*>(r)[1];
        v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
        v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
        st_f32((float*)p.C + off);
    } else if constexpr (EPI == EPI_BF16_GELU_D) {
        float gv[8], dv[8];
#pragma unroll
        for (int j = 0; j < 8; j++) gelu_pair_fast_f(v[j], gv[j], dv[j]);
        *reinterpret_cast<uint4*>((bf16_t*)p.C + off) = pack8(dv);
        const uint4 g8 = pack8(gv);
        if (p.C2) *reinterpret_cast<uint4*>((bf16_t*)p.C2 + off) = g8;
        if constexpr (MX) {
            if (p.mx_q) mx_out8(p, m, n, g8.x, g8.y, g8.z, g8.w, lane);
            if (wb) stage_back8(wb, g8.x, g8.y, g8.z, g8.w);
        }
    } else if constexpr (epi_aux16(EPI)) {
        const uint4 h = *reinterpret_cast<const uint4*>((const bf16_t*)p.aux + (long long)m * p.ldaux + n);
        const uint32_t hw[4] = {h.x, h.y, h.z, h.w};
        {  // products rounded before the column sums (no FMA contraction; see the staged epilogue)
#pragma clang fp contract(off)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const float lo = __uint_as_float(hw[j] << 16), hi = __uint_as_float(hw[j] & 0xffff0000u);
            if constexpr (EPI == EPI_BF16_DGELU) {
                v[2 * j] *= gelu_grad_fast_f(lo);
                v[2 * j + 1] *= gelu_grad_fast_f(hi);
            } else {
                v[2 * j] *= lo;
                v[2 * j + 1] *= hi;
            }
        }
#pragma unroll
        for (int j = 0; j < 8; j++) cs[j] += v[j];
        }
        const uint4 d8 = pack8(v);
        if (p.C) *reinterpret_cast<uint4*>((bf16_t*)p.C + off) = d8;
        if constexpr (MX) {
            if (p.mx_q) mx_out8(p, m, n, d8.x, d8.y, d8.z, d8.w, lane);
            if (wb) stage_back8(wb, d8.x, d8.y, d8.z, d8.w);
        }
    }
}

// Epilogue of one wave's 128x64 accumulator tile (8x4 16x16 tiles; lane (i,g) of tile (a,b) holds
// row 16a+i, columns 16b+4g..+3) through a wave-private LDS area of 64 x 68 fp32 (17 KiB, two
// passes of 64 rows): each lane then owns 8 consecutive columns of a row, so every global load
// and store of the epilogue is a 16-B access and a wave instruction covers 8 rows x 128 B (bf16)
// or 8 rows x 256 B (fp32) instead of 16 rows x 32 B.  Callers guarantee the area is free
// (every wave past the main loop and its LDS-DMA retired).
constexpr int STG_LD = 68;                       // padded row (floats): conflict-free b128 access
constexpr int STG_WAVE_BYTES = 64 * STG_LD * 4;  // 17,408 B per wave
// Interior wave tiles (all 128 rows < M, all 64 columns < N): one pass of 64 rows with every
// global load of the pass (aux rows, bias) issued before the first computation, and no branch
// between loads and stores.  The generic loop below serialised load -> s_waitcnt vmcnt(0) ->
// compute -> store per 8-row step (the wait also drained the previous step's stores), so the
// DGELU / RESID epilogues ran one HBM round trip per step.
typedef unsigned int epi_u32x4v __attribute__((ext_vector_type(4)));
// the aux operand rows of one interior 64-row pass (bf16: 8 x 16 B per lane, fp32: 16 x 16 B)
template <int EPI>
struct EpiAux {
    static constexpr bool AUX16 = epi_aux16(EPI);
    static constexpr bool AUX32 = EPI == EPI_F32_RESID || EPI == EPI_F32_ACC;
    static constexpr int N = AUX16 ? 8 : (AUX32 ? 16 : 0);
    epi_u32x4v ax[N > 0 ? N : 1];
    __device__ __forceinline__ void load(const GemmParams& p, int rr, int mrow, int n) {
        if constexpr (AUX16) {
#pragma unroll
            for (int it = 0; it < 8; it++)
                ax[it] = epi_ld16(p, (const bf16_t*)p.aux + (long long)(mrow + it * 8 + rr) * p.ldaux + n);
        } else if constexpr (AUX32) {
            const float* src = EPI == EPI_F32_RESID ? (const float*)p.aux : (const float*)p.C;
            const long long ld = EPI == EPI_F32_RESID ? p.ldaux : p.ldc;
#pragma unroll
            for (int it = 0; it < 8; it++) {
                const float* q = src + (long long)(mrow + it * 8 + rr) * ld + n;
                ax[2 * it] = epi_ld16(p, q);
                ax[2 * it + 1] = epi_ld16(p, q + 4);
            }
        }
    }
};
template <int EPI>
__device__ __forceinline__ void staged_pass_interior(const GemmParams& p, const float* st, int rr,
                                                     int cc, int mrow, int n, float (&cs)[8],
                                                     const float* bpre, const EpiAux<EPI>* pre = nullptr) {
    const int cc_lane = cc >> 3;  // the lane's column group (lane bits 0-2): mx_out8's block lanes
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (epi_bias(EPI)) {
        if (bpre) {  // the lane's 8 bias values, loaded by the caller under the main loop's tail
#pragma unroll
            for (int j = 0; j < 8; j++) bv[j] = bpre[j];
        } else if (p.bias) {
            const float4 b0 = *reinterpret_cast<const float4*>(p.bias + n);
            const float4 b1 = *reinterpret_cast<const float4*>(p.bias + n + 4);
            bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
            bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
        }
    }
    constexpr bool AUX16 = epi_aux16(EPI);
    constexpr bool AUX32 = EPI == EPI_F32_RESID || EPI == EPI_F32_ACC;
    EpiAux<EPI> own;
    if (!pre) own.load(p, rr, mrow, n);
    const u32x4* ax = pre ? pre->ax : own.ax;
    float* slab = nullptr;
    if constexpr (EPI == EPI_F32_SLAB) slab = (float*)p.C + (long long)split_index(p.tiles) * p.M * p.ldc;
#pragma unroll
    for (int it = 0; it < 8; it++) {
        const int r = it * 8 + rr;
        const f32x4_t lo = *reinterpret_cast<const f32x4_t*>(st + r * STG_LD + cc);
        const f32x4_t hi = *reinterpret_cast<const f32x4_t*>(st + r * STG_LD + cc + 4);
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const long long off = (long long)(mrow + r) * p.ldc + n;
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] += bv[j];
        auto pack8 = [](const float (&w)[8]) {
            return u32x4{pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]), pack_bf16x2(w[4], w[5]),
                         pack_bf16x2(w[6], w[7])};
        };
        auto st_f32 = [&](float* q) {
            epi_st16(p, q, u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])});
            epi_st16(p, q + 4, u32x4{__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7])});
        };
        if constexpr (EPI == EPI_F32_STORE) {
            st_f32((float*)p.C + off);
        } else if constexpr (EPI == EPI_F32_SLAB) {
            st_f32(slab + off);
        } else if constexpr (AUX32) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                v[j] += __uint_as_float(ax[2 * it][j]);
                v[4 + j] += __uint_as_float(ax[2 * it + 1][j]);
            }
            st_f32((float*)p.C + off);
        } else if constexpr (EPI == EPI_BF16_STORE) {
            epi_st16(p, (bf16_t*)p.C + off, pack8(v));
        } else if constexpr (EPI == EPI_BF16_GELU) {
            float gv[8];
#pragma unroll
            for (int j = 0; j < 8; j++) gv[j] = gelu_fast_f(v[j]);
            epi_st16(p, (bf16_t*)p.C + off, pack8(v));
            const u32x4 g8 = pack8(gv);
            if (p.C2) epi_st16(p, (bf16_t*)p.C2 + off, g8);
            if (p.mx_q) mx_out8(p, mrow + r, n, g8[0], g8[1], g8[2], g8[3], cc_lane);
            if (p.mxc_q) stage_back8(const_cast<float*>(st) + r * STG_LD + cc, g8[0], g8[1], g8[2], g8[3]);
        } else if constexpr (EPI == EPI_BF16_GELU_D) {
            float gv[8], dv[8];
#pragma unroll
            for (int j = 0; j < 8; j++) gelu_pair_fast_f(v[j], gv[j], dv[j]);
            epi_st16(p, (bf16_t*)p.C + off, pack8(dv));
            const u32x4 g8 = pack8(gv);
            if (p.C2) epi_st16(p, (bf16_t*)p.C2 + off, g8);
            if (p.mx_q) mx_out8(p, mrow + r, n, g8[0], g8[1], g8[2], g8[3], cc_lane);
            if (p.mxc_q) stage_back8(const_cast<float*>(st) + r * STG_LD + cc, g8[0], g8[1], g8[2], g8[3]);
        } else if constexpr (AUX16) {
            // the products are rounded before the column sums in every engine: no contraction of
            // v *= aux; cs += v into an FMA (hipcc decided that per kernel, so two engines with the same
            // arithmetic could differ in the sums' last bits)
#pragma clang fp contract(off)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float lo = __uint_as_float(ax[it][j] << 16), hi = __uint_as_float(ax[it][j] & 0xffff0000u);
                if constexpr (EPI == EPI_BF16_DGELU) {
                    v[2 * j] *= gelu_grad_fast_f(lo);
                    v[2 * j + 1] *= gelu_grad_fast_f(hi);
                } else {
                    v[2 * j] *= lo;
                    v[2 * j + 1] *= hi;
                }
            }
#pragma unroll
            for (int j = 0; j < 8; j++) cs[j] += v[j];
            const u32x4 d8 = pack8(v);
            if (p.C) epi_st16(p, (bf16_t*)p.C + off, d8);
            if (p.mx_q) mx_out8(p, mrow + r, n, d8[0], d8[1], d8[2], d8[3], cc_lane);
            if (p.mxc_q) stage_back8(const_cast<float*>(st) + r * STG_LD + cc, d8[0], d8[1], d8[2], d8[3]);
        }
    }
}

GemmParams make_gemm_params(const GemmArgs& a, int kchunk);  // gemm.hip

// one 64-row pass of a wave's 128x64 tile, staged in `st` (64 x STG_LD fp32, row r = tile row
// 64*pass + r): every lane owns 8 consecutive columns of a row per access
template <int EPI>
__device__ __forceinline__ void staged_pass(const GemmParams& p, const float* st, int lane, int m0,
                                            int n0, int pass, bool interior, float (&cs)[8],
                                            const float* bpre = nullptr, const EpiAux<EPI>* pre = nullptr) {
    const int rr = lane >> 3, cc = (lane & 7) * 8;
    if (interior) {
        staged_pass_interior<EPI>(p, st, rr, cc, m0 + pass * 64, n0 + cc, cs, bpre, pre);
        return;
    }
#pragma unroll
    for (int it = 0; it < 8; it++) {
        const int r = it * 8 + rr;
        float v[8];
        const f32x4_t lo = *reinterpret_cast<const f32x4_t*>(st + r * STG_LD + cc);
        const f32x4_t hi = *reinterpret_cast<const f32x4_t*>(st + r * STG_LD + cc + 4);
        v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
        v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
        const int m = m0 + pass * 64 + r, n = n0 + cc;
        if (m >= p.M) continue;
        if (n + 8 <= p.N) {
            epilogue8<EPI>(p, m, n, v, cs, lane,
                           epi_mx(EPI) && p.mxc_q ? const_cast<float*>(st) + r * STG_LD + cc : nullptr);
        } else if (n + 4 <= p.N) {  // ragged N (N % 8 == 4): the 4-wide form
            f32x4_t t = lo;
            epilogue<EPI>(p, m, n, t);
            if constexpr (epi_aux16(EPI)) {  // the 4-wide form does not sum: the output it stored
#pragma clang fp contract(off)
                cs[0] += t[0];
                cs[1] += t[1];
                cs[2] += t[2];
                cs[3] += t[3];
            }
        }
    }
}
// column-wise MX of one 64-row pass whose bf16 outputs stage_back8 left in `st` (the fp8 engine,
// GemmArgs::mxc_q): lane c takes column n0 + c, two 32-row blocks (a wave reads one staging row
// per step: conflict free), and writes 32 e4m3 bytes of the column's token run + the block's
// scale byte (as quantize_mx_cols_k).  M % 64 == 0 (host): a pass is wholly inside or outside M.
__device__ __forceinline__ void mx_cols_pass(const GemmParams& p, const float* st, int lane, int mrow, int n0) {
    if (mrow >= p.M) return;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const int c = n0 + lane;
#pragma unroll
    for (int b = 0; b < 2; b++) {
        float v[32];
        float amax = 0.f;
#pragma unroll
        for (int i = 0; i < 32; i++) {
            v[i] = st[(32 * b + i) * STG_LD + lane];
            amax = fmaxf(amax, fabsf(v[i]));
        }
        const int sb = mx_scale_byte(amax);
        const int tok = p.mxc_off + mrow + 32 * b, kb = tok >> 5;
        p.mxc_s[((long long)(kb >> 1) * p.mxc_rg + (c >> 5)) * 64 + (kb & 1) * 32 + (c & 31)] = (uint8_t)sb;
        const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);
        uint32_t w[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            int t = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * j] * inv, v[4 * j + 1] * inv, 0, false);
            t = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * j + 2] * inv, v[4 * j + 3] * inv, t, true);
            w[j] = (uint32_t)t;
        }
        uint8_t* dst = p.mxc_q + (long long)c * p.mxc_ld + tok;
        *reinterpret_cast<u32x4*>(dst) = u32x4{w[0], w[1], w[2], w[3]};
        *reinterpret_cast<u32x4*>(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
    }
}
template <int EPI>
__device__ __forceinline__ bool staged_interior(const GemmParams& p, int m0, int n0) {
    return EPI != EPI_F32_ATOMIC && m0 + 128 <= p.M && n0 + 64 <= p.N;
}
// fused bias gradient of the next GEMM: column sums of the DGELU / MUL output.  The wave's 128 x 64
// tile reduces its 8 row groups by shuffles and stores its 64 column sums as partial row m0/128
// (each (row, column) of the partial matrix has exactly one writer: no atomics, fixed order)
template <int EPI>
__device__ __forceinline__ void staged_colsum(const GemmParams& p, int lane, int m0, int n0, float (&cs)[8]) {
    if constexpr (epi_aux16(EPI)) {
        if (p.colsum_out) {
            const int rr = lane >> 3, cc = (lane & 7) * 8;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                float t = cs[j];
                t += __shfl_xor(t, 8, 64);
                t += __shfl_xor(t, 16, 64);
                t += __shfl_xor(t, 32, 64);
                cs[j] = t;
            }
            if (rr == 0 && m0 < p.M) {  // (a wave tile wholly past M has no partial row)
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (n0 + cc + j < p.N) p.colsum_out[(long long)(m0 >> 7) * p.N + n0 + cc + j] = cs[j];
            }
        }
    }
}

// the lane's 8 bias columns of the staged epilogue (n0 + 8 (lane & 7) ..), loaded ahead of it so
// the epilogue's first pass does not wait a memory round trip for them (zeros past N / no bias)
template <int EPI>
__device__ __forceinline__ void staged_bias_prefetch(const GemmParams& p, int lane, int n0, float (&bv)[8]) {
#pragma unroll
    for (int j = 0; j < 8; j++) bv[j] = 0.f;
    if constexpr (epi_bias(EPI)) {
        const int n = n0 + (lane & 7) * 8;
        if (p.bias && n + 8 <= p.N) {
            const float4 b0 = *reinterpret_cast<const float4*>(p.bias + n);
            const float4 b1 = *reinterpret_cast<const float4*>(p.bias + n + 4);
            bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w;
            bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
        }
    }
}
template <int EPI>
__device__ __forceinline__ void staged_epilogue(const GemmParams& p, f32x4_t (&acc)[8][4],
                                                char* stage, int lane, int m0, int n0,
                                                const float* bpre = nullptr) {
    float* st = reinterpret_cast<float*>(stage);
    const int i = lane & 15, g = lane >> 4;
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const bool interior = staged_interior<EPI>(p, m0, n0);
    auto stage_pass = [&](int pass) {
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 4; b++)
                *reinterpret_cast<f32x4_t*>(st + (a * 16 + i) * STG_LD + b * 16 + 4 * g) = acc[pass * 4 + a][b];
    };
    if (interior && EpiAux<EPI>::N > 0) {
        // aux-reading epilogues: both passes' aux rows are loaded up front, so the second pass
        // waits for its own loads only (vmcnt counts in issue order: loads issued after the first
        // pass's stores would wait for those stores too)
        const int rr = lane >> 3, n = n0 + (lane & 7) * 8;
        EpiAux<EPI> a0, a1;
        a0.load(p, rr, m0, n);
        a1.load(p, rr, m0 + 64, n);
        stage_pass(0);
        staged_pass_interior<EPI>(p, st, rr, (lane & 7) * 8, m0, n, cs, bpre, &a0);
        stage_pass(1);
        staged_pass_interior<EPI>(p, st, rr, (lane & 7) * 8, m0 + 64, n, cs, bpre, &a1);
    } else {
#pragma unroll
        for (int pass = 0; pass < 2; pass++) {
            stage_pass(pass);
            staged_pass<EPI>(p, st, lane, m0, n0, pass, interior, cs, bpre);
        }
    }
    staged_colsum<EPI>(p, lane, m0, n0, cs);
}

// ------------------------------------------------ 32-row swizzled staging (persistent 256x256 engine)
// The persistent engine stages a wave's 128 x 64 accumulator tile in four 32-row passes through 8 KiB
// of LDS (two free ring slots hold the eight waves), 64 fp32 per row with the 16-B chunk index XORed
// with (row & 15): the accumulator writes (8 rows x one chunk per ds_write_b128 lane group) and the
// row reads (lane (rr, cc): row 8 it + rr, chunks cc/4 and cc/4 + 1) hit distinct banks.
__device__ __forceinline__ int sq_off(int r, int col) {
    return r * 64 + ((((col >> 2) ^ (r & 15)) << 2) | (col & 3));
}
template <int EPI>
struct EpiAuxQ {  // aux operand rows of one interior 32-row pass (rows mrow + 8 it + rr, it < 4)
    static constexpr bool AUX16 = epi_aux16(EPI);
    static constexpr bool AUX32 = EPI == EPI_F32_RESID || EPI == EPI_F32_ACC;
    static constexpr int N = AUX16 ? 4 : (AUX32 ? 8 : 0);
    epi_u32x4v ax[N > 0 ? N : 1];
    __device__ __forceinline__ void load(const GemmParams& p, int rr, int mrow, int n) {
        if constexpr (AUX16) {
#pragma unroll
            for (int it = 0; it < 4; it++)
                ax[it] = epi_ld16(p, (const bf16_t*)p.aux + (long long)(mrow + it * 8 + rr) * p.ldaux + n);
        } else if constexpr (AUX32) {
            const float* src = EPI == EPI_F32_RESID ? (const float*)p.aux : (const float*)p.C;
            const long long ld = EPI == EPI_F32_RESID ? p.ldaux : p.ldc;
#pragma unroll
            for (int it = 0; it < 4; it++) {
                const float* q = src + (long long)(mrow + it * 8 + rr) * ld + n;
                ax[2 * it] = epi_ld16(p, q);
                ax[2 * it + 1] = epi_ld16(p, q + 4);
            }
        }
    }
};
// the 8 bf16 values (packed as stored) back into swizzled staging row r, columns cc..cc+7, as fp32
// (the column-wise MX pass of the fp8 engine reads them)
__device__ __forceinline__ void stage_back8_q(float* st, int r, int cc, uint32_t w0, uint32_t w1, uint32_t w2,
                                              uint32_t w3) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<f4*>(st + sq_off(r, cc)) = f4{__uint_as_float(w0 << 16), __uint_as_float(w0 & 0xffff0000u),
                                                    __uint_as_float(w1 << 16), __uint_as_float(w1 & 0xffff0000u)};
    *reinterpret_cast<f4*>(st + sq_off(r, cc + 4)) = f4{__uint_as_float(w2 << 16), __uint_as_float(w2 & 0xffff0000u),
                                                        __uint_as_float(w3 << 16), __uint_as_float(w3 & 0xffff0000u)};
}
// column-wise MX of one 32-row pass (one MX block per column) whose bf16 outputs stage_back8_q left in
// the swizzled staging: lane c takes column n0 + c (as mx_cols_pass, one block instead of two)
__device__ __forceinline__ void mx_cols_pass_q(const GemmParams& p, const float* st, int lane, int mrow, int n0) {
    if (mrow >= p.M) return;
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const int c = n0 + lane;
    // two sweeps over the column (amax, then quantize) instead of 32 values held in registers:
    // the persistent engine keeps the next tile's DMA state live through the epilogue
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 32; i++) amax = fmaxf(amax, fabsf(st[sq_off(i, lane)]));
    const int sb = mx_scale_byte(amax);
    const int tok = p.mxc_off + mrow, kb = tok >> 5;
    p.mxc_s[((long long)(kb >> 1) * p.mxc_rg + (c >> 5)) * 64 + (kb & 1) * 32 + (c & 31)] = (uint8_t)sb;
    const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const float v0 = st[sq_off(4 * j, lane)], v1 = st[sq_off(4 * j + 1, lane)];
        const float v2 = st[sq_off(4 * j + 2, lane)], v3 = st[sq_off(4 * j + 3, lane)];
        int t = __builtin_amdgcn_cvt_pk_fp8_f32(v0 * inv, v1 * inv, 0, false);
        t = __builtin_amdgcn_cvt_pk_fp8_f32(v2 * inv, v3 * inv, t, true);
        w[j] = (uint32_t)t;
    }
    uint8_t* dst = p.mxc_q + (long long)c * p.mxc_ld + tok;
    *reinterpret_cast<u32x4*>(dst) = u32x4{w[0], w[1], w[2], w[3]};
    *reinterpret_cast<u32x4*>(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
}
// one interior 32-row pass (all rows < M, all 64 columns < N); the MX outputs (mx_q row form,
// mxc_q column form via stage_back8_q) are the fp8 engine's
template <int EPI, bool MX>
__device__ __forceinline__ void staged_pass_interior_q(const GemmParams& p, float* st, int rr, int cc,
                                                       int mrow, int n, float (&cs)[8], const float* bv,
                                                       const EpiAuxQ<EPI>& aux) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    constexpr bool AUX16 = epi_aux16(EPI);
    constexpr bool AUX32 = EPI == EPI_F32_RESID || EPI == EPI_F32_ACC;
    const int cc_lane = cc >> 3;
#pragma unroll
    for (int it = 0; it < 4; it++) {
        const int r = it * 8 + rr;
        const f32x4_t lo = *reinterpret_cast<const f32x4_t*>(st + sq_off(r, cc));
        const f32x4_t hi = *reinterpret_cast<const f32x4_t*>(st + sq_off(r, cc + 4));
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const long long off = (long long)(mrow + r) * p.ldc + n;
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] += bv[j];
        auto pack8 = [](const float (&w)[8]) {
            return u32x4{pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3]), pack_bf16x2(w[4], w[5]),
                         pack_bf16x2(w[6], w[7])};
        };
        auto st_f32 = [&](float* q) {
            epi_st16(p, q, u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])});
            epi_st16(p, q + 4, u32x4{__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7])});
        };
        if constexpr (EPI == EPI_F32_STORE) {
            st_f32((float*)p.C + off);
        } else if constexpr (AUX32) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                v[j] += __uint_as_float(aux.ax[2 * it][j]);
                v[4 + j] += __uint_as_float(aux.ax[2 * it + 1][j]);
            }
            st_f32((float*)p.C + off);
        } else if constexpr (EPI == EPI_BF16_STORE) {
            epi_st16(p, (bf16_t*)p.C + off, pack8(v));
        } else if constexpr (EPI == EPI_BF16_GELU) {
            float gv[8];
#pragma unroll
            for (int j = 0; j < 8; j++) gv[j] = gelu_fast_f(v[j]);
            epi_st16(p, (bf16_t*)p.C + off, pack8(v));
            const u32x4 g8 = pack8(gv);
            if (p.C2) epi_st16(p, (bf16_t*)p.C2 + off, g8);
            if constexpr (MX) {
                if (p.mx_q) mx_out8(p, mrow + r, n, g8[0], g8[1], g8[2], g8[3], cc_lane);
                if (p.mxc_q) stage_back8_q(st, r, cc, g8[0], g8[1], g8[2], g8[3]);
            }
        } else if constexpr (EPI == EPI_BF16_GELU_D) {
            float gv[8], dv[8];
#pragma unroll
            for (int j = 0; j < 8; j++) gelu_pair_fast_f(v[j], gv[j], dv[j]);
            epi_st16(p, (bf16_t*)p.C + off, pack8(dv));
            const u32x4 g8 = pack8(gv);
            if (p.C2) epi_st16(p, (bf16_t*)p.C2 + off, g8);
            if constexpr (MX) {
                if (p.mx_q) mx_out8(p, mrow + r, n, g8[0], g8[1], g8[2], g8[3], cc_lane);
                if (p.mxc_q) stage_back8_q(st, r, cc, g8[0], g8[1], g8[2], g8[3]);
            }
        } else if constexpr (AUX16) {
            {  // products rounded before the column sums (no FMA contraction)
#pragma clang fp contract(off)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float a0 = __uint_as_float(aux.ax[it][j] << 16), a1 = __uint_as_float(aux.ax[it][j] & 0xffff0000u);
                if constexpr (EPI == EPI_BF16_DGELU) {
                    v[2 * j] *= gelu_grad_fast_f(a0);
                    v[2 * j + 1] *= gelu_grad_fast_f(a1);
                } else {
                    v[2 * j] *= a0;
                    v[2 * j + 1] *= a1;
                }
            }
#pragma unroll
            for (int j = 0; j < 8; j++) cs[j] += v[j];
            }
            const u32x4 d8 = pack8(v);
            if (p.C) epi_st16(p, (bf16_t*)p.C + off, d8);
            if constexpr (MX) {
                if (p.mx_q) mx_out8(p, mrow + r, n, d8[0], d8[1], d8[2], d8[3], cc_lane);
                if (p.mxc_q) stage_back8_q(st, r, cc, d8[0], d8[1], d8[2], d8[3]);
            }
        }
    }
}
// Epilogue of one wave's 128 x 64 tile through 8 KiB of swizzled staging (four 32-row passes); the
// interior form loads the next pass's aux rows under the current pass.  Same outputs, bit for bit,
// as staged_epilogue (same values, same column-sum order: the cs partials add the tile's rows in the
// same order per lane, rows 8 it + rr of pass 0..3 = rows 8 it' + rr of the 64-row passes).
// stage_pass(pass) writes rows 32 pass .. 32 pass + 31 of the wave tile into st (sq_off layout)
template <int EPI, bool MX, typename StagePass>
__device__ __forceinline__ void staged_epilogue_q_any(const GemmParams& p, StagePass stage_pass, float* st, int lane,
                                                      int m0, int n0, const float* bpre) {
    const int rr = lane >> 3, cc = (lane & 7) * 8, n = n0 + cc;
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto mx_cols = [&](int pass) {
        if constexpr (MX && epi_mx(EPI)) {
            if (p.mxc_q) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                mx_cols_pass_q(p, st, lane, m0 + pass * 32, n0);
            }
        }
    };
    if (staged_interior<EPI>(p, m0, n0)) {
        if constexpr (!MX) {  // the next pass's aux rows load under the current pass
            EpiAuxQ<EPI> a0, a1;
            a0.load(p, rr, m0, n);
#pragma unroll
            for (int pass = 0; pass < 4; pass += 2) {
                a1.load(p, rr, m0 + (pass + 1) * 32, n);
                stage_pass(pass);
                staged_pass_interior_q<EPI, MX>(p, st, rr, cc, m0 + pass * 32, n, cs, bpre, a0);
                if (pass + 2 < 4) a0.load(p, rr, m0 + (pass + 2) * 32, n);
                stage_pass(pass + 1);
                staged_pass_interior_q<EPI, MX>(p, st, rr, cc, m0 + (pass + 1) * 32, n, cs, bpre, a1);
            }
        } else {  // fp8 engine (MX outputs): one set of aux registers, loaded ahead of the staging writes
#pragma unroll
            for (int pass = 0; pass < 4; pass++) {
                EpiAuxQ<EPI> a0;
                a0.load(p, rr, m0 + pass * 32, n);
                stage_pass(pass);
                staged_pass_interior_q<EPI, MX>(p, st, rr, cc, m0 + pass * 32, n, cs, bpre, a0);
                mx_cols(pass);
            }
        }
    } else {
#pragma unroll
        for (int pass = 0; pass < 4; pass++) {
            stage_pass(pass);
#pragma unroll
            for (int it = 0; it < 4; it++) {
                const int r = it * 8 + rr;
                const f32x4_t lo = *reinterpret_cast<const f32x4_t*>(st + sq_off(r, cc));
                const f32x4_t hi = *reinterpret_cast<const f32x4_t*>(st + sq_off(r, cc + 4));
                float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                const int m = m0 + pass * 32 + r;
                if (m >= p.M) continue;
                if (n + 8 <= p.N) {
                    if constexpr (MX && epi_mx(EPI)) {
                        float wb[8];
                        epilogue8<EPI>(p, m, n, v, cs, lane, p.mxc_q ? wb : nullptr);
                        if (p.mxc_q) {
                            typedef float f4 __attribute__((ext_vector_type(4)));
                            *reinterpret_cast<f4*>(st + sq_off(r, cc)) = f4{wb[0], wb[1], wb[2], wb[3]};
                            *reinterpret_cast<f4*>(st + sq_off(r, cc + 4)) = f4{wb[4], wb[5], wb[6], wb[7]};
                        }
                    } else {
                        epilogue8<EPI, false>(p, m, n, v, cs, lane, nullptr);
                    }
                } else if (n + 4 <= p.N) {
                    f32x4_t t = lo;
                    epilogue<EPI>(p, m, n, t);
                    if constexpr (epi_aux16(EPI)) {
#pragma clang fp contract(off)
                        cs[0] += t[0]; cs[1] += t[1]; cs[2] += t[2]; cs[3] += t[3];
                    }
                }
            }
            mx_cols(pass);
        }
    }
    staged_colsum<EPI>(p, lane, m0, n0, cs);
}
// the bf16 engines' 16x16 accumulator tiles: lane (i,g) of tile (a,b) holds row 16a+i, columns
// 16b+4g..+3
template <int EPI>
__device__ __forceinline__ void staged_epilogue_q(const GemmParams& p, f32x4_t (&acc)[8][4], float* st, int lane,
                                                  int m0, int n0, const float* bpre) {
    const int i = lane & 15, g = lane >> 4;
    auto stage_pass = [&](int pass) {
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 4; b++)
                *reinterpret_cast<f32x4_t*>(st + sq_off(a * 16 + i, b * 16 + 4 * g)) = acc[pass * 2 + a][b];
    };
    staged_epilogue_q_any<EPI, false>(p, stage_pass, st, lane, m0, n0, bpre);
}

}  // namespace vit
