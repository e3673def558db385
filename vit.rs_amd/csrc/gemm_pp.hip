// gemm_pp.hip — variant 11: the two-group ping-pong persistent bf16 GEMM (matmul_forward /
// matmul_backward's input gradient, train_vit.rs:384-398 / :532-541, with the trainer's fused
// epilogues).
//
// Why: the streaming 256x256 engine (variant 7, gemm.hip g2::gemm_kernel_s) runs its
// main loop at ~1.2-1.3 PF/s, then every wave of the CU runs the tile's epilogue (bias, GELU pair,
// fp32 residual, x aux + column sums, bf16 / fp32 stores) with the matrix pipes idle: ~5 ms of a
// 36 ms ViT-B/16 step.  Two 256x256 accumulator sets do not fit one CU's registers (256 + 256 of the
// 512 per SIMD lane), so the tile is 192 x 256: each SIMD holds one wave of each of two groups,
// 96 x 128 accumulators per wave (192 registers), and the groups alternate —
//
//     group 0:  main loop tile 0 | epilogue tile 0     | main loop tile 2 | epilogue tile 2 ...
//     group 1:  (idle)           | main loop tile 1    | epilogue tile 1  | main loop tile 3 ...
//
// so a tile's epilogue (VALU, LDS staging, global stores) runs beside the next tile's MFMAs on the
// same SIMDs: one wave per SIMD issues MFMAs (16x16x32 bf16 holds the SIMD's vector issue 8 of its
// 16 cycles) while its partner issues the epilogue's VALU and stores in the other 8.
//
// One LDS ring serves both groups: 4 slots of one 32-deep K-step (A 192 x 32 + B 256 x 32 bf16 =
// 28 KiB), streamed across tile boundaries; plus 4 x 8.25 KiB of epilogue staging (145 KiB).  One
// s_barrier per K-step; the epilogue group takes part in every barrier, running one or two chunks
// (4 rows x 128 columns of its wave tile) between them.  The DMA for K-step T is issued by the group
// that will read it, three steps ahead: by the main group inside its tile, and for the next tile's
// first three steps by the epilogue group in the last three intervals of the current tile, so every
// counted vmcnt wait covers only the waiting wave's own LDS-DMA pieces.  Operands go through buffer
// resources per tile (rows past M read as zero: no clamping registers).
//
// Same MFMAs in the same K order per accumulator and the same per-element epilogue arithmetic as the
// one-tile and streaming engines, so every output is bit-identical to variants 2 / 7 except the
// x-aux epilogues' column sums (partial rows per 96 output rows here, per 128 there: fp32
// association differs; deterministic).
#include <type_traits>

#include "gemm_common.h"

namespace vit {
namespace g6 {
constexpr int BM = 192, BN = 256, BK = 32, NT = 512;
constexpr int A_BYTES = BM * BK * 2;      // 12 KiB: 12 pieces of 16 rows x 64 B
constexpr int B_BYTES = BN * BK * 2;      // 16 KiB: 16 pieces
constexpr int SLOT = A_BYTES + B_BYTES;   // 28 KiB
constexpr int NS = 4;                     // ring slots (DMA three steps ahead)
constexpr int ST_LD = 132;                // staging row (floats; st_pos): conflict-free writes and reads
constexpr int ST_WAVE = 16 * ST_LD * 4;   // 8,448 B: one 16-row pass of a 96 x 128 wave tile
constexpr int LDS_BYTES = NS * SLOT + 4 * ST_WAVE;
constexpr int NCHUNK = 24;                // epilogue chunks per wave tile: 6 passes x 4 row groups
static_assert(LDS_BYTES <= 160 * 1024, "LDS");
#ifndef VIT_PP_EPRIO
#define VIT_PP_EPRIO 0  // s_setprio of the epilogue group (the main group runs at 1)
#endif
#ifndef VIT_PP_NOEPI
#define VIT_PP_NOEPI 0  // diagnostic compile: no epilogue code (register-pressure experiments)
#endif

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long off, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((char*)const_cast<void*>(base) + off, (short)0,
                                             (int)(bytes > 0 ? bytes : 0), 0x00020000);
}

// tile j of this workgroup (as the streaming engine: round j is the tile the one-tile grid gives
// block j * nblk + b, XCD-aware; groups of gm row panels walked column by column)
struct Tile {
    int tm0, tn0;
};
__device__ __forceinline__ Tile tile_of(const GemmParams& p, int j, int ntm, int ntn) {
    const int tiles = ntm * ntn;
    const int t = xcd_remap(j * (int)gridDim.x + (int)blockIdx.x, tiles);
    Tile r;
    if (p.gm > 0) {
        const int per = p.gm * ntn, g = t / per, rem = t - g * per, rows = min(p.gm, ntm - g * p.gm);
        r.tm0 = (g * p.gm + rem % rows) * BM;
        r.tn0 = (rem / rows) * BN;
    } else {
        r.tm0 = (t / ntn) * BM;
        r.tn0 = (t % ntn) * BN;
    }
    return r;
}

// piece q (0..6: A pieces 0..2, then B pieces 0..3) of this wave's LDS-DMA share of K-step ks of tile t
template <int Q>
__device__ __forceinline__ void issue_piece(const GemmParams& p, Tile t, int ks, char* dst, int wq, uint32_t la,
                                            uint32_t lb) {
    uint32_t kb = (uint32_t)ks * (BK * 2);
    asm volatile("" : "+v"(la), "+v"(lb), "+s"(kb));  // (as issue_step: no hoisted offsets)
    if constexpr (Q < 3) {
        const auto ra = rsrc(p.A, (long long)t.tm0 * p.lda * 2, (long long)(p.M - t.tm0) * p.lda * 2);
        const int blk = Q * 4 + wq;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(dst + blk * 1024), 16,
                                                 la + (uint32_t)blk * (16u * 2u * (uint32_t)p.lda) + kb, 0, 0, 0);
    } else {
        const auto rb = rsrc(p.B, (long long)t.tn0 * p.ldb * 2, (long long)(p.N - t.tn0) * p.ldb * 2);
        const int blk = (Q - 3) * 4 + wq;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void*)(dst + A_BYTES + blk * 1024),
                                                 16, lb + (uint32_t)blk * (16u * 2u * (uint32_t)p.ldb) + kb, 0, 0, 0);
    }
}
// this wave's 7 LDS-DMA pieces (A: 3, B: 4) of K-step ks of tile t into slot dst.  Piece blk covers
// image rows 16 blk .. 16 blk + 15; lane l lands at dst + 1024 blk + 16 l = row 16 blk + l / 4, 16-B
// position l % 4, and carries global chunk (l % 4) ^ kc_swz(row) (the g2 swizzle: kc_swz(r) =
// (r >> 1) & 3, a function of the lane alone since 16 blk is a multiple of 16).  la / lb: the lane's
// byte offset inside a piece (row l / 4 and its chunk).
__device__ __forceinline__ void issue_step(const GemmParams& p, Tile t, int ks, char* dst, int wq, uint32_t la,
                                           uint32_t lb) {
    const auto ra = rsrc(p.A, (long long)t.tm0 * p.lda * 2, (long long)(p.M - t.tm0) * p.lda * 2);
    const auto rb = rsrc(p.B, (long long)t.tn0 * p.ldb * 2, (long long)(p.N - t.tn0) * p.ldb * 2);
    uint32_t kb = (uint32_t)ks * (BK * 2);
    // computed here, at the issue: hipcc otherwise hoists the 21 offsets of the epilogue group's three
    // DMA intervals (constant K-steps 0..2) out of the tile loop and spills them
    asm volatile("" : "+v"(la), "+v"(lb), "+s"(kb));
    const uint32_t pa = 16u * 2u * (uint32_t)p.lda, pb = 16u * 2u * (uint32_t)p.ldb;
#pragma unroll
    for (int q = 0; q < 3; q++) {
        const int blk = q * 4 + wq;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(dst + blk * 1024), 16,
                                                 la + (uint32_t)blk * pa + kb, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int blk = q * 4 + wq;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rb, (__attribute__((address_space(3))) void*)(dst + A_BYTES + blk * 1024), 16, lb + (uint32_t)blk * pb + kb,
            0, 0, 0);
    }
}

// 8 bf16 of image rows r0 .. r0 + 15 (r0 % 16 == 0) for the slot's 32-deep k: lane (i, g) gets
// k = 8 g .. 8 g + 7 of row r0 + i, at img + 64 r0 + fo with the lane's offset fo = frag_off(lane)
// (the swizzle (r >> 1) & 3 depends on i alone), so a read is one uniform base + one VGPR + an
// immediate
__device__ __forceinline__ uint32_t frag_off(int lane) {
    const int i = lane & 15, g = lane >> 4;
    return (uint32_t)(i * 64 + ((g ^ ((i >> 1) & 3)) << 4));
}
__device__ __forceinline__ bf16x8_t frag(const char* img, int r0, uint32_t fo) {
    return *reinterpret_cast<const bf16x8_t*>(img + fo + r0 * 64);
}
#if VIT_PP_TRACE
// trace build, debug flag 128 (timing only, wrong results): every main-loop fragment read hits row 0
#define FRAG(img, r0, fo) frag(img, (p.dbg & 128) ? 0 : (r0), (p.dbg & 128) ? 0u : (fo))
#else
#define FRAG(img, r0, fo) frag(img, r0, fo)
#endif
#if VIT_PP_TRACE
// trace build, debug flag 128 (timing only, wrong results): every main-loop fragment read hits row 0
#define FRAG(img, r0, fo) frag(img, (p.dbg & 128) ? 0 : (r0), (p.dbg & 128) ? 0u : (fo))
#else
#define FRAG(img, r0, fo) frag(img, r0, fo)
#endif

__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
        case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

// the aux operand of one chunk (row m, the lane's 8 columns n .. n + 7)
template <int EPI>
struct Aux {
    static constexpr bool A16 = epi_aux16(EPI);
    static constexpr bool A32 = EPI == EPI_F32_RESID || EPI == EPI_F32_ACC;
    u32x4 h;
    f32x4_t f[2];
    __device__ __forceinline__ void load(const GemmParams& p, int m, int n) {
        m = min(m, p.M - 1);  // rows past M feed no output
        if constexpr (A16) {
            h = *reinterpret_cast<const u32x4*>((const bf16_t*)p.aux + (long long)m * p.ldaux + n);
        } else if constexpr (A32) {
            const float* q = EPI == EPI_F32_RESID ? (const float*)p.aux + (long long)m * p.ldaux + n
                                                  : (const float*)p.C + (long long)m * p.ldc + n;
            f[0] = *reinterpret_cast<const f32x4_t*>(q);
            f[1] = *reinterpret_cast<const f32x4_t*>(q + 4);
        }
    }
};

__device__ __forceinline__ void st_f4(float* q, f32x4_t v) {
    *reinterpret_cast<u32x4*>(q) = u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                                         __float_as_uint(v[3])};
}

// the epilogue of 4 values of one row (columns n + 4h .. n + 4h + 3 of the lane's 8), with the
// per-element arithmetic of the staged epilogues (gemm_common.h staged_pass_interior_q); bf16
// results come back packed in o[0..1] (and o2 for the GELU pairs' second output) for the caller's
// 16-B store.  Halves, not all 8 at once: fewer live temporaries while the epilogue shares the
// register file with the not yet staged accumulators.
template <int EPI>
__device__ __forceinline__ void epi_half(const GemmParams& p, long long off, int h, f32x4_t v, const float (&bv)[8],
                                         float (&cs)[8], const Aux<EPI>& ax, uint32_t* o, uint32_t* o2) {
#pragma unroll
    for (int j = 0; j < 4; j++) v[j] += bv[4 * h + j];
    if constexpr (EPI == EPI_F32_STORE) {
        st_f4((float*)p.C + off + 4 * h, v);
    } else if constexpr (EPI == EPI_F32_RESID || EPI == EPI_F32_ACC) {
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] += ax.f[h][j];
        st_f4((float*)p.C + off + 4 * h, v);
    } else if constexpr (EPI == EPI_BF16_STORE) {
        o[0] = pack_bf16x2(v[0], v[1]);
        o[1] = pack_bf16x2(v[2], v[3]);
    } else if constexpr (EPI == EPI_BF16_GELU) {
        float g[4];
#pragma unroll
        for (int j = 0; j < 4; j++) g[j] = gelu_fast_f(v[j]);
        o[0] = pack_bf16x2(v[0], v[1]);
        o[1] = pack_bf16x2(v[2], v[3]);
        o2[0] = pack_bf16x2(g[0], g[1]);
        o2[1] = pack_bf16x2(g[2], g[3]);
    } else if constexpr (EPI == EPI_BF16_GELU_D) {
        float g[4], d[4];
#pragma unroll
        for (int j = 0; j < 4; j++) gelu_pair_fast_f(v[j], g[j], d[j]);
        o[0] = pack_bf16x2(d[0], d[1]);
        o[1] = pack_bf16x2(d[2], d[3]);
        o2[0] = pack_bf16x2(g[0], g[1]);
        o2[1] = pack_bf16x2(g[2], g[3]);
    } else if constexpr (epi_aux16(EPI)) {
        {
#pragma clang fp contract(off)  // products rounded before the column sums (as every engine)
            const uint32_t hw[2] = {ax.h[2 * h], ax.h[2 * h + 1]};
#pragma unroll
            for (int j = 0; j < 2; j++) {
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
            for (int j = 0; j < 4; j++) cs[4 * h + j] += v[j];
        }
        o[0] = pack_bf16x2(v[0], v[1]);
        o[1] = pack_bf16x2(v[2], v[3]);
    }
}

// staging position of tile row r, column c (one 16-row pass of a wave's 96 x 128 tile): rows of
// ST_LD words, the second 64-column half 4 words further on.  Accumulator writes (lane (i, g):
// row i, columns 16 b + 4 g) and row reads (lane (rr, cc): row r, columns 8 cc .. 8 cc + 7, two
// ds_read_b128) then touch 64 distinct banks per 16 lanes.
__device__ __forceinline__ int st_pos(int r, int c) { return r * ST_LD + c + ((c >> 6) << 2); }

// Epilogue of a wave's 96 x 128 tile (rows m0.., columns n0..) in NCHUNK chunks: chunk c = rows
// 16 (c / 4) + 4 (c % 4) + rr of the tile, lane (rr = lane / 16, cc = lane % 16) taking the 8
// consecutive columns 8 cc .. 8 cc + 7, so every global access is 16 B per lane (a wave instruction
// covers 4 rows x 256 B of bf16).  Each pass (16 rows = acc[a][0..7]) is staged through the wave's
// 16 x ST_LD fp32 area.  Software-pipelined so that no step waits on a latency inside its interval:
// chunk c's values were read from the staging in the previous step, and this step computes and
// stores chunk c, stages the next pass if chunk c + 1 opens it, reads chunk c + 1, and loads the aux
// rows of chunk c + 3.  SYNC: the steps are spread over I barrier intervals of the main group (I
// barriers in all, one after a step when I >= NCHUNK, else I of them spread evenly), and the
// barriers do not wait for the wave's own LDS reads (ebar).
template <int EPI, bool SYNC, typename Bar>
__device__ __forceinline__ void epilogue(const GemmParams& p, f32x4_t (&acc)[6][8], float* st, int lane, int m0,
                                         int n0, int I, Bar ebar) {
    const int rr = lane >> 4, cc = lane & 15, i16 = lane & 15, g4 = lane >> 4;
    const int n = n0 + 8 * cc;
    auto stage = [&](int a) {
#pragma unroll
        for (int b = 0; b < 8; b++) *reinterpret_cast<f32x4_t*>(st + st_pos(i16, 16 * b + 4 * g4)) = acc[a][b];
    };
    auto rd = [&](int c, f32x4_t& lo, f32x4_t& hi) {
        const int r = 4 * (c & 3) + rr;
        lo = *reinterpret_cast<const f32x4_t*>(st + st_pos(r, 8 * cc));
        hi = *reinterpret_cast<const f32x4_t*>(st + st_pos(r, 8 * cc + 4));
    };
    // pass 0 leaves the registers first: the epilogue's own state (bias, aux prefetch, column sums)
    // is allocated while 5 of the 6 accumulator passes are still live, not 6
    f32x4_t vlo, vhi;
    stage(0);
    rd(0, vlo, vhi);
    __builtin_amdgcn_sched_barrier(0);
    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (epi_bias(EPI)) {
        if (p.bias) {
            const f32x4_t b0 = *reinterpret_cast<const f32x4_t*>(p.bias + n);
            const f32x4_t b1 = *reinterpret_cast<const f32x4_t*>(p.bias + n + 4);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                bv[j] = b0[j];
                bv[4 + j] = b1[j];
            }
        }
    }
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    constexpr int PF = Aux<EPI>::A32 ? 2 : 3;  // aux rows loaded PF chunks ahead
    Aux<EPI> ax[PF + 1];
    auto row_of = [&](int c) { return m0 + 16 * (c >> 2) + 4 * (c & 3) + rr; };
#pragma unroll
    for (int c = 0; c < PF; c++) ax[c].load(p, row_of(c), n);
#pragma unroll
    for (int c = 0; c < NCHUNK; c++) {
        const int m = row_of(c);
        if (m < p.M) {
            const long long off = (long long)m * p.ldc + n;
            uint32_t o[4], o2[4];
            epi_half<EPI>(p, off, 0, vlo, bv, cs, ax[c % (PF + 1)], o, o2);
            epi_half<EPI>(p, off, 1, vhi, bv, cs, ax[c % (PF + 1)], o + 2, o2 + 2);
            if constexpr (EPI == EPI_BF16_STORE || EPI == EPI_BF16_GELU || EPI == EPI_BF16_GELU_D || epi_aux16(EPI)) {
                if ((EPI != EPI_BF16_MUL && EPI != EPI_BF16_DGELU) || p.C)
                    *reinterpret_cast<u32x4*>((bf16_t*)p.C + off) = u32x4{o[0], o[1], o[2], o[3]};
            }
            if constexpr (EPI == EPI_BF16_GELU || EPI == EPI_BF16_GELU_D) {
                if (p.C2) *reinterpret_cast<u32x4*>((bf16_t*)p.C2 + off) = u32x4{o2[0], o2[1], o2[2], o2[3]};
            }
        }
        if (c + 1 < NCHUNK) {
            if (((c + 1) & 3) == 0) stage((c + 1) >> 2);  // pass (c + 1) / 4 opens: its reads follow in order
            rd(c + 1, vlo, vhi);
        }
        if (c + PF < NCHUNK) ax[(c + PF) % (PF + 1)].load(p, row_of(c + PF), n);
        if constexpr (SYNC) {
            if (I >= NCHUNK || ((c + 1) * I) / NCHUNK != (c * I) / NCHUNK) ebar();
        }
    }
    if constexpr (epi_aux16(EPI)) {
        if (p.colsum_out) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                float t = cs[j];
                t += __shfl_xor(t, 16, 64);
                t += __shfl_xor(t, 32, 64);
                cs[j] = t;
            }
            if (rr == 0 && m0 < p.M) {
                float* q = p.colsum_out + (long long)(m0 / 96) * p.N + n;
                st_f4(q, f32x4_t{cs[0], cs[1], cs[2], cs[3]});
                st_f4(q + 4, f32x4_t{cs[4], cs[5], cs[6], cs[7]});
            }
        }
    }
    if constexpr (SYNC) {
        for (int i = NCHUNK; i < I; i++) ebar();
    }
}

template <int EPI>
__global__ __launch_bounds__(NT, 1) void gemm_kernel_pp(GemmParams p) {
    __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wave >> 2, wq = wave & 3, wm = wq >> 1, wn = wq & 1;
    const int ntm = cdiv(p.M, BM), ntn = p.N / BN, tiles = ntm * ntn;
    const int nblk = gridDim.x;
    const int my_tiles = (tiles - (int)blockIdx.x + nblk - 1) / nblk;
    const int nk = p.K / BK;  // host: K % 64 == 0, nk >= 8
    if (my_tiles <= 0) return;
    // the lane's byte offset inside a DMA piece: row l / 4 of the piece, global chunk (l % 4) ^ kc_swz
    const int prow = lane >> 2, pch = (lane & 3) ^ ((lane >> 3) & 3);
    const uint32_t la = (uint32_t)((prow * p.lda + pch * 8) * 2);
    const uint32_t lb = (uint32_t)((prow * p.ldb + pch * 8) * 2);
    float* st = reinterpret_cast<float*>(smem + NS * SLOT + wq * ST_WAVE);
    const uint32_t fo = frag_off(lane);
    f32x4_t acc[6][8];
#if VIT_PP_TRACE
    // diagnostic build (tools/pp_trace.py): lane 0 of every wave of workgroups 0..7 stamps s_memtime
    // (shader cycles) on arrival at and release from each barrier, into its own 512-word record
    unsigned long long* tr = p.trace && blockIdx.x < 8 ? p.trace + ((long long)blockIdx.x * 8 + wave) * 512 : nullptr;
    int tc = 0;
    auto stamp = [&]() {
        if (tr && lane == 0 && tc < 512) tr[tc] = __builtin_amdgcn_s_memtime();
        tc++;
    };
#else
    auto stamp = [&]() {};
#endif
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        stamp();
#if VIT_PP_TRACE
        if (!(p.dbg & 32))  // (trace build, debug flag 32: no barriers at all, timing only)
#endif
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        stamp();
        __builtin_amdgcn_sched_barrier(0);
    };
    // the epilogue group's barrier: its LDS traffic is its private staging, so no lgkmcnt(0) (its
    // reads of the next chunk stay in flight across the barrier)
    auto ebar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        stamp();
#if VIT_PP_TRACE
        if (!(p.dbg & 32))  // (trace build, debug flag 32: no barriers at all, timing only)
#endif
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        stamp();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto slot = [&](int S) { return smem + (S & (NS - 1)) * SLOT; };
    // prologue: tile 0's group fetches its first three K-steps
    if (grp == 0) {
        const Tile t0 = tile_of(p, 0, ntm, ntn);
#pragma unroll
        for (int s = 0; s < 3; s++) issue_step(p, t0, s, slot(s), wq, la, lb);
        wait_vm(14);
    }
    bar();
    const int I = nk - 3;  // the epilogue group's barrier intervals before its DMA intervals
    // the three DMA intervals at the end of another group's tile: this group's tile jn's first steps
    auto dma_intervals = [&](int jn) {
        const bool own = jn < my_tiles;
        const Tile tn = tile_of(p, own ? jn : 0, ntm, ntn);
        for (int k = 0; k < 3; k++) {
            if (own) issue_step(p, tn, k, slot(jn * nk + k), wq, la, lb);
            if (k == 2 && own) wait_vm(14);
            bar();
        }
    };
    if (grp == 1) {  // tile 0 runs on group 0: nothing to finish yet, then fetch tile 1
        for (int i = 0; i < I; i++) bar();
        dma_intervals(1);
    }
    // This group's tiles are jj = grp, grp + 2, ...: it runs tile jj, then, while the other group runs
    // tile jj + 1, finishes tile jj (epilogue) and fetches tile jj + 2's first three K-steps.  Every
    // path through the loop body consumes the accumulators before the next tile zeroes them.
    for (int jj = grp; jj < my_tiles; jj += 2) {
        // ------------------------------------------------------------------ main loop of tile jj
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int a = 0; a < 6; a++)
#pragma unroll
            for (int b = 0; b < 8; b++) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const Tile t = tile_of(p, jj, ntm, ntn);
        // K-step s: MFMA groups b = 0..6 (B fragment b of the 8 against the 6 A fragments; B fragments
        // 4..7 read into the registers of 0..3 as those free up; DMA piece b of step s + 3 after group
        // b), the wait for this wave's pieces of step s + 1, the barrier, then group 7 with the next
        // step's fragments read into the registers it frees: the barrier sits one MFMA group before
        // the step's end, so step s + 1 starts on fragments already in registers.
        bf16x8_t fa[6], fb[4];
        {
            const char* img = slot(jj * nk);
#pragma unroll
            for (int b = 0; b < 4; b++) fb[b] = frag(img + A_BYTES + wn * 128 * 64, 16 * b, fo);
#pragma unroll
            for (int a = 0; a < 6; a++) fa[a] = frag(img + wm * 96 * 64, 16 * a, fo);
        }
        // one loop body for every step (straight-line tail steps spilled accumulators): the last three
        // steps skip their DMA by a uniform branch, the last one prefetches fragments it never uses
        // (slot S + 1 then holds the other group's next tile or stale data: harmless reads)
        for (int s = 0; s < nk; s++) {
            const int S = jj * nk + s;
            const bool dma = s + 3 < nk;
            const char* imgB = slot(S) + A_BYTES + wn * 128 * 64;
            char* dst = slot(S + 3);
            // MFMA groups b = 0..5 (B fragment b against the 6 A fragments); B fragments 4..7 are read
            // into the registers of 0..3 as those free up; the step's 7 LDS-DMA pieces go between groups
#pragma unroll
            for (int b = 0; b < 6; b++) {
#pragma unroll
                for (int a = 0; a < 6; a++)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b & 3], fa[a], acc[a][b], 0, 0, 0);
                if (b < 4) fb[b] = FRAG(imgB, 16 * (b + 4), fo);
#if VIT_PP_TRACE
                if (dma && !(p.dbg & 64)) {  // (trace build, debug flag 64: no DMA in the main loop, timing only)
#else
                if (dma) {
#endif
                    switch (b) {
                        case 0: issue_piece<0>(p, t, s + 3, dst, wq, la, lb); break;
                        case 1: issue_piece<1>(p, t, s + 3, dst, wq, la, lb); break;
                        case 2: issue_piece<2>(p, t, s + 3, dst, wq, la, lb); break;
                        case 3: issue_piece<3>(p, t, s + 3, dst, wq, la, lb); break;
                        case 4: issue_piece<4>(p, t, s + 3, dst, wq, la, lb); break;
                        default:
                            issue_piece<5>(p, t, s + 3, dst, wq, la, lb);
                            issue_piece<6>(p, t, s + 3, dst, wq, la, lb);
                            break;
                    }
                }
            }
            // this wave's pieces of step s + 1 landed (younger: steps s + 2, s + 3 as far as issued)
            wait_vm(dma ? 14 : (s + 2 < nk ? 7 : 0));
            bar();
            // groups 6 and 7 after the barrier, A fragment by A fragment, with the next step's fragments
            // read into the registers they free (B 0, 1 at once; A a after its last use; B 2, 3 last):
            // step s + 1 opens on fragments already in registers.  (The last step's reads are of data
            // it never uses: slot S + 1 then holds the other group's next tile or stale data.)
            const char* nA = slot(S + 1) + wm * 96 * 64;
            const char* nB = slot(S + 1) + A_BYTES + wn * 128 * 64;
            fb[0] = FRAG(nB, 0, fo);
            fb[1] = FRAG(nB, 16, fo);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
            for (int a = 0; a < 6; a++) {
                acc[a][6] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[2], fa[a], acc[a][6], 0, 0, 0);
                acc[a][7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[3], fa[a], acc[a][7], 0, 0, 0);
                fa[a] = FRAG(nA, 16 * a, fo);
                __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            fb[2] = FRAG(nB, 32, fo);
            fb[3] = FRAG(nB, 48, fo);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        // ------------------------------------------------- epilogue of tile jj (+ DMA for jj + 2)
        __builtin_amdgcn_s_setprio(VIT_PP_EPRIO);
        const int m0 = t.tm0 + wm * 96, n0 = t.tn0 + wn * 128;
        if (jj + 1 < my_tiles) {  // beside the other group's tile jj + 1
            if (!VIT_PP_NOEPI && !(p.no_epi & 1)) {
                epilogue<EPI, true>(p, acc, st, lane, m0, n0, I, ebar);
            } else {  // diagnostic main-loop-only timing: the accumulators stay live, nothing stored
#pragma unroll
                for (int a = 0; a < 6; a++)
#pragma unroll
                    for (int b = 0; b < 8; b++) asm volatile("" ::"v"(acc[a][b]));
                for (int i = 0; i < I; i++) bar();
            }
            dma_intervals(jj + 2);
        } else {  // the last tile: after every other wave's work, no barriers
            if (!VIT_PP_NOEPI && !(p.no_epi & 1)) {
                epilogue<EPI, false>(p, acc, st, lane, m0, n0, 0, bar);
            } else {
#pragma unroll
                for (int a = 0; a < 6; a++)
#pragma unroll
                    for (int b = 0; b < 8; b++) asm volatile("" ::"v"(acc[a][b]));
            }
        }
    }
}
}  // namespace g6

// the shapes the ping-pong engine takes: K-contiguous A and B, no split-K, N % 256 == 0, K % 64 == 0
// with >= 8 K-steps, M >= 192, 32-bit tile-relative offsets, no fused MX output
bool gemm_pp_shape(const GemmArgs& a) {
    if (!a.a_kcontig || !a.b_kcontig || a.mx_q || a.mxc_q) return false;
    if (a.N % g6::BN || a.K % 64 || a.K / g6::BK < 8 || a.M < g6::BM) return false;
    if ((long long)a.M * a.lda * 2 >= (1LL << 31) || (long long)a.N * a.ldb * 2 >= (1LL << 31)) return false;
    if (a.ldc % 4 || (a.aux && a.ldaux % 4)) return false;
    switch (a.epi) {
        case EPI_F32_STORE: case EPI_F32_ACC: case EPI_BF16_STORE: case EPI_BF16_GELU: case EPI_F32_RESID:
        case EPI_BF16_DGELU: case EPI_BF16_GELU_D: case EPI_BF16_MUL: return true;
        default: return false;
    }
}

void gemm_bf16_pp(const GemmArgs& a, const GemmParams& p, hipStream_t s) {
    const int tiles = cdiv(a.M, g6::BM) * (a.N / g6::BN);
    const int cus = gemm_cu_count();
    const dim3 grid(tiles < cus ? tiles : cus);
    switch (a.epi) {
#define VIT_CASE(E) \
    case E: g6::gemm_kernel_pp<E><<<grid, g6::NT, 0, s>>>(p); break;
        VIT_CASE(EPI_F32_STORE)
        VIT_CASE(EPI_F32_ACC)
        VIT_CASE(EPI_BF16_STORE)
        VIT_CASE(EPI_BF16_GELU)
        VIT_CASE(EPI_F32_RESID)
        VIT_CASE(EPI_BF16_DGELU)
        VIT_CASE(EPI_BF16_GELU_D)
        VIT_CASE(EPI_BF16_MUL)
#undef VIT_CASE
        default: set_error("gemm_bf16_pp: unsupported epilogue %d", a.epi); return;
    }
}

}  // namespace vit
