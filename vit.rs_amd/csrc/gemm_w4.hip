// gemm_w4.hip — one-wave-per-SIMD persistent bf16 GEMM engine (variant 9) for matmul_forward and
// the input-gradient half of matmul_backward (train_vit.rs:384-398, 530-557), K-contiguous A and B.
//
// Why a second persistent engine.  g2::gemm_kernel_s (gemm.hip) runs 8 waves per CU, two per SIMD,
// each wave a 128 x 64 accumulator tile (128 registers) with its fragments re-read every 16 MFMAs;
// its 32-deep K-step is 4 barriers, and PMC shows the matrix pipe busy only 36-49 % of the
// cycles (profiles/r04_gemm_pmc.md).  With ONE wave per SIMD a wave may hold 512 VGPR+AGPR
// registers (MI355X_MICROARCH.md "Register files"): here each of the 4 waves owns a 128 x 128
// tile (256 fp32 accumulators, AGPRs), so a 32-deep K-step is 64 MFMAs (1024 matrix cycles) per
// wave between ONE barrier, with the next step's 16 fragment reads and the ring's 8 LDS-DMA pieces
// issued between this step's MFMAs (two fragment sets in registers).  LDS reads per MFMA halve
// (1 ds_read_b128 per 4 MFMAs instead of 12 per 32 ... per 16 at the g2 phase granularity).
//
// Tile 256 x 256, 4 waves as 2 (M) x 2 (N).  LDS: a 4-slot ring of 32 KiB K-steps (A | B images,
// the g2 swizzled layout, filled by global_load_lds two to three steps ahead, never drained across
// tile boundaries) + 32 KiB of epilogue staging (8 KiB per wave, the g2 32-row swizzled passes) =
// 160 KiB, one workgroup per CU.  Per step kt of a tile (slot sl):
//   wait own DMA pieces of step kt+1 (counted vmcnt) ; lgkmcnt(0) (this step's fragments) ; s_barrier
//   LDS-DMA of step kt+4 into slot sl (every wave finished reading it before the barrier)
//   16 fragment reads of step kt+1 from slot sl+1   } interleaved
//   64 MFMAs of step kt                              }
// The MFMAs, their operands and their K order per accumulator are those of g2 (D = B^T A^T with
// v_mfma_f32_16x16x32_bf16, one 32-deep slice per step in order), and the epilogue is g2's staged
// 32-row epilogue applied to each 64-column half of the wave tile: outputs (and the fused column
// sums) are bit-identical to variants 2 and 7 (tests/test_gpu_ops.py).
#include "gemm_common.h"

#include <type_traits>

namespace vit {
namespace g5 {
constexpr int BM = 256, BN = 256, BK = 32, NT = 256;
constexpr int IMG_BYTES = 256 * BK * 2;    // 16 KiB per operand per slot
constexpr int SLOT_BYTES = 2 * IMG_BYTES;  // 32 KiB (A | B)
constexpr int NS = 4;                      // ring slots
constexpr int STG_BYTES = 8192;            // epilogue staging per wave (32 rows x 64 fp32)
constexpr int SMEM = NS * SLOT_BYTES + 4 * STG_BYTES;  // 160 KiB
constexpr int LEAD = NS;                   // the DMA of step kt + LEAD is issued in step kt
static_assert(SMEM <= 160 * 1024, "LDS");

__device__ __forceinline__ int kc_swz(int row) { return (row >> 1) & 3; }

// s_waitcnt vmcnt(n) for the literal counts the pipeline uses
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
        case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

template <int EPI>
__global__ __launch_bounds__(NT, 1) void gemm_kernel_w4(GemmParams p) {
    __shared__ __attribute__((aligned(1024))) char smem[SMEM];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int ntm = cdiv(p.M, BM), ntn = cdiv(p.N, BN), tiles = ntm * ntn;
    const int nblk = gridDim.x;
    const int my_tiles = (tiles - (int)blockIdx.x + nblk - 1) / nblk;
    const int nk = p.K / BK;  // host: K % 64 == 0, K >= 128 (nk even, >= LEAD)
    const char* A = (const char*)p.A;
    const char* B = (const char*)p.B;
    f32x4_t acc[8][8];
    auto zero_acc = [&]() {
#pragma unroll
        for (int a = 0; a < 8; a++)
#pragma unroll
            for (int b = 0; b < 8; b++) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    };
    zero_acc();
    if (my_tiles <= 0) return;
    // DMA sources of a tile: piece q of this wave's share of the A / B image (1 KiB block 4 q + wave
    // = 16 rows x 64 B), as 32-bit byte offsets from the operand base at k = 0 (g2's swizzle)
    struct TileSrc {
        int tm0, tn0, t;
        uint32_t a[4], b[4];
    };
    auto tile_src = [&](int j, TileSrc& ts) {
        ts.t = xcd_remap(j * nblk + (int)blockIdx.x, tiles);
        ts.tm0 = (ts.t / ntn) * BM;
        ts.tn0 = (ts.t % ntn) * BN;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int row = (q * 4 + wave) * 16 + (lane >> 2);
            const int c = (lane & 3) ^ kc_swz(row);
            ts.a[q] = (uint32_t)((min(ts.tm0 + row, p.M - 1) * p.lda + c * 8) * 2);
            ts.b[q] = (uint32_t)((min(ts.tn0 + row, p.N - 1) * p.ldb + c * 8) * 2);
        }
    };
    TileSrc cur, nxt;
    tile_src(0, cur);
    nxt = cur;
    if (my_tiles > 1) tile_src(1, nxt);  // (no next tile: nxt = cur, see issue())
    auto glds = [&](const char* src, char* dst) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    };
    // the 8 LDS-DMA pieces of step kt2 of the current tile (kt2 >= nk: step kt2 - nk of the next
    // one) into slot sl; piece q in 0..3 = A, 4..7 = B.  Branch-free: after the last tile `nxt`
    // equals `cur`, so the ring's last LEAD fills re-fetch steps of the current tile into free
    // slots (retired before the epilogue, never read).
    // The source address is a wave-uniform base (operand + k offset, SGPRs) plus the lane's 32-bit
    // offset, so the DMA issues in the saddr form with no per-piece 64-bit VALU address chain (an
    // in-order wave would stall its MFMA stream on that chain before every piece).
    auto issue = [&](int kt2, int sl, int q) {
        const bool c = kt2 < nk;
        const int koff = __builtin_amdgcn_readfirstlane((c ? kt2 : kt2 - nk) * (BK * 2));
        char* dst = smem + sl * SLOT_BYTES;
        if (q < 4) {
            const uint32_t off = c ? cur.a[q] : nxt.a[q];
            glds(A + koff + off, dst + (q * 4 + wave) * 1024);
        } else {
            const uint32_t off = c ? cur.b[q - 4] : nxt.b[q - 4];
            glds(B + koff + off, dst + IMG_BYTES + ((q - 4) * 4 + wave) * 1024);
        }
    };
    // the lane's fragment-read offset inside a 16-row block (rows r0 + i, 16-B chunk g of the
    // 32-deep k-slice): r0 % 16 == 0, so the swizzle term is lane-constant
    const int i16 = lane & 15, g4 = lane >> 4;
    const int foff = i16 * 64 + ((g4 ^ kc_swz(i16)) << 4);
    const int arow = wm * 128, brow = wn * 128;
    auto read_frags = [&](int sl, bf16x8_t (&fa)[8], bf16x8_t (&fb)[8]) {  // (tile start)
        const char* img = smem + sl * SLOT_BYTES + foff;
#pragma unroll
        for (int a = 0; a < 8; a++) fa[a] = *reinterpret_cast<const bf16x8_t*>(img + (arow + a * 16) * 64);
#pragma unroll
        for (int b = 0; b < 8; b++) fb[b] = *reinterpret_cast<const bf16x8_t*>(img + IMG_BYTES + (brow + b * 16) * 64);
    };
    // lgkmcnt(0) through the builtin (encoding: vmcnt / expcnt at their maxima, lgkmcnt 0), so that
    // the compiler's own wait tracking sees the fragments land here and adds no wait of its own in
    // front of the first MFMA (an asm wait is invisible to it)
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    int sl = 0;  // slot of step kt (global step count % NS)
    // one K-step: F = this step's fragments (loaded), G = the next step's (read here unless LAST,
    // the tile's final step)
    auto step = [&](auto last_c, int kt, int j, bf16x8_t (&fa)[8], bf16x8_t (&fb)[8], bf16x8_t (&ga)[8],
                    bf16x8_t (&gb)[8]) {
        constexpr bool LAST = decltype(last_c)::value;
        // own pieces of step kt + 1 landed (the younger ones: steps kt + 2, kt + 3).  In a later
        // tile's first LEAD - 1 steps they were retired before the previous epilogue, which issued
        // stores since: no counted wait there
        if constexpr (!LAST) {
            if (j == 0 || kt >= LEAD - 1) wait_vm(8 * (LEAD - 2));
        }
        bar();
#ifndef VIT_W4_DIAG
#define VIT_W4_DIAG 0  // diagnostic builds (timing only, wrong results): 1 no DMA in the loop, 2 no fragment reads
#endif
        if constexpr (!LAST && (VIT_W4_DIAG & 2)) {
#pragma unroll
            for (int a = 0; a < 8; a++) asm volatile("" : "=v"(ga[a]) : "0"(fa[a]));
#pragma unroll
            for (int b = 0; b < 8; b++) asm volatile("" : "=v"(gb[b]) : "0"(fb[b]));
        }
#ifndef VIT_W4_SCHED
#define VIT_W4_SCHED 1
#endif
        const char* img = smem + ((sl + 1) & (NS - 1)) * SLOT_BYTES + foff;
        auto read_pair = [&](int r) {  // fragment reads 2r, 2r + 1 of the next step (A 0..7, B 0..7)
            if constexpr (!LAST && !(VIT_W4_DIAG & 2)) {
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    const int f = 2 * r + u;
                    if (f < 8) ga[f] = *reinterpret_cast<const bf16x8_t*>(img + (arow + f * 16) * 64);
                    else gb[f - 8] = *reinterpret_cast<const bf16x8_t*>(img + IMG_BYTES + (brow + (f - 8) * 16) * 64);
                }
            }
        };
        auto dma = [&](int q) {
            if constexpr (!(VIT_W4_DIAG & 1)) issue(kt + LEAD, sl, q);
        };
        if constexpr (VIT_W4_SCHED == 1) {
            // DMA piece q, then fragment reads 2q, 2q + 1, in source order, so the compiler (which
            // keeps LDS reads and LDS-DMA writes in program order: it cannot tell slot sl from sl+1)
            // may spread both over the step: per 8 MFMAs one piece and two reads.  Every wave then
            // issues its 8 pieces evenly instead of all four waves issuing at once.
#pragma unroll
            for (int r = 0; r < 8; r++) {
                dma(r);
                read_pair(r);
            }
        } else {
#pragma unroll
            for (int r = 0; r < 8; r++) read_pair(r);
#pragma unroll
            for (int q = 0; q < 8; q++) dma(q);
        }
#pragma unroll
        for (int a = 0; a < 8; a++)
#pragma unroll
            for (int b = 0; b < 8; b++)
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b], fa[a], acc[a][b], 0, 0, 0);
        // interleave (LLVM SchedGroupMask: MFMA 0x8, VMEM_READ 0x20, DS_READ 0x100)
        if constexpr (VIT_W4_SCHED == 1) {
            // MFMAs first after the barrier, the step's scalar address work (SALU 0x4) spread over the
            // first four gaps instead of a clump in front of the first MFMA (28 SALU there measured),
            // then one non-MFMA issue per gap: DMA, MFMA x2, read, MFMA x2, read, MFMA x2
#pragma unroll
            for (int r = 0; r < 4; r++) {
                __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x4, 7, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
            if constexpr (!LAST) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
            if constexpr (!LAST) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
            for (int r = 1; r < 8; r++) {
                __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
                if constexpr (!LAST) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
                if constexpr (!LAST) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x8, 2, 0);
            }
        } else {  // the 16 reads between the first 32 MFMAs, the 8 pieces between the other 32
#pragma unroll
            for (int r = 0; r < 8; r++) {
                if constexpr (!LAST) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x8, 4, 0);
            }
#pragma unroll
            for (int r = 0; r < 8; r++) {
                __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x8, 4, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        sl = (sl + 1) & (NS - 1);
    };
    using T_ = std::integral_constant<bool, true>;
    using F_ = std::integral_constant<bool, false>;

    // first tile: steps 0 .. LEAD-1 in flight, step 0 landed and visible
#pragma unroll
    for (int s = 0; s < LEAD; s++)
#pragma unroll
        for (int q = 0; q < 8; q++) issue(s, s, q);
    wait_vm(8 * (LEAD - 1));
    bar();
    bf16x8_t fa0[8], fb0[8], fa1[8], fb1[8];
    for (int j = 0; j < my_tiles; j++) {
        const bool more = j + 1 < my_tiles;
        if (p.trace && tid == 0) p.trace[(long long)cur.t * TRACE_WORDS] = __builtin_amdgcn_s_memrealtime();
        read_frags(sl, fa0, fb0);
        for (int kt = 0; kt < nk - 2; kt += 2) {
            step(F_{}, kt, j, fa0, fb0, fa1, fb1);
            step(F_{}, kt + 1, j, fa1, fb1, fa0, fb0);
        }
        step(F_{}, nk - 2, j, fa0, fb0, fa1, fb1);
        step(T_{}, nk - 1, j, fa1, fb1, fa0, fb0);
        if (p.trace && tid == 0) p.trace[(long long)cur.t * TRACE_WORDS + 1] = __builtin_amdgcn_s_memrealtime();
        const int n0 = cur.tn0 + wn * 128, m0 = cur.tm0 + wm * 128;
        float bpre0[8], bpre1[8];
        staged_bias_prefetch<EPI>(p, lane, n0, bpre0);
        staged_bias_prefetch<EPI>(p, lane, n0 + 64, bpre1);
        // the next tile's steps 0 .. LEAD-1 (and the bias) landed, visible to every wave after the
        // barrier; the staging area is the wave's own
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (!skip_epilogue(p, acc)) {
            float* st = reinterpret_cast<float*>(smem + NS * SLOT_BYTES + wave * STG_BYTES);
            const int i = lane & 15, g = lane >> 4;
            // the staging writes take the accumulators straight from their AGPRs (inline asm with an
            // "a" operand): written as C++ stores, the register allocator copied the finished
            // accumulators into VGPRs at the last MFMA and spilled (the aux epilogues)
            uint32_t sa[4];
#pragma unroll
            for (int b = 0; b < 4; b++)
                sa[b] = (uint32_t)(uintptr_t)LDS_PTR(char, reinterpret_cast<char*>(st + sq_off(i, b * 16 + 4 * g)));
#pragma unroll
            for (int h = 0; h < 2; h++) {
                auto stage_pass = [&](int pass) {
#pragma unroll
                    for (int a = 0; a < 2; a++)
#pragma unroll
                        for (int b = 0; b < 4; b++)
                            asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(sa[b]), "a"(acc[pass * 2 + a][h * 4 + b]),
                                         "i"(a * 16 * 64 * 4)
                                         : "memory");
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                };
                staged_epilogue_q_any<EPI, false>(p, stage_pass, st, lane, m0, n0 + h * 64, h ? bpre1 : bpre0);
            }
        }
        if (p.trace && (tid & 63) == 0) {
            const long long rec = (long long)cur.t * TRACE_WORDS;
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            p.trace[rec + 4 + wave] = t;
            if (wave == 0) {
                p.trace[rec + 2] = t;
                p.trace[rec + 3] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                                   __builtin_amdgcn_s_getreg((31 << 11) | 4);
            }
        }
        zero_acc();
        if (more) tile_src(j + 1, cur);
        if (j + 2 < my_tiles) tile_src(j + 2, nxt);
        else nxt = cur;
    }
}
}  // namespace g5

// variant 9 launcher (gemm.hip launch_g2): K-contiguous A and B, no split-K, K % 64 == 0,
// K >= 128, 32-bit DMA offsets; false = not taken (the caller falls back)
bool gemm_bf16_w4(const GemmArgs& a, const GemmParams& p, int tiles, hipStream_t s) {
    if (!(a.a_kcontig && a.b_kcontig) || a.K % 64 || a.K < 4 * g5::BK ||
        (long long)p.M * p.lda * 2 >= (1LL << 31) || (long long)p.N * p.ldb * 2 >= (1LL << 31))
        return false;
    const int cus = gemm_cu_count();
    const dim3 pg(tiles < cus ? tiles : cus);
    switch (a.epi) {
#define VIT_CASE(E) \
    case E: g5::gemm_kernel_w4<E><<<pg, g5::NT, 0, s>>>(p); return true;
        VIT_CASE(EPI_F32_STORE)
        VIT_CASE(EPI_F32_ACC)
        VIT_CASE(EPI_BF16_STORE)
        VIT_CASE(EPI_BF16_GELU)
        VIT_CASE(EPI_F32_RESID)
        VIT_CASE(EPI_BF16_DGELU)
        VIT_CASE(EPI_BF16_GELU_D)
        VIT_CASE(EPI_BF16_MUL)
#undef VIT_CASE
        default: return false;
    }
}

}  // namespace vit
