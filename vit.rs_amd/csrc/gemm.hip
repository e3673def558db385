// gemm.hip — MFMA GEMMs for matmul_forward / matmul_backward (train_vit.rs:384-398, 530-557).
//
// gemm_bf16: 128x128x64 block tile, 256 threads = 4 waves (2x2), 64x64 per wave as 4x4
//   v_mfma_f32_16x16x32_bf16 tiles, register-staged double-buffered LDS, one barrier per
//   K-tile, XCD-aware bijective block remap.  Both operand kinds use one fragment scheme:
//   a 32-deep k-step is read as two 8-byte halves at k = 4g.. and 16+4g.. (g = lane>>4), from a
//   K-contiguous image with ds_read_b64 or from an M/N-contiguous image with
//   ds_read_b64_tr_b16 (the gfx950 transpose read).  Because every operand uses the same k
//   permutation the products are exact, and the padded row strides (144 B / 288 B) make both
//   reads bank-conflict free for the 32-lane halves.  The MFMA is issued with the operands
//   swapped (D = B^T A^T) so each lane owns 4 consecutive output columns of one row: the
//   epilogue stores 8-16 contiguous bytes per lane.
// gemm_f32: 64x64x16 tile on v_mfma_f32_16x16x4_f32 (exact fp32 fma chain), generic strides,
//   bounds-checked scalar staging; the fp32 parity path.
#include "gemm_common.h"

#include <algorithm>
#include <cstdlib>

// one phase per K-step in the persistent engine (the fp8 engine's r06 form): measured slower for bf16
// (per ViT-B/16 layer 2.595 / 2.601 vs 2.544 / 2.545 ms, step 36.13 / 36.02 vs 35.88 / 35.80 ms,
// two interleaved rounds, profiles/r06_onephase.txt), so off
#ifndef VIT_G2_ONEPHASE
#define VIT_G2_ONEPHASE 0
#endif

namespace vit {

// ============================================================================ bf16 MFMA GEMM
namespace bf {
constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int SK = 72;    // K-contig image row stride (elements): 144 B
constexpr int SMN = 144;  // M/N-contig image row stride (elements): 288 B
constexpr int TILE = 9216;  // = 128*72 = 64*144 elements per operand image
static_assert(BM * SK == TILE && BK * SMN == TILE, "image sizes");

template <bool KC, int ROWS>
struct Stager {
    uint4 r[4];
    // ROWS = rows of the operand tile along M (or N); K-tile = BK
    __device__ __forceinline__ void load(const bf16_t* __restrict__ base, long long ld, int row0,
                                         int rows_lim, int k0, int k_lim, int tid) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const int idx = c * NT + tid;
            int row, col;
            bool ok;
            const bf16_t* p;
            if constexpr (KC) {
                row = idx >> 3;
                col = (idx & 7) * 8;
                ok = (row0 + row < rows_lim) && (k0 + col < k_lim);
                p = base + (long long)(row0 + row) * ld + (k0 + col);
            } else {
                row = idx >> 4;  // k row
                col = (idx & 15) * 8;
                ok = (k0 + row < k_lim) && (row0 + col < rows_lim);
                p = base + (long long)(k0 + row) * ld + (row0 + col);
            }
            r[c] = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
        }
    }
    // M/N-contig image: this thread's 8 columns ((tid&15)*8 ..) summed over its 4 rows
    __device__ __forceinline__ void colsum(float (&acc)[8]) const {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(&r[c]);
#pragma unroll
            for (int e = 0; e < 4; e++) {
                acc[2 * e] += __uint_as_float(w[e] << 16);
                acc[2 * e + 1] += __uint_as_float(w[e] & 0xffff0000u);
            }
        }
    }
    __device__ __forceinline__ void store(bf16_t* img, int tid) const {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const int idx = c * NT + tid;
            int off;
            if constexpr (KC)
                off = (idx >> 3) * SK + (idx & 7) * 8;
            else
                off = (idx >> 4) * SMN + (idx & 15) * 8;
            *reinterpret_cast<uint4*>(img + off) = r[c];
        }
    }
};

// fragment of rows [r0, r0+16) for k-step s (32 deep) — element j<4: k = 32s+4g+j,
// j>=4: k = 32s+16+4g+(j-4)
template <bool KC>
__device__ __forceinline__ bf16x8_t frag(const bf16_t* img, int r0, int s, int lane) {
    const int i = lane & 15, g = lane >> 4;
    bf16x4_t lo, hi;
    if constexpr (KC) {
        const bf16_t* p = img + (r0 + i) * SK + 32 * s + 4 * g;
        lo = *reinterpret_cast<const bf16x4_t*>(p);
        hi = *reinterpret_cast<const bf16x4_t*>(p + 16);
    } else {
        const bf16_t* p = img + (32 * s + 4 * g + (i >> 2)) * SMN + r0 + 4 * (i & 3);
        lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4_t, p));
        hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(LDS_PTR(bf16x4_t, p + 16 * SMN));
    }
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <bool AK, bool BKC, int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(GemmParams p) {
    __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TILE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int ntm = cdiv(p.M, BM), ntn = cdiv(p.N, BN);
    const int wg = xcd_remap(blockIdx.x, ntm * ntn);
    const int tm0 = (wg / ntn) * BM, tn0 = (wg % ntn) * BN;
    const int kbeg = blockIdx.y * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);
    const int nk = cdiv(kend - kbeg, BK);
    const bf16_t* A = (const bf16_t*)p.A;
    const bf16_t* B = (const bf16_t*)p.B;

    f32x4_t acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    Stager<AK, BM> sa;
    Stager<BKC, BN> sb;
    // fused bias gradient (wgrad): the blocks of the first N tile sum their A tiles
    const bool do_db = !AK && p.dbias != nullptr && tn0 == 0;
    float dbacc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (nk > 0) {
        sa.load(A, p.lda, tm0, p.M, kbeg, kend, tid);
        sb.load(B, p.ldb, tn0, p.N, kbeg, kend, tid);
        if constexpr (!AK) if (do_db) sa.colsum(dbacc);
        sa.store(smem, tid);
        sb.store(smem + TILE, tid);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; kt++) {
        const int cur = kt & 1;
        const bf16_t* imgA = smem + cur * 2 * TILE;
        const bf16_t* imgB = imgA + TILE;
        const bool more = kt + 1 < nk;
        if (more) {
            const int k0 = kbeg + (kt + 1) * BK;
            sa.load(A, p.lda, tm0, p.M, k0, kend, tid);
            sb.load(B, p.ldb, tn0, p.N, k0, kend, tid);
        }
#pragma unroll
        for (int s = 0; s < 2; s++) {
            bf16x8_t af[4], bfr[4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                af[t] = frag<AK>(imgA, wm * 64 + t * 16, s, lane);
                bfr[t] = frag<BKC>(imgB, wn * 64 + t * 16, s, lane);
            }
#pragma unroll
            for (int a = 0; a < 4; a++)
#pragma unroll
                for (int b = 0; b < 4; b++)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], af[a], acc[a][b],
                                                                        0, 0, 0);
        }
        if (more) {
            bf16_t* nxt = smem + (cur ^ 1) * 2 * TILE;
            if constexpr (!AK) if (do_db) sa.colsum(dbacc);
            sa.store(nxt, tid);
            sb.store(nxt + TILE, tid);
        }
        __syncthreads();
    }

    if constexpr (!AK) {
        if (do_db) {  // reduce the 16 threads sharing a column chunk, one atomic per column
            float* red = reinterpret_cast<float*>(smem);  // [16 row groups][128 cols]
#pragma unroll
            for (int e = 0; e < 8; e++) red[(tid >> 4) * 128 + (tid & 15) * 8 + e] = dbacc[e];
            __syncthreads();
            if (tid < 128 && tm0 + tid < p.M) {
                float t = 0.f;
#pragma unroll
                for (int q = 0; q < 16; q++) t += red[q * 128 + tid];
                atomicAdd(p.dbias + tm0 + tid, t);
            }
        }
    }

    // epilogue: lane holds C[m][n..n+3], m = tm0 + wm*64 + a*16 + (lane&15),
    //           n = tn0 + wn*64 + b*16 + 4*(lane>>4)
    const int i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int a = 0; a < 4; a++) {
        const int m = tm0 + wm * 64 + a * 16 + i;
        if (m >= p.M) continue;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int n = tn0 + wn * 64 + b * 16 + 4 * g;
            if (n >= p.N) continue;
            if constexpr (EPI == EPI_F32_SLAB) {  // this K-split's slab (blockIdx.y; ldc = N)
                const long long off = (long long)blockIdx.y * p.M * p.ldc + (long long)m * p.ldc + n;
                *reinterpret_cast<float4*>((float*)p.C + off) =
                    make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
            } else {
                epilogue<EPI>(p, m, n, acc[a][b]);
            }
        }
    }
}
}  // namespace bf

// ============================================================================ bf16 GEMM, 256x256
// The large-shape path (every ViT-B/L/H training GEMM): 256x256x64 block tile, 512 threads =
// 8 waves (2 M x 4 N), 128x64 per wave = 8x4 v_mfma_f32_16x16x32_bf16 tiles; operands staged by
// global_load_lds (16 B, LDS-DMA, no VGPR round trip) into a double-buffered 128 KiB LDS ring.
// LDS images are lane-linear (the DMA writes base + 16*lane); bank conflicts are removed by
// XOR-permuting the 16-B chunks on the global SOURCE address and reading through the same
// involution (cdna_hip_programming.md §5.4 rule 21), with the swizzles chosen by
// tools/lds_banks.py:
//   K-contig image  [256 rows][64 k]  (128 B rows): chunk' = chunk ^ (row & 7)  -> ds_read_b128
//                                                     fragments conflict free
//   M/N-contig image [64 k][256 cols] (512 B rows): chunk' = chunk ^ f(k),
//       f(k) = (k&3)<<2 | ((k>>3)&1)<<1             -> ds_read_b64_tr_b16 conflict free
// Fragments use the standard 16x16x32 map (lane (i,g): k = 8g + j); rows/cols past M/N are
// clamped on load (they only feed masked outputs); K must be a multiple of 64.
namespace g2 {
constexpr int BM = 256, BN = 256, BK = 32, NT = 512;
constexpr int IMG_BYTES = 256 * BK * 2;    // 16 KiB per operand per slot
constexpr int SLOT_BYTES = 2 * IMG_BYTES;  // 32 KiB (A | B)
constexpr int KTILE = 64;                  // K granularity required of callers (and split chunks)

// K-contig image: [256 rows][32 k] = 64 B rows, 4 chunks; swizzle chunk' = chunk ^ ((row>>1)&3)
__device__ __forceinline__ int kc_swz(int row) { return (row >> 1) & 3; }
// M/N-contig image: [32 k][256 cols] = 512 B rows; swizzle chunk' = chunk ^ f(k)
__device__ __forceinline__ int mn_swz(int k) { return ((k & 3) << 2) | (((k >> 3) & 1) << 1); }

// this thread's 2 LDS-DMA pieces of one operand image (wave w, piece j -> 1 KiB block j*8+w)
template <bool KC>
__device__ __forceinline__ void stage(const bf16_t* __restrict__ base, long long ld, int row0,
                                      int rows_lim, int k0, char* img, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int blk = j * 8 + wave;
        const bf16_t* src;
        if constexpr (KC) {
            const int row = blk * 16 + (lane >> 2);
            const int c = (lane & 3) ^ kc_swz(row);
            const int gr = min(row0 + row, rows_lim - 1);
            src = base + (long long)gr * ld + k0 + c * 8;
        } else {
            const int k = blk * 2 + (lane >> 5);
            const int c = (lane & 31) ^ mn_swz(k);
            const int gc = min(row0 + c * 8, rows_lim - 8);
            src = base + (long long)(k0 + k) * ld + gc;
        }
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(img + blk * 1024),
                                         16, 0, 0);
    }
}

// 8 bf16 of rows/cols [r0, r0+16) for the slot's 32-deep k: lane (i,g) gets k = 8g + j
template <bool KC>
__device__ __forceinline__ bf16x8_t frag(const char* img, int r0, int lane) {
    const int i = lane & 15, g = lane >> 4;
    if constexpr (KC) {
        const int r = r0 + i;
        return *reinterpret_cast<const bf16x8_t*>(img + r * 64 + ((g ^ kc_swz(r)) << 4));
    } else {
        const int q = i >> 2, p = i & 3;
        const int ch = (r0 >> 3) + (p >> 1);
        const int k0 = 8 * g + q, k1 = k0 + 4;
        // k1 = k0 + 4 lies in k0's 8-row group, so mn_swz(k1) == mn_swz(k0): a1 = a0 + 4 rows
        (void)k1;
        const char* a0 = img + k0 * 512 + ((ch ^ mn_swz(k0)) << 4) + (p & 1) * 8;
        const bf16x4_t lo = ds_read_tr16_asm<0>(a0);
        const bf16x4_t hi = ds_read_tr16_asm<4 * 512>(a0);
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
}

// instruction interleave hints (LLVM SchedGroupMask: MFMA 0x8, VMEM_READ 0x20, DS_READ 0x100)
__device__ __forceinline__ void sched_phase0() {  // 4 A-fragment reads among 16 MFMAs
#pragma unroll
    for (int j = 0; j < 4; j++) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 4, 0);
    }
}
__device__ __forceinline__ void sched_phase1() {  // 4 LDS-DMA pieces + 8 fragment reads among 16 MFMAs
#pragma unroll
    for (int j = 0; j < 4; j++) {
        __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, 4, 0);
    }
}

__device__ __forceinline__ void barrier_lds() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Pipeline (cdna_hip_programming.md §5 8-phase template, adapted): each 32-deep K-step is two
// phases of 16 MFMAs per wave; every phase is [A: LDS fragment reads + 2 LDS-DMA pieces] barrier
// [B: MFMAs] barrier.  Waves 4-7 (the SIMD partners of waves 0-3) run one barrier behind, so on
// every SIMD one wave is in its MFMA region while its partner issues reads and DMA.  Ring of
// NSLOT slots, DMA two steps ahead; a wave retires its own pieces of step s+1 (vmcnt) in phase 1
// of step s, two barriers (three with the stagger) before anyone reads them; a slot is refilled
// >= 6 barriers after its last read; every barrier is preceded by lgkmcnt(0).
// DEPTH = K-steps of LDS-DMA in flight ahead of the step being read (ring of DEPTH + 2 slots:
// a slot is refilled >= 2 steps after its last read).  Depth 2 (4 x 32 KiB) is the default:
// depth 3 (5 slots, 160 KiB) measured ~10 % slower on every trainer GEMM (tools/bench_gemm.py
// --modes 0,4).  The DMA of steps past the tile's K range is not issued, so the counted waits
// below drop to the pieces that are.
template <int DEPTH>
constexpr int smem_bytes() {
    return (DEPTH + 2) * SLOT_BYTES > 8 * STG_WAVE_BYTES ? (DEPTH + 2) * SLOT_BYTES : 8 * STG_WAVE_BYTES;
}
// s_waitcnt vmcnt(n) for the counts the pipeline uses (the immediate must be a literal)
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}
template <bool AK, bool BKC, int EPI, int DEPTH>
__global__ __launch_bounds__(NT, 1) void gemm_kernel(GemmParams p) {
    constexpr int NS = DEPTH + 2;
    __shared__ __attribute__((aligned(1024))) char smem[smem_bytes<DEPTH>()];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    first_round_stagger(p.stagger, true);
    trace_stamp(p, 0);
    const int ntm = cdiv(p.M, BM), ntn = cdiv(p.N, BN);
    int wg, split;
    split_remap(ntm * ntn, wg, split);
    const int tm0 = (wg / ntn) * BM, tn0 = (wg % ntn) * BN;
    const int kbeg = split * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);
    const int nk = (kend - kbeg) / BK;
    const bf16_t* A = (const bf16_t*)p.A;
    const bf16_t* B = (const bf16_t*)p.B;
    const bool do_db = !AK && p.dbias != nullptr && tn0 == 0;
    float dbacc = 0.f;

    f32x4_t acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    auto slot_of = [&](int st) { return smem + (st % NS) * SLOT_BYTES; };
    auto issue_a = [&](int st) {  // A-image pieces of step st (none past the K range)
        if (st < nk) stage<AK>(A, p.lda, tm0, p.M, kbeg + st * BK, slot_of(st), wave, lane);
    };
    auto issue_b = [&](int st) {
        if (st < nk) stage<BKC>(B, p.ldb, tn0, p.N, kbeg + st * BK, slot_of(st) + IMG_BYTES, wave, lane);
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    auto mfma_half = [&](int half, const bf16x8_t (&fa)[4], const bf16x8_t (&fb)[4]) {
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 4; b++)
                acc[half * 4 + a][b] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b], fa[a], acc[half * 4 + a][b], 0, 0, 0);
    };
    auto bias_sum = [&](int kt) {
        if constexpr (!AK) {
            if (do_db) {  // fused bias gradient: column sums of this A image (rows of dW)
                const char* imgA = slot_of(kt);
                const int m = tid & 255, kh = (tid >> 8) * 16;
#pragma unroll
                for (int kk = 0; kk < 16; kk++) {
                    const int k = kh + kk;
                    const int c = (m >> 3) ^ mn_swz(k);
                    dbacc += bf2f(*reinterpret_cast<const bf16_t*>(imgA + k * 512 + c * 16 + (m & 7) * 2));
                }
            }
        }
    };

    const bool lagging = wave >= 4;
    if (nk > 0) {
#pragma unroll
        for (int st = 0; st < DEPTH; st++) { issue_a(st); issue_b(st); }
        wait_vm(4 * (min(DEPTH, nk) - 1));  // own pieces of step 0
        bar();
        trace_stamp(p, 12);
        if (lagging) {
            __builtin_amdgcn_s_setprio(1);  // static priority for the younger half (T5)
            bar();                          // stagger: one barrier behind waves 0-3
        }
    }
    bf16x8_t fb[4], alo[4], ahi[4];
    for (int kt = 0; kt < nk; kt++) {
        const char* img = slot_of(kt);
        // ---- phase 0
#pragma unroll
        for (int b = 0; b < 4; b++) fb[b] = frag<BKC>(img + IMG_BYTES, wn * 64 + b * 16, lane);
#pragma unroll
        for (int a = 0; a < 4; a++) alo[a] = frag<AK>(img, wm * 128 + a * 16, lane);
        issue_a(kt + DEPTH);
        bar();
        mfma_half(0, alo, fb);
        bar();
        // ---- phase 1
#pragma unroll
        for (int a = 0; a < 4; a++) ahi[a] = frag<AK>(img, wm * 128 + (4 + a) * 16, lane);
        bias_sum(kt);
        // own pieces of step kt+1 landed: the younger ones are steps kt+2 .. kt+DEPTH-1 (4 each)
        // and the A half of step kt+DEPTH (2), as far as they were issued
        wait_vm(4 * max(0, min(kt + DEPTH, nk) - (kt + 2)) + (kt + DEPTH < nk ? 2 : 0));
        issue_b(kt + DEPTH);
        bar();
        mfma_half(1, ahi, fb);
        bar();
    }
    if (nk > 0 && !lagging) bar();  // balance the stagger barrier
    trace_stamp(p, 1);
    float bpre[8];  // the epilogue's bias columns, loaded under the trailing DMA wait
    staged_bias_prefetch<EPI>(p, lane, tn0 + wn * 64, bpre);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // retire the trailing re-staged pieces
    __builtin_amdgcn_s_setprio(0);
    if constexpr (!AK) {
        if (do_db) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            float* red = reinterpret_cast<float*>(smem);
            red[tid] = dbacc;
            __syncthreads();
            if (tid < 256 && tm0 + tid < p.M) atomicAdd(p.dbias + tm0 + tid, red[tid] + red[tid + 256]);
        }
    }

    if (skip_epilogue(p, acc)) return;
    // every wave's LDS-DMA retired and its reads done before the ring becomes staging space
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    staged_epilogue<EPI>(p, acc, smem + wave * STG_WAVE_BYTES, lane, tm0 + wm * 128, tn0 + wn * 64, bpre);
    trace_stamp(p, 2);
}

// Persistent streaming form (variant 7; K-contiguous A and B: the forward and input-gradient
// GEMMs, no split-K).  One workgroup per CU walks its tiles (round j: the tile the one-tile kernel
// gives block j * 256 + blockIdx.x, so the XCD / L2 placement is unchanged) with the LDS-DMA ring
// streaming across tile boundaries: the DMA of "step kt + 2" in a tile's last two steps fetches
// the NEXT tile's steps 0 and 1, which land during this tile's epilogue.  The per-tile trace
// (tools/gemm_trace.py) of the one-tile kernel showed ~3 us per tile from launch to the first
// operands (every CU starting a tile at once) and the epilogue running with nothing else on the
// CU.  The epilogue stages through the tile's last two slots (free once every wave has read them):
// 8 KiB per wave, four 32-row passes (staged_epilogue_q), while the next tile's first two steps
// sit in the other two.  Waits: before the epilogue vmcnt(0) retires the next tile's steps 0 and
// 1 (so the epilogue's own loads and stores are never waited for by a wait meant for a DMA piece,
// except in phase 1 of the next tile's second step, when those have long completed).  Same MFMA
// order per accumulator and the same epilogue arithmetic as gemm_kernel: bit-identical outputs.
// TS (variant 10): the tiles of the full rounds (p.tfull) as above, then the last round's tiles split
// into p.tsplit K-ranges of p.kchunk (work items tfull + u * tsplit + part, part-major per tile), each
// storing its raw fp32 accumulators as a 256x256 partial tile (tpart); gemm_tail_fix_k adds the parts
// in order and applies the epilogue.  The tail round then keeps every CU busy instead of 1/3 of them.
template <int EPI, bool TS = false>
__global__ __launch_bounds__(NT, 1) void gemm_kernel_s(GemmParams p) {
    constexpr int NS = 4;  // DMA two steps ahead
    __shared__ __attribute__((aligned(1024))) char smem[NS * SLOT_BYTES];
    static_assert(8 * 8192 <= 2 * SLOT_BYTES, "epilogue staging: two slots");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int ntm = cdiv(p.M, BM), ntn = cdiv(p.N, BN), tiles = ntm * ntn;
    const int nblk = gridDim.x;
    const int items = TS ? p.tfull + (tiles - p.tfull) * p.tsplit : tiles;
    const int my_tiles = (items - (int)blockIdx.x + nblk - 1) / nblk;
    const int nk_all = p.K / BK;
    const char* A = (const char*)p.A;
    const char* B = (const char*)p.B;
    f32x4_t acc[8][4];
    auto zero_acc = [&]() {
#pragma unroll
        for (int a = 0; a < 8; a++)
#pragma unroll
            for (int b = 0; b < 4; b++) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    };
    zero_acc();
    if (my_tiles <= 0) return;
    first_round_stagger(p.stagger, true);
    // the lane's DMA source of piece j of the A / B image of a tile, as a 32-bit byte offset from
    // the operand base at k = 0 (K-contiguous image: as stage<true>; host: M*lda, N*ldb < 2^31)
    struct TileSrc {
        int tm0, tn0, t, kbeg, nk, part;  // part: index of the partial tile (TS tail items), else -1
        uint32_t a[2], b[2];
    };
    auto tile_src = [&](int j, TileSrc& ts) {
        const int it = j * nblk + (int)blockIdx.x;
        ts.kbeg = 0;
        ts.nk = nk_all;
        ts.part = -1;
        if (!TS || it < p.tfull) {
            ts.t = xcd_remap(it, TS ? p.tfull : tiles);
        } else {
            const int v = it - p.tfull, u = v / p.tsplit;
            ts.t = p.tfull + u;
            ts.part = v;
            ts.kbeg = (v - u * p.tsplit) * p.kchunk;
            ts.nk = (min(p.K, ts.kbeg + p.kchunk) - ts.kbeg) / BK;  // host: >= 2 steps
        }
        if (!TS && p.gm > 0) {  // (the split-tail variant keeps the row-major order its fix-up assumes)
            // groups of gm row panels walked column by column: the tiles an XCD runs at once share
            // gm A panels and 32 / gm B panels instead of ~3 A panels and every B panel
            const int per = p.gm * ntn, g = ts.t / per, r = ts.t - g * per, rows = min(p.gm, ntm - g * p.gm);
            ts.tm0 = (g * p.gm + r % rows) * BM;
            ts.tn0 = (r / rows) * BN;
        } else {
            ts.tm0 = (ts.t / ntn) * BM;
            ts.tn0 = (ts.t % ntn) * BN;
        }
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int row = (q * 8 + wave) * 16 + (lane >> 2);
            const int c = (lane & 3) ^ kc_swz(row);
            ts.a[q] = (uint32_t)((min(ts.tm0 + row, p.M - 1) * p.lda + c * 8) * 2);
            ts.b[q] = (uint32_t)((min(ts.tn0 + row, p.N - 1) * p.ldb + c * 8) * 2);
        }
    };
    TileSrc cur, nxt;
    tile_src(0, cur);
    nxt = cur;
    if (my_tiles > 1) tile_src(1, nxt);
    auto glds = [&](const char* src, char* dst) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    };
    // A / B pieces of step kt2 of the current tile (kt2 >= nk: step kt2 - nk of the next one, if
    // this workgroup has one) into slot sl
    auto issue_a = [&](int kt2, int sl, bool more) {
        const int nk = cur.nk;
        if (kt2 >= nk && !more) return;
        const bool c = kt2 < nk;
        const char* base = A + (long long)(c ? cur.kbeg / BK + kt2 : nxt.kbeg / BK + kt2 - nk) * (BK * 2);
        char* dst = smem + sl * SLOT_BYTES;
#pragma unroll
        for (int q = 0; q < 2; q++) glds(base + (c ? cur.a[q] : nxt.a[q]), dst + (q * 8 + wave) * 1024);
    };
    auto issue_b = [&](int kt2, int sl, bool more) {
        const int nk = cur.nk;
        if (kt2 >= nk && !more) return;
        const bool c = kt2 < nk;
        const char* base = B + (long long)(c ? cur.kbeg / BK + kt2 : nxt.kbeg / BK + kt2 - nk) * (BK * 2);
        char* dst = smem + sl * SLOT_BYTES + IMG_BYTES;
#pragma unroll
        for (int q = 0; q < 2; q++) glds(base + (c ? cur.b[q] : nxt.b[q]), dst + (q * 8 + wave) * 1024);
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    auto mfma_half = [&](int half, const bf16x8_t (&fa)[4], const bf16x8_t (&fb)[4]) {
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 4; b++)
                acc[half * 4 + a][b] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b], fa[a], acc[half * 4 + a][b], 0, 0, 0);
        // the phase's MFMAs stay in front of the barrier that closes it: hipcc's instruction
        // selection otherwise sank 10 of the 16 past it (the wave then reached the barrier early
        // and its partner's read phase overlapped its own MFMAs).  An empty asm naming the 16
        // accumulators orders them; it emits nothing and reads nothing.
        f32x4_t* q = &acc[half * 4][0];
        asm volatile("" ::"v"(q[0]), "v"(q[1]), "v"(q[2]), "v"(q[3]), "v"(q[4]), "v"(q[5]), "v"(q[6]), "v"(q[7]),
                     "v"(q[8]), "v"(q[9]), "v"(q[10]), "v"(q[11]), "v"(q[12]), "v"(q[13]), "v"(q[14]), "v"(q[15]));
    };
    const bool lagging = wave >= 4;
    issue_a(0, 0, false); issue_b(0, 0, false);
    issue_a(1, 1, my_tiles > 1); issue_b(1, 1, my_tiles > 1);  // nk >= 2 (K % 64 == 0)
    wait_vm(4);
    int sl = 0;  // slot of the step being read (global step % 4)
    bf16x8_t fb[4], alo[4], ahi[4];
    for (int j = 0; j < my_tiles; j++) {
        const bool more = j + 1 < my_tiles;
        const int nk = cur.nk;
        if (p.trace && tid == 0) p.trace[(long long)cur.t * TRACE_WORDS] = __builtin_amdgcn_s_memrealtime();
        bar();
        if (lagging) {
            __builtin_amdgcn_s_setprio(1);
            bar();
        }
        for (int kt = 0; kt < nk; kt++) {
            const char* img = smem + sl * SLOT_BYTES;
            const int sl2 = (sl + 2) & 3;
            // ---- phase 0
#pragma unroll
            for (int b = 0; b < 4; b++) fb[b] = frag<true>(img + IMG_BYTES, wn * 64 + b * 16, lane);
#pragma unroll
            for (int a = 0; a < 4; a++) alo[a] = frag<true>(img, wm * 128 + a * 16, lane);
#if VIT_G2_ONEPHASE
            // one phase per step: all 12 fragments read before one barrier, the 32 MFMAs after it
            // (two barriers per step instead of four)
#pragma unroll
            for (int a = 0; a < 4; a++) ahi[a] = frag<true>(img, wm * 128 + (4 + a) * 16, lane);
            issue_a(kt + 2, sl2, more);
            issue_b(kt + 2, sl2, more);
            // own pieces of the next step landed (the one after, 4 pieces, in flight); in a later
            // tile's first step they were retired before the previous epilogue
            if (kt > 0 || j == 0) {
                if (kt + 2 < nk || more) wait_vm(4);
                else wait_vm(0);
            }
            bar();
            mfma_half(0, alo, fb);
            mfma_half(1, ahi, fb);
            bar();
            sl = (sl + 1) & 3;
            continue;
#endif
            issue_a(kt + 2, sl2, more);
            bar();
            mfma_half(0, alo, fb);
            bar();
            // ---- phase 1
#pragma unroll
            for (int a = 0; a < 4; a++) ahi[a] = frag<true>(img, wm * 128 + (4 + a) * 16, lane);
            // own pieces of the next step landed (the A half of the one after stays in flight); in a
            // later tile's first step they were retired before the previous epilogue
            if (kt > 0 || j == 0) {
                if (kt + 2 < nk || more) wait_vm(2);
                else wait_vm(0);
            }
            issue_b(kt + 2, sl2, more);
            bar();
            mfma_half(1, ahi, fb);
            bar();
            sl = (sl + 1) & 3;
        }
        if (!lagging) bar();  // balance the stagger barrier
        if (p.trace && tid == 0) p.trace[(long long)cur.t * TRACE_WORDS + 1] = __builtin_amdgcn_s_memrealtime();
        float bpre[8];
        staged_bias_prefetch<EPI>(p, lane, cur.tn0 + wn * 64, bpre);
        // the next tile's steps 0 and 1 (and the bias) landed; every wave's reads of this tile's
        // last two slots done before they become staging space.  Through the builtin, not asm: hipcc
        // then knows no LDS-DMA is pending after the epilogue and does not put a vmcnt(0) in front
        // of the next tile's first fragment reads (it did: a wait for all of this epilogue's stores)
#if VIT_G2_EPI_WAIT_ASM
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#else
        __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) expcnt(7) lgkmcnt(0), visible to the compiler (below)
#endif
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (!skip_epilogue(p, acc)) {
            // this tile's last two steps were in slots sl - 1, sl - 2 (mod 4)
            char* stg = smem + ((wave < 4 ? sl + 2 : sl + 3) & 3) * SLOT_BYTES + (wave & 3) * 8192;
            if (TS && cur.part >= 0) {
                // raw accumulators into the partial tile in accumulator order (a wave's 32 x 16-B
                // stores cover whole 1 KiB blocks; no staging, no epilogue registers):
                // float4 (wave, a, b, lane) at ((wave * 32 + a * 4 + b) * 64 + lane) * 4
                float* dst = p.tpart + (long long)cur.part * (BM * BN) + wave * 32 * 256 + lane * 4;
#pragma unroll
                for (int a = 0; a < 8; a++)
#pragma unroll
                    for (int b = 0; b < 4; b++) *reinterpret_cast<f32x4_t*>(dst + (a * 4 + b) * 256) = acc[a][b];
            } else {
                staged_epilogue_q<EPI>(p, acc, reinterpret_cast<float*>(stg), lane, cur.tm0 + wm * 128,
                                       cur.tn0 + wn * 64, bpre);
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
        if (p.dbg & 16) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // diagnostic: store drain
        zero_acc();
        // recomputed rather than carried: nothing of the next tiles' sources stays live through the epilogue
        if (more) tile_src(j + 1, cur);
        if (j + 2 < my_tiles) tile_src(j + 2, nxt);
    }
}

// finish of the split tail (variant 10): tile tfull + u = the sum of its tsplit partial tiles in
// part order, then the GEMM's epilogue (bias, fp32 residual or bf16 store) as epilogue8 applies it.
// Block (u, rc): rows 32 rc .. 32 rc + 31 of the tile, thread = (row, 8-column group).
template <int EPI>
__global__ __launch_bounds__(256) void gemm_tail_fix_k(GemmParams p) {
    const int ntn = cdiv(p.N, BN), u = blockIdx.x, t = p.tfull + u;
    const int tm0 = (t / ntn) * BM, tn0 = (t % ntn) * BN;
    const int cg = threadIdx.x & 31, r0 = blockIdx.y * 32 + (threadIdx.x >> 5);
    float cs[8];
#pragma unroll
    for (int it = 0; it < 4; it++) {
        const int r = r0 + it * 8;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        // (r, 8 cg ..) in the accumulator order of gemm_kernel_s: wave (r / 128) * 4 + c / 64, tile
        // a = (r % 128) / 16, b = (c % 64) / 16, lane 16 g + r % 16 with g = (c % 16) / 4
        const int c = cg * 8, wv = (r >> 7) * 4 + (c >> 6), a = (r & 127) >> 4, b = (c & 63) >> 4;
        const int g = (c & 15) >> 2, i = r & 15;
        const long long o0 = ((long long)(wv * 32 + a * 4 + b) * 64 + g * 16 + i) * 4, o1 = o0 + 16 * 4;
        for (int part = 0; part < p.tsplit; part++) {
            const float* q = p.tpart + ((long long)u * p.tsplit + part) * (BM * BN);
            const float4 x0 = *reinterpret_cast<const float4*>(q + o0), x1 = *reinterpret_cast<const float4*>(q + o1);
            v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w;
            v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
        }
        const int m = tm0 + r, n = tn0 + cg * 8;
        if (m >= p.M) continue;
        if (n + 8 <= p.N) {
            epilogue8<EPI, false>(p, m, n, v, cs);
        } else if (n + 4 <= p.N) {
            f32x4_t w = {v[0], v[1], v[2], v[3]};
            epilogue<EPI>(p, m, n, w);
        }
    }
}

}  // namespace g2

// ============================================================================ bf16 GEMM, 256x128
// Two workgroups per CU.  A 256x128x32 block tile on 256 threads = 4 waves (2 M x 2 N), one
// wave per SIMD, 128x64 per wave (8x4 v_mfma_f32_16x16x32_bf16 tiles, as g2).  The LDS ring is
// 3 slots x 24 KiB = 72 KiB, so two workgroups share a CU (144 KiB) and the hardware pairs
// their waves on every SIMD: while one workgroup stores its epilogue (bias / GELU / residual,
// HBM-bound for K = 768) or issues its fragment reads, the other keeps the matrix pipe busy.
// With one 256x256 workgroup per CU those phases ran serialised with the MFMAs, and all CUs hit
// their epilogues at the same moment.  Per K-step: counted vmcnt retires this wave's own pieces
// of step s (step s+1 stays in flight across the barrier), one raw s_barrier, LDS-DMA of step
// s+2 into the slot read at step s-1, 12 fragment reads, 32 MFMAs.
namespace g4 {
constexpr int BM = 256, BN = 128, BK = 32, NT = 256;
constexpr int NSLOT = 3;
constexpr int A_BYTES = BM * BK * 2;           // 16 KiB
constexpr int B_BYTES = BN * BK * 2;           // 8 KiB
constexpr int SLOT_BYTES = A_BYTES + B_BYTES;  // 24 KiB
constexpr int KTILE = BK;                      // K granularity required of callers
constexpr int PIECES = BM / 64 + BN / 64;      // LDS-DMA instructions per wave per K-step (6)
static_assert(PIECES == 6, "vmcnt literal below");
static_assert(NSLOT * SLOT_BYTES >= 4 * STG_WAVE_BYTES, "staged epilogue area");

// K-contig image [R rows][32 k] (64 B rows): 16-B chunk' = chunk ^ ((row >> 1) & 3)
__device__ __forceinline__ int kc_swz(int row) { return (row >> 1) & 3; }
// M/N-contig image [32 k][R] (2R-byte rows): chunk' = chunk ^ f(k), f spreading the 8 k rows a
// 32-lane half of ds_read_b64_tr_b16 touches over distinct 32-B bank groups
template <int R>
__device__ __forceinline__ int mn_swz(int k) {
    if constexpr (R == 256) return ((k & 3) << 2) | (((k >> 3) & 1) << 1);
    else return ((k & 3) << 1) | (((k >> 3) & 1) << 3);
}

// this wave's R/64 one-KiB pieces of an operand image (piece blk = 4j + wave)
template <bool KC, int R>
__device__ __forceinline__ void stage(const bf16_t* __restrict__ base, long long ld, int row0,
                                      int rows_lim, int k0, char* img, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < R / 64; j++) {
        const int blk = j * 4 + wave;
        const bf16_t* src;
        if constexpr (KC) {
            const int row = blk * 16 + (lane >> 2);
            const int c = (lane & 3) ^ kc_swz(row);
            const int gr = min(row0 + row, rows_lim - 1);
            src = base + (long long)gr * ld + k0 + c * 8;
        } else {
            constexpr int CPR = R / 8;             // 16-B chunks per k row
            constexpr int KPB = 64 / CPR;          // k rows per piece
            const int k = blk * KPB + lane / CPR;
            const int c = (lane % CPR) ^ mn_swz<R>(k);
            const int gc = min(row0 + c * 8, rows_lim - 8);
            src = base + (long long)(k0 + k) * ld + gc;
        }
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(img + blk * 1024),
                                         16, 0, 0);
    }
}

// 8 bf16 of rows/cols [r0, r0+16) for the slot's 32-deep k: lane (i,g) gets k = 8g + j
template <bool KC, int R>
__device__ __forceinline__ bf16x8_t frag(const char* img, int r0, int lane) {
    const int i = lane & 15, g = lane >> 4;
    if constexpr (KC) {
        const int r = r0 + i;
        return *reinterpret_cast<const bf16x8_t*>(img + r * 64 + ((g ^ kc_swz(r)) << 4));
    } else {
        const int q = i >> 2, p = i & 3;
        const int ch = (r0 >> 3) + (p >> 1);
        const int k0 = 8 * g + q, k1 = k0 + 4;
        (void)k1;  // mn_swz<R>(k0 + 4) == mn_swz<R>(k0): a1 = a0 + 4 rows
        const char* a0 = img + k0 * (2 * R) + ((ch ^ mn_swz<R>(k0)) << 4) + (p & 1) * 8;
        const bf16x4_t lo = ds_read_tr16_asm<0>(a0);
        const bf16x4_t hi = ds_read_tr16_asm<4 * 2 * R>(a0);
        return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
}

// tile order inside the XCD-contiguous range: groups of GM M-tiles walked column by column, so
// the workgroups resident on one XCD share a few A panels and a few B panels in its L2
__device__ __forceinline__ void group_order(int t, int ntm, int ntn, int& tm, int& tn) {
    constexpr int GM = 8;
    const int per = GM * ntn;
    const int grp = t / per;
    const int first = grp * GM;
    const int gsz = min(GM, ntm - first);
    const int r = t - grp * per;
    tm = first + r % gsz;
    tn = r / gsz;
}

template <bool AK, bool BKC, int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(GemmParams p) {
    __shared__ __attribute__((aligned(1024))) char smem[NSLOT * SLOT_BYTES];
    first_round_stagger(p.stagger);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int ntm = cdiv(p.M, BM), ntn = cdiv(p.N, BN);
    int tm, tn, wg, split;
    split_remap(ntm * ntn, wg, split);
    group_order(wg, ntm, ntn, tm, tn);
    const int tm0 = tm * BM, tn0 = tn * BN;
    const int kbeg = split * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);
    const int nk = (kend - kbeg) / BK;
    const bf16_t* A = (const bf16_t*)p.A;
    const bf16_t* B = (const bf16_t*)p.B;

    f32x4_t acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    auto issue = [&](int st) {
        char* sl = smem + (st % NSLOT) * SLOT_BYTES;
        const int k0 = kbeg + st * BK;
        stage<AK, BM>(A, p.lda, tm0, p.M, k0, sl, wave, lane);
        stage<BKC, BN>(B, p.ldb, tn0, p.N, k0, sl + A_BYTES, wave, lane);
    };
    if (nk > 0) issue(0);
    if (nk > 1) issue(1);
    for (int kt = 0; kt < nk; kt++) {
        // this wave's pieces of step kt have landed (step kt+1's stay in flight); its reads of
        // step kt-1 are done; after the barrier both hold for every wave
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 2 < nk) issue(kt + 2);  // into the slot of step kt-1
        const char* img = smem + (kt % NSLOT) * SLOT_BYTES;
        bf16x8_t fa[8], fb[4];
#pragma unroll
        for (int b = 0; b < 4; b++) fb[b] = frag<BKC, BN>(img + A_BYTES, wn * 64 + b * 16, lane);
#pragma unroll
        for (int a = 0; a < 8; a++) fa[a] = frag<AK, BM>(img, wm * 128 + a * 16, lane);
        if constexpr (!AK || !BKC) {  // asm transposed reads are not counted by the compiler
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int a = 0; a < 8; a++)
#pragma unroll
            for (int b = 0; b < 4; b++)
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b], fa[a], acc[a][b], 0, 0, 0);
    }

    if (skip_epilogue(p, acc)) return;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    staged_epilogue<EPI>(p, acc, smem + wave * STG_WAVE_BYTES, lane, tm0 + wm * 128, tn0 + wn * 64);
}

// Software-pipelined form (variant 5; K-contiguous A and B: every forward and input-gradient GEMM
// of the trainer).  The kernel above reads a K-step's 12 fragments and then issues its 32 MFMAs, so
// a wave alone on its SIMD leaves the matrix pipe idle for the read latency of every step: it
// relies on the other resident workgroup's wave to fill those gaps, and while that workgroup runs
// its epilogue (GELU pair, fp32 residual: up to 40 % of a heavy-epilogue launch) nothing does.
// Here a wave's reads run under its own MFMAs, so one wave keeps its SIMD's matrix pipe busy and
// the two workgroups of a CU hide each other's epilogues.  Each K-step is two phases of 16 MFMAs:
//   phase 0: MFMAs of A rows 0-63 (alo) x B (fb)   ||  reads of A rows 64-127 (ahi) of step s
//   [vmcnt: own pieces of s+1 landed; lgkmcnt(0); barrier; DMA of step s+3 into slot s % 3]
//   phase 1: MFMAs of ahi x fb                      ||  reads of fb, alo of step s+1
// so the fragments in flight cost 16 + 16 VGPRs beyond one step's 48 (two named B sets, the loop
// unrolled by two).  Ring of 3 slots, DMA three steps ahead.  After step s's barrier every wave
// has read all of slot s (lgkmcnt(0) before it) and its own pieces of s+1 have landed (s+2's stay
// in flight: vmcnt(6)), so slot s+1 is readable by all and slot s takes step s+3.  The DMA
// sources are one 32-bit byte offset per piece from the scalar operand base (6 VGPRs).
template <int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_kernel_pipe(GemmParams p) {
    __shared__ __attribute__((aligned(1024))) char smem[NSLOT * SLOT_BYTES];
    first_round_stagger(p.stagger);
    trace_stamp(p, 0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int ntm = cdiv(p.M, BM), ntn = cdiv(p.N, BN);
    int tm, tn, wg, split;
    split_remap(ntm * ntn, wg, split);
    group_order(wg, ntm, ntn, tm, tn);
    const int tm0 = tm * BM, tn0 = tn * BN;
    const int kbeg = split * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);
    const int nk = (kend - kbeg) / BK;
    const char* A = (const char*)p.A;
    const char* B = (const char*)p.B;

    f32x4_t acc[8][4];
#pragma unroll
    for (int a = 0; a < 8; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // per-piece byte offsets of this lane's 16-B DMA source (K-contig image, as stage<true, R>)
    uint32_t offa[BM / 64], offb[BN / 64];
#pragma unroll
    for (int j = 0; j < BM / 64; j++) {
        const int row = (j * 4 + wave) * 16 + (lane >> 2);
        const int c = (lane & 3) ^ kc_swz(row);
        offa[j] = (uint32_t)(((long long)min(tm0 + row, p.M - 1) * p.lda + c * 8) * 2);
    }
#pragma unroll
    for (int j = 0; j < BN / 64; j++) {
        const int row = (j * 4 + wave) * 16 + (lane >> 2);
        const int c = (lane & 3) ^ kc_swz(row);
        offb[j] = (uint32_t)(((long long)min(tn0 + row, p.N - 1) * p.ldb + c * 8) * 2);
    }
    auto issue = [&](int st) {
        char* sl = smem + (st % NSLOT) * SLOT_BYTES;
        const long long kb = (long long)(kbeg + st * BK) * 2;
        const char* a0 = A + kb;
        const char* b0 = B + kb;
#pragma unroll
        for (int j = 0; j < BM / 64; j++)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(a0 + offa[j]),
                                             (__attribute__((address_space(3))) void*)(sl + (j * 4 + wave) * 1024),
                                             16, 0, 0);
#pragma unroll
        for (int j = 0; j < BN / 64; j++)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(b0 + offb[j]),
                                             (__attribute__((address_space(3))) void*)(sl + A_BYTES + (j * 4 + wave) * 1024),
                                             16, 0, 0);
    };
    // fragment reads as inline asm (ds_read_b128, immediate offsets): the compiler neither counts
    // nor waits for them, the phases below do (hipcc's own counting put lgkmcnt(0) in front of
    // phase 0, waiting for the reads meant to run under its MFMAs).  Lane (i, g) of a 16-row
    // fragment at rows r0 + i: kc_swz(r0 + i) = (i >> 1) & 3 for r0 % 16 == 0, so one lane address
    // per operand and slot, the fragments at + 1 KiB each.
    const uint32_t lds0 = (uint32_t)(uintptr_t)LDS_PTR(char, smem);
    const uint32_t a_lane = lds0 + (wm * 128 + (lane & 15)) * 64 + (((lane >> 4) ^ kc_swz(lane & 15)) << 4);
    const uint32_t b_lane = lds0 + A_BYTES + (wn * 64 + (lane & 15)) * 64 + (((lane >> 4) ^ kc_swz(lane & 15)) << 4);
    auto read_b = [&](int st, bf16x8_t (&fb)[4]) {
        const uint32_t o = b_lane + (st % NSLOT) * SLOT_BYTES;
        asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\t"
                     "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072"
                     : "=&v"(fb[0]), "=&v"(fb[1]), "=&v"(fb[2]), "=&v"(fb[3]) : "v"(o));
    };
    auto read_a = [&](int st, int half, bf16x8_t (&fa)[4]) {
        const uint32_t o = a_lane + (st % NSLOT) * SLOT_BYTES + half * 4096;
        asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\t"
                     "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072"
                     : "=&v"(fa[0]), "=&v"(fa[1]), "=&v"(fa[2]), "=&v"(fa[3]) : "v"(o));
    };
    auto mfma16 = [&](int half, const bf16x8_t (&fa)[4], const bf16x8_t (&fb)[4]) {
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 4; b++)
                acc[half * 4 + a][b] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b], fa[a], acc[half * 4 + a][b], 0, 0, 0);
    };
    bf16x8_t alo[4], ahi[4], fbA[4], fbB[4];
    // step s with B fragments cb (read in the previous step) and the next step's into nb
    auto step = [&](int s, const bf16x8_t (&cb)[4], bf16x8_t (&nb)[4]) {
        // phase 0: alo x cb, ahi of step s read underneath (reads issued first)
        __builtin_amdgcn_sched_barrier(0);
        read_a(s, 1, ahi);
        // the 8 reads of the previous phase (cb, alo) are done, this phase's 4 (ahi) stay in flight
        asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        mfma16(0, alo, cb);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 2 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (s + 3 < nk) issue(s + 3);  // into slot s % 3: every wave has read all of it
        __builtin_amdgcn_sched_barrier(0);
        // phase 1: ahi x cb, step s+1's fb and alo read underneath (unconditionally: past the
        // last step the slot holds stale data nobody uses and no DMA writes it, and straight-line
        // reads keep the compiler's lgkmcnt tracking exact)
        read_b(s + 1, nb);
        read_a(s + 1, 0, alo);
        __builtin_amdgcn_sched_barrier(0);
        mfma16(1, ahi, cb);  // ahi: retired by the lgkmcnt(0) in front of the barrier
        __builtin_amdgcn_sched_barrier(0);
    };

    if (nk > 0) {
        issue(0);
        if (nk > 1) issue(1);
        if (nk > 2) issue(2);
        // own pieces of step 0 landed (1 and 2 stay in flight), then fb, alo of step 0
        __builtin_amdgcn_sched_barrier(0);
        if (nk > 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else if (nk > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        trace_stamp(p, 12);
        read_b(0, fbA);
        read_a(0, 0, alo);
        __builtin_amdgcn_sched_barrier(0);
    }
    for (int kt = 0; kt < nk; kt += 2) {  // nk is even (host: K and the split chunk % 64 == 0)
        step(kt, fbA, fbB);
        step(kt + 1, fbB, fbA);
    }
    trace_stamp(p, 1);

    if (skip_epilogue(p, acc)) return;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    staged_epilogue<EPI>(p, acc, smem + wave * STG_WAVE_BYTES, lane, tm0 + wm * 128, tn0 + wn * 64);
    trace_stamp(p, 2);
}
}  // namespace g4

// ============================================================================ fp32 MFMA GEMM
namespace f32 {
constexpr int BM = 64, BN = 64, BK = 16, NT = 256, S = 80;  // S: LDS row stride (floats)

template <int EPI>
__global__ __launch_bounds__(NT) void gemm_f32_kernel(GemmParams p, int a_kc, int b_kc) {
    __shared__ float As[BK * S];
    __shared__ float Bs[BK * S];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int ntm = cdiv(p.M, BM), ntn = cdiv(p.N, BN);
    const int wg = blockIdx.x;
    const int tm0 = (wg / ntn) * BM, tn0 = (wg % ntn) * BN;
    (void)ntm;
    const int kbeg = blockIdx.y * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);
    const float* A = (const float*)p.A;
    const float* B = (const float*)p.B;
    f32x4_t acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    for (int k0 = kbeg; k0 < kend; k0 += BK) {
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int idx = e * NT + tid;
            int m, k;
            if (a_kc) { m = idx >> 4; k = idx & 15; } else { k = idx >> 6; m = idx & 63; }
            const int gm = tm0 + m, gk = k0 + k;
            float v = 0.f;
            if (gm < p.M && gk < kend)
                v = a_kc ? A[(long long)gm * p.lda + gk] : A[(long long)gk * p.lda + gm];
            As[k * S + m] = v;
            int n;
            if (b_kc) { n = idx >> 4; k = idx & 15; } else { k = idx >> 6; n = idx & 63; }
            const int gn = tn0 + n;
            const int gk2 = k0 + k;
            float w = 0.f;
            if (gn < p.N && gk2 < kend)
                w = b_kc ? B[(long long)gn * p.ldb + gk2] : B[(long long)gk2 * p.ldb + gn];
            Bs[k * S + n] = w;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < BK / 4; kk++) {
            const int kr = kk * 4 + (lane >> 4);
            float af[2], bfv[2];
#pragma unroll
            for (int t = 0; t < 2; t++) {
                af[t] = As[kr * S + wm * 32 + t * 16 + (lane & 15)];
                bfv[t] = Bs[kr * S + wn * 32 + t * 16 + (lane & 15)];
            }
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int b = 0; b < 2; b++)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a], bfv[b], acc[a][b], 0, 0, 0);
        }
        __syncthreads();
    }
    // C layout: row = (lane>>4)*4 + r, col = lane&15
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int m = tm0 + wm * 32 + a * 16 + (lane >> 4) * 4 + r;
                const int n = tn0 + wn * 32 + b * 16 + (lane & 15);
                if (m >= p.M || n >= p.N) continue;
                float v = acc[a][b][r];
                float* q = (float*)p.C + (long long)m * p.ldc + n;
                if constexpr (EPI == EPI_F32_STORE) {
                    *q = p.bias ? v + p.bias[n] : v;
                } else if constexpr (EPI == EPI_F32_ACC) {
                    *q += p.bias ? v + p.bias[n] : v;
                } else {  // EPI_F32_SLAB: this K-split's slab (p.C = slab base, ldc = N)
                    q[(long long)blockIdx.y * p.M * p.ldc] = v;
                }
            }
}
}  // namespace f32

// ============================================================================ column sums
// part[blockIdx.y][n] = sum of rows blockIdx.y*rpb .. +rpb-1 of column n (ascending); with
// add_direct the single row block adds straight into out (one add per column: deterministic)
template <typename TX>
__global__ __launch_bounds__(256) void colsum_part_k(float* __restrict__ out, const TX* __restrict__ X, int M, int N,
                                                     long long ld, int rpb, int add_direct) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    const int r0 = blockIdx.y * rpb;
    const int r1 = min(M, r0 + rpb);
    if (n >= N) return;
    float s = 0.f;
    for (int r = r0; r < r1; r++) {
        if constexpr (sizeof(TX) == 2)
            s += bf2f(X[(long long)r * ld + n]);
        else
            s += X[(long long)r * ld + n];
    }
    if (add_direct) out[n] += s;
    else out[(long long)blockIdx.y * N + n] = s;
}

// rows_reduce_add.  Vector form (ncols, ld % 4 == 0, 16-B aligned src): a workgroup takes 64
// columns of one job as 16 float4 lanes x 16 row phases; phase p sums rows p, p+16, ... in two
// interleaved chains (rows p+32i and p+16+32i), then the 16 phases are added in ascending order.
// Scalar form otherwise: 64 columns x 4 phases.  Both orders are fixed: deterministic.
struct RowsJobs {
    RowsJob j[ROWS_MAX_JOBS];
    int blk0[ROWS_MAX_JOBS + 1];
    int vec;
};
__global__ __launch_bounds__(256) void rows_reduce_k(RowsJobs jobs) {
    __shared__ float4 red[16][17];
    int jb = 0;
#pragma unroll 1
    while (jb + 1 < ROWS_MAX_JOBS && (int)blockIdx.x >= jobs.blk0[jb + 1]) jb++;
    const RowsJob& J = jobs.j[jb];
    const int c0 = (blockIdx.x - jobs.blk0[jb]) * 64;
    if (jobs.vec) {
        const int q = threadIdx.x & 15, ph = threadIdx.x >> 4, c = c0 + 4 * q;
        float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
        if (c < J.ncols) {
            const float* base = J.src + c;
            int r = ph;
            for (; r + 16 < J.nrows; r += 32) {
                const float4 a = *reinterpret_cast<const float4*>(base + (long long)r * J.ld);
                const float4 b = *reinterpret_cast<const float4*>(base + (long long)(r + 16) * J.ld);
                s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
                s1.x += b.x; s1.y += b.y; s1.z += b.z; s1.w += b.w;
            }
            if (r < J.nrows) {
                const float4 a = *reinterpret_cast<const float4*>(base + (long long)r * J.ld);
                s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
            }
        }
        red[ph][q] = make_float4(s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w);
        __syncthreads();
        if (threadIdx.x < 64) {
            const int qq = threadIdx.x >> 2, e = threadIdx.x & 3, cc = c0 + threadIdx.x;
            float t = 0.f;
#pragma unroll
            for (int p = 0; p < 16; p++) t += reinterpret_cast<const float*>(&red[p][qq])[e];
            if (cc < J.ncols) J.dst[cc] += t;
        }
        return;
    }
    float* reds = reinterpret_cast<float*>(red);  // [4][64]
    const int c = c0 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
    float s0 = 0.f, s1 = 0.f;
    if (c < J.ncols) {
        int r = ph;
        for (; r + 4 < J.nrows; r += 8) {  // two chains: rows ph+8i and ph+4+8i
            s0 += J.src[(long long)r * J.ld + c];
            s1 += J.src[(long long)(r + 4) * J.ld + c];
        }
        if (r < J.nrows) s0 += J.src[(long long)r * J.ld + c];
    }
    reds[ph * 64 + (threadIdx.x & 63)] = s0 + s1;
    __syncthreads();
    if (ph == 0 && c < J.ncols)
        J.dst[c] += ((reds[threadIdx.x] + reds[64 + threadIdx.x]) + reds[128 + threadIdx.x]) + reds[192 + threadIdx.x];
}
void rows_reduce_add(const RowsJob* jobs, int njobs, hipStream_t s) {
    for (int b = 0; b < njobs; b += ROWS_MAX_JOBS) {
        RowsJobs J{};
        J.vec = 1;
        int nb = 0, k = 0;
        for (; k < ROWS_MAX_JOBS && b + k < njobs; k++) {
            const RowsJob& x = jobs[b + k];
            J.j[k] = x;
            J.blk0[k] = nb;
            nb += x.nrows > 0 ? cdiv(x.ncols, 64) : 0;
            if (x.nrows > 0 && ((x.ncols | x.ld) % 4 || ((uintptr_t)x.src & 15))) J.vec = 0;
        }
        for (; k <= ROWS_MAX_JOBS; k++) J.blk0[k] = nb;
        if (nb == 0) continue;
        rows_reduce_k<<<nb, 256, 0, s>>>(J);
        after_launch("rows_reduce_add");
    }
}
template <typename TX>
static void colsum_any(float* dbias, const TX* X, int M, int N, long long ld, hipStream_t s, float* ws) {
    if (M <= 0 || N <= 0) return;
    if constexpr (sizeof(TX) == 4) {
        // few fp32 rows (the trainer's M = B head column sums): the fixed-order rows reduce, 16 row
        // phases x 64 columns per workgroup, instead of one thread per column walking all M rows
        // (4 / 3 workgroups, 30-60 us at B = 256 on the backward's critical path)
        if (M <= 1024) {
            RowsJob j{dbias, X, M, ld, N};
            rows_reduce_add(&j, 1, s);
            return;
        }
    }
    const int rpb = 256, nch = cdiv(M, rpb);
    if (nch == 1) {
        colsum_part_k<TX><<<dim3(cdiv(N, 256), 1), 256, 0, s>>>(dbias, X, M, N, ld, rpb, 1);
        after_launch("colsum");
        return;
    }
    if (!ws) ws = (float*)workspace((size_t)nch * N * sizeof(float));
    if (!ws) return;
    colsum_part_k<TX><<<dim3(cdiv(N, 256), nch), 256, 0, s>>>(ws, X, M, N, ld, rpb, 0);
    after_launch("colsum");
    RowsJob j{dbias, ws, nch, N, N};
    rows_reduce_add(&j, 1, s);
}
static int gemm_variant();
// debug flag 512: variant 11 takes every shape gemm_pp_shape accepts (A/B measurements, tests)
static int g_debug_flags_fwd();
static bool pp_all() { return (g_debug_flags_fwd() & 512) != 0; }
// the ping-pong engine (variant 11) takes this bf16 GEMM: the big-tile path of gemm_bf16 without
// split-K, on a shape gemm_pp_shape accepts
// (the output width C GEMMs only, N <= 1280: proj / fcproj forward and every input gradient.  Measured
// per GEMM at ViT-B/16 against the streaming engine (tools/bench_gemm.py --variants 7,11): those run
// 4-15 % faster — their N = 768 grids quantize better in 192-row tiles and the fp32-residual epilogue
// hides behind the next tile — while the K = 768 GEMMs with the heavy GELU-pair / x-aux epilogues and
// N = 2304 / 3072 run 5-15 % slower: the epilogue group then cannot keep pace with one MFMA wave per
// SIMD)
static bool pp_taken(const GemmArgs& a) {
    return gemm_variant() == 11 && !a.a_scale && a.epi != EPI_F32_ATOMIC && gemm_bf16_supported(a) &&
           a.K % g2::KTILE == 0 && a.M >= 256 && a.N >= 256 && (a.N <= 1280 || pp_all()) && gemm_pp_shape(a);
}
int gemm_colsum_rows(const GemmArgs& a, bool fp8) { return cdiv(a.M, !fp8 && pp_taken(a) ? 96 : 128); }
float* colsum_rows_begin(const GemmArgs& a) {
    if (!epi_aux16(a.epi) || !(a.colsum_out || a.colsum_part)) return nullptr;
    float* r = a.colsum_part ? a.colsum_part
                             : (float*)workspace((size_t)gemm_colsum_rows(a, a.a_scale != nullptr) * a.N * sizeof(float));
    return r;
}
void colsum_rows_end(const GemmArgs& a, float* rows, hipStream_t s) {
    if (!rows || !a.colsum_out) return;
    RowsJob j{a.colsum_out, rows, gemm_colsum_rows(a, a.a_scale != nullptr), a.N, a.N};
    rows_reduce_add(&j, 1, s);
}

// C[m][n] += sum_z slab[z][m][n], any N (the fp32 engine's split-K)
__global__ __launch_bounds__(256) void slab_reduce1_k(float* __restrict__ C, long long ldc,
                                                      const float* __restrict__ slab, int M, int N,
                                                      int splits) {
    const long long n1 = (long long)M * N;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n1; e += (long long)gridDim.x * 256) {
        const int m = (int)(e / N), n = (int)(e - (long long)m * N);
        float acc = slab[e];
        for (int z = 1; z < splits; z++) acc += slab[z * n1 + e];
        C[(long long)m * ldc + n] += acc;
    }
}
// C[m][n] += sum_z slab[z][m][n]   (M x N fp32, ldc == N for the slabs)
__global__ __launch_bounds__(256) void slab_reduce_k(float* __restrict__ C, long long ldc,
                                                     const float* __restrict__ slab, int M, int N,
                                                     int splits) {
    const long long n4 = (long long)M * N / 4;
    const long long plane = (long long)M * N;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const long long e = i * 4;
        const int m = (int)(e / N), n = (int)(e - (long long)m * N);
        float4 acc = reinterpret_cast<const float4*>(slab)[i];
        for (int z = 1; z < splits; z++) {
            const float4 t = *reinterpret_cast<const float4*>(slab + z * plane + e);
            acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
        }
        float4* c = reinterpret_cast<float4*>(C + (long long)m * ldc + n);
        float4 o = *c;
        o.x += acc.x; o.y += acc.y; o.z += acc.z; o.w += acc.w;
        *c = o;
    }
}

// engine selection (gemm_bf16_set_variant; default from VIT_GEMM, else 7):
//   1 = 128x128 register-staged everywhere, 2 = 256x256 one workgroup per CU (one tile per
//   workgroup; split-K weight gradients on 256x128), 4 = 256x128 two per CU everywhere, 5 = as 4
//   with the software-pipelined main loop (g4::gemm_kernel_pipe) for K-contiguous operands,
//   7 = production: as 2 with the persistent streaming 256x256 engine (g2::gemm_kernel_s) for the
//   K-contiguous GEMMs without split-K, 11 = as 7 with the two-group ping-pong
//   192x256 engine (gemm_pp.hip) for the shapes it takes.  Debug flag 2 skips the
//   epilogues (main-loop-only timing; results are garbage).
static int g_variant = -1;
static int g_debug_flags = 0;
// variants 5 (software-pipelined 256x128), 9 (one wave per SIMD, gemm_w4.hip) and 10 (split tail) measured
// slower than 7 and are built only with `make EXPERIMENTAL=1`
#if VIT_GEMM_EXPERIMENTAL
static bool known_variant(int v) { return v == 1 || v == 2 || v == 4 || v == 5 || v == 7 || v == 9 || v == 10 || v == 11; }
#else
static bool known_variant(int v) { return v == 1 || v == 2 || v == 4 || v == 7 || v == 11; }
#endif
static constexpr int kDefaultVariant = 7;
static int gemm_variant() {
    if (g_variant < 0) {
        const char* e = getenv("VIT_GEMM");
        g_variant = e ? atoi(e) : kDefaultVariant;
        if (!known_variant(g_variant)) g_variant = kDefaultVariant;
    }
    return g_variant;
}
// 0 (or any unknown value) clears the selection, so the next call re-reads VIT_GEMM (an A/B run
// under VIT_GEMM=2 stays on variant 2 after a test fixture's reset)
void gemm_set_variant(int v) { g_variant = known_variant(v) ? v : -1; }
int gemm_cu_count() {
    static int n = [] {
        int dev = 0, cu = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
        return cu > 0 ? cu : 256;
    }();
    return n;
}
// workgroups of the persistent GEMM engines (VIT_PERSIST_CUS, A/B): default one per CU
int gemm_persist_grid() {
    static const int n = [] {
        const char* e = getenv("VIT_PERSIST_CUS");
        const int v = e ? atoi(e) : 0;
        return v >= 64 && v <= gemm_cu_count() ? v : gemm_cu_count();
    }();
    return n;
}
int gemm_variant_selected() { return gemm_variant(); }
bool gemm_streaming() { return gemm_variant() == 7 || gemm_variant() == 9 || gemm_variant() == 10 || gemm_variant() == 11; }
void gemm_set_debug(int flags) { g_debug_flags = flags; }
static int g_debug_flags_fwd() { return g_debug_flags; }
static unsigned long long* g_trace = nullptr;
void gemm_set_trace(unsigned long long* trace) { g_trace = trace; }

GemmParams make_gemm_params(const GemmArgs& a, int kchunk) {
    GemmParams p;
    p.A = a.A; p.B = a.B; p.C = a.C; p.C2 = a.C2; p.aux = a.aux; p.bias = a.bias; p.dbias = a.dbias; p.colsum_out = nullptr;
    p.lda = a.lda; p.ldb = a.ldb; p.ldc = a.ldc; p.ldaux = a.ldaux;
    if (g_debug_flags & 32) p.ldc = 0;  // diagnostic (timing only, wrong outputs): every row stores onto row 0
    p.M = a.M; p.N = a.N; p.K = a.K; p.kchunk = kchunk;
    p.no_epi = (g_debug_flags & 2) ? 1 : 0;
    p.dbg = g_debug_flags & 0xF0;
    // persistent-engine tile order (bench_gemm, ViT-B/16 shapes, GM 0 / 4 / 8 / 16): groups of 8 row
    // panels help where the A panels are small (K <= 768: qkv fwd 188 -> 179 us, proj fwd 137 -> 133)
    // and hurt where they are large (K = 3072: fcproj fwd 289 -> 302, fc dgrad 235 -> 247: each A panel
    // is then re-read once per column group); VIT_GEMM_GM overrides
    static const int gm_env = [] {
        const char* e = getenv("VIT_GEMM_GM");
        return e && *e ? atoi(e) : -1;
    }();
    const int gm_dbg = (g_debug_flags >> 16) & 0xF;  // diagnostic: (gm + 1) << 16 forces gm (tests)
    p.gm = gm_dbg ? gm_dbg - 1 : gm_env >= 0 ? gm_env : (a.K <= 768 ? 8 : 0);
    p.stagger = ((g_debug_flags >> 8) & 0xFF) * 50;  // debug: 0.5 us units
    p.trace = g_trace;
    p.mx_q = a.mx_q;
    p.mx_s = a.mx_s;
    p.mx_rg = (int)(mx_rows_padded(a.M) / 32);
    p.mxc_q = a.mxc_q;
    p.mxc_s = a.mxc_s;
    p.mxc_ld = a.mxc_ld;
    p.mxc_off = (int)a.mxc_off;
    p.mxc_rg = (int)(mx_rows_padded(a.N) / 32);
    p.tiles = 1;
    p.tsplit = 0;
    p.tfull = 0;
    p.tpart = nullptr;
    return p;
}

// split-K for one-block-per-CU kernels: the smallest split whose last wave of blocks fills
// >= 90% of the 256 CUs (or the best fill up to 32), keeping >= 16 K-tiles per split
int choose_split_waves(int tiles, int nk) {
    const int slots = 256;
    int best = 1;
    double best_eff = 0.0;
    for (int s = 1; s <= 32 && nk / s >= 16; s++) {
        const int blocks = tiles * s;
        const int waves = (blocks + slots - 1) / slots;
        const double eff = (double)blocks / (waves * (double)slots) * (blocks >= slots / 2 ? 1.0 : blocks / (slots / 2.0));
        if (eff > best_eff + 1e-9) { best_eff = eff; best = s; }
        if (eff >= 0.9) break;
    }
    return best;
}

static int choose_split(int tiles, int K, int ktile, int want_blocks) {
    int nk = cdiv(K, ktile);
    int s = 1;
    while (tiles * s < want_blocks && nk / (s * 2) >= 8) s *= 2;
    return s;
}

static int grid_blocks(long long n) {
    long long b = (n + 255) / 256;
    return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}
// split-K slabs: the caller's buffer (a.ws) or the thread workspace; error when neither fits
float* slab_buffer(const GemmArgs& a, int split) {
    const size_t need = (size_t)split * a.M * a.N * sizeof(float);
    float* slab = a.ws ? (a.ws_bytes >= need ? a.ws : nullptr) : (float*)workspace(need);
    if (!slab) set_error("gemm: split-K workspace of %zu bytes unavailable", need);
    return slab;
}
void slab_reduce(const GemmArgs& a, float* slab, int split, hipStream_t s) {
    if (a.N % 4 == 0)
        slab_reduce_k<<<grid_blocks((long long)a.M * a.N / 4), 256, 0, s>>>((float*)a.C, a.ldc, slab, a.M, a.N, split);
    else
        slab_reduce1_k<<<grid_blocks((long long)a.M * a.N), 256, 0, s>>>((float*)a.C, a.ldc, slab, a.M, a.N, split);
    after_launch("gemm_slab_reduce");
    count_hit(VIT_HIT_SPLITK_REDUCE);
}

void gemm_f32(const GemmArgs& a, hipStream_t s) {
    if (a.M <= 0 || a.N <= 0) return;
    if (a.mx_q || a.mxc_q) {
        set_error("gemm_f32: the fused MX output is an fp8-engine feature");
        return;
    }
    const int tiles = cdiv(a.M, f32::BM) * cdiv(a.N, f32::BN);
    int split = 1;
    if (a.epi == EPI_F32_ATOMIC) split = a.splitk > 0 ? a.splitk : choose_split(tiles, a.K, f32::BK, 512);
    int kchunk = cdiv(cdiv(a.K, split), f32::BK) * f32::BK;
    if (kchunk <= 0) kchunk = f32::BK;
    split = cdiv(a.K > 0 ? a.K : 1, kchunk);
    GemmArgs b = a;
    float* slab = nullptr;
    if (a.epi == EPI_F32_ATOMIC) {  // one split accumulates in place; more go through slabs
        if (split > 1) {
            if (!(slab = slab_buffer(a, split))) return;
            b.epi = EPI_F32_SLAB; b.C = slab; b.ldc = a.N;
        } else {
            b.epi = EPI_F32_ACC;
        }
    }
    GemmParams p = make_gemm_params(b, kchunk);
    dim3 grid(tiles, split);
    int akc = a.a_kcontig, bkc = a.b_kcontig;
    switch (b.epi) {
        case EPI_F32_STORE: f32::gemm_f32_kernel<EPI_F32_STORE><<<grid, f32::NT, 0, s>>>(p, akc, bkc); break;
        case EPI_F32_ACC: f32::gemm_f32_kernel<EPI_F32_ACC><<<grid, f32::NT, 0, s>>>(p, akc, bkc); break;
        case EPI_F32_SLAB: f32::gemm_f32_kernel<EPI_F32_SLAB><<<grid, f32::NT, 0, s>>>(p, akc, bkc); break;
        default: set_error("gemm_f32: unsupported epilogue %d", a.epi); return;
    }
    after_launch("gemm_f32");
    count_hit(VIT_HIT_GEMM_F32 + b.epi);
    if (slab) slab_reduce(a, slab, split, s);
}

bool gemm_bf16_supported(const GemmArgs& a) {
    auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    if ((a.a_kcontig || a.b_kcontig) && a.K % 8) return false;  // 16-B chunks along K
    if (a.lda % 8 || a.ldb % 8 || a.N % 4 || a.ldc % 4) return false;
    if (!al16(a.A) || !al16(a.B)) return false;
    if (!a.a_kcontig && a.M % 8) return false;
    if (!a.b_kcontig && a.N % 8) return false;
    return true;
}

template <bool AK, bool BKC>
static void launch_bf16(const GemmArgs& a, const GemmParams& p, dim3 grid, hipStream_t s) {
    switch (a.epi) {
#define VIT_CASE(E) \
    case E: bf::gemm_bf16_kernel<AK, BKC, E><<<grid, bf::NT, 0, s>>>(p); break;
        VIT_CASE(EPI_F32_STORE)
        VIT_CASE(EPI_F32_ACC)
        VIT_CASE(EPI_F32_SLAB)
        VIT_CASE(EPI_BF16_STORE)
        VIT_CASE(EPI_BF16_GELU)
        VIT_CASE(EPI_F32_RESID)
        VIT_CASE(EPI_BF16_DGELU)
        VIT_CASE(EPI_BF16_GELU_D)
        VIT_CASE(EPI_BF16_MUL)
#undef VIT_CASE
        default: set_error("gemm_bf16: unsupported epilogue %d", a.epi); return;
    }
}

template <bool AK, bool BKC>
static void launch_g2(const GemmArgs& a, const GemmParams& p, dim3 grid, hipStream_t s) {
    if constexpr (AK && BKC) {
#if VIT_GEMM_EXPERIMENTAL
        // one-wave-per-SIMD persistent engine (gemm_w4.hip)
        if (gemm_variant() == 9 && grid.y == 1 && gemm_bf16_w4(a, p, (int)grid.x, s)) return;
        // persistent streaming engine with a split tail (variant 10): when the last round fills at
        // most half the CUs, its tiles run as K-ranges on all of them (bias / residual / bf16 store
        // epilogues; fp32 partial tiles in a.tail_ws or the thread workspace + gemm_tail_fix_k)
        if (gemm_variant() == 10 && a.tail_ws && grid.y == 1 && p.K >= 2 * g2::BK && p.kchunk == p.K &&
            (a.epi == EPI_F32_STORE || a.epi == EPI_BF16_STORE || a.epi == EPI_F32_RESID) &&
            (long long)p.M * p.lda * 2 < (1LL << 31) && (long long)p.N * p.ldb * 2 < (1LL << 31)) {
            const int cus = gemm_cu_count(), tiles = (int)grid.x;
            const int nblk = tiles < cus ? tiles : cus, full = tiles / nblk * nblk, tail = tiles - full;
            const int nk = p.K / g2::BK;
            int split = tail > 0 && full > 0 ? std::min(nblk / tail, nk / 2) : 1;
            if (split >= 2) {
                const int kchunk = cdiv(cdiv(p.K, split), 2 * g2::BK) * (2 * g2::BK);  // even step count
                split = cdiv(p.K, kchunk);
                const size_t need = (size_t)tail * split * g2::BM * g2::BN * sizeof(float);
                // the caller's per-stream buffer only: the thread workspace is shared by concurrent streams
                float* part = a.tail_ws_bytes >= need ? a.tail_ws : nullptr;
                if (split >= 2 && part) {
                    GemmParams q = p;
                    q.tsplit = split;
                    q.tfull = full;
                    q.kchunk = kchunk;
                    q.tpart = part;
                    switch (a.epi) {
#define VIT_CASE(E)                                                                   \
    case E:                                                                           \
        g2::gemm_kernel_s<E, true><<<nblk, g2::NT, 0, s>>>(q);                         \
        g2::gemm_tail_fix_k<E><<<dim3(tail, g2::BM / 32), 256, 0, s>>>(q);            \
        return;
                        VIT_CASE(EPI_F32_STORE)
                        VIT_CASE(EPI_BF16_STORE)
                        VIT_CASE(EPI_F32_RESID)
#undef VIT_CASE
                        default: break;
                    }
                }
            }
        }
#endif
        // persistent streaming engine: one workgroup per CU (at most one per tile), no split-K;
        // its DMA ring runs two K-steps ahead across one tile boundary, so K >= 2 steps
        if ((gemm_variant() == 7 || gemm_variant() == 10 || gemm_variant() == 11) && grid.y == 1 && p.K >= 2 * g2::BK &&
            (long long)p.M * p.lda * 2 < (1LL << 31) &&
            (long long)p.N * p.ldb * 2 < (1LL << 31)) {
            const int cus = gemm_persist_grid();
            const dim3 pg((int)grid.x < cus ? grid.x : cus);
            switch (a.epi) {
#define VIT_CASE(E) \
    case E: g2::gemm_kernel_s<E><<<pg, g2::NT, 0, s>>>(p); return;
                VIT_CASE(EPI_F32_STORE)
                VIT_CASE(EPI_F32_ACC)
                VIT_CASE(EPI_BF16_STORE)
                VIT_CASE(EPI_BF16_GELU)
                VIT_CASE(EPI_F32_RESID)
                VIT_CASE(EPI_BF16_DGELU)
                VIT_CASE(EPI_BF16_GELU_D)
                VIT_CASE(EPI_BF16_MUL)
#undef VIT_CASE
                default: break;
            }
        }
    }
    switch (a.epi) {
#define VIT_CASE(E) \
    case E: g2::gemm_kernel<AK, BKC, E, 2><<<grid, g2::NT, 0, s>>>(p); break;
        VIT_CASE(EPI_F32_STORE)
        VIT_CASE(EPI_F32_ACC)
        VIT_CASE(EPI_BF16_STORE)
        VIT_CASE(EPI_BF16_GELU)
        VIT_CASE(EPI_F32_RESID)
        VIT_CASE(EPI_BF16_DGELU)
        VIT_CASE(EPI_F32_SLAB)
        VIT_CASE(EPI_BF16_GELU_D)
        VIT_CASE(EPI_BF16_MUL)
#undef VIT_CASE
        default: set_error("gemm_bf16: unsupported epilogue %d", a.epi); return;
    }
}


template <bool AK, bool BKC>
static void launch_g4(const GemmArgs& a, const GemmParams& p, dim3 grid, hipStream_t s) {
    if constexpr (AK && BKC) {
        // software-pipelined main loop: an even step count per split and 32-bit DMA offsets
        const bool fits = p.kchunk % 64 == 0 && p.K % 64 == 0 && (long long)p.M * p.lda * 2 < (1LL << 32) &&
                          (long long)p.N * p.ldb * 2 < (1LL << 32);
#if VIT_GEMM_EXPERIMENTAL
        if (gemm_variant() == 5 && fits) {
            switch (a.epi) {
#define VIT_CASE(E) \
    case E: g4::gemm_kernel_pipe<E><<<grid, g4::NT, 0, s>>>(p); return;
                VIT_CASE(EPI_F32_STORE)
                VIT_CASE(EPI_F32_ACC)
                VIT_CASE(EPI_BF16_STORE)
                VIT_CASE(EPI_BF16_GELU)
                VIT_CASE(EPI_F32_RESID)
                VIT_CASE(EPI_BF16_DGELU)
                VIT_CASE(EPI_F32_SLAB)
                VIT_CASE(EPI_BF16_GELU_D)
                VIT_CASE(EPI_BF16_MUL)
#undef VIT_CASE
                default: break;
            }
        }
#else
        (void)fits;
#endif
    }
    switch (a.epi) {
#define VIT_CASE(E) \
    case E: g4::gemm_kernel<AK, BKC, E><<<grid, g4::NT, 0, s>>>(p); break;
        VIT_CASE(EPI_F32_STORE)
        VIT_CASE(EPI_F32_ACC)
        VIT_CASE(EPI_BF16_STORE)
        VIT_CASE(EPI_BF16_GELU)
        VIT_CASE(EPI_F32_RESID)
        VIT_CASE(EPI_BF16_DGELU)
        VIT_CASE(EPI_F32_SLAB)
        VIT_CASE(EPI_BF16_GELU_D)
        VIT_CASE(EPI_BF16_MUL)
#undef VIT_CASE
        default: set_error("gemm_bf16: unsupported epilogue %d", a.epi); return;
    }
}

// split-K for two-workgroups-per-CU kernels, keeping >= 32 K-steps per split: the one-round rule
// below (fill_pct > 0: the caller's fill target, else VIT_G4_FILL), falling back to the best fill
// over any number of rounds of the 512 workgroup slots
static int choose_split_g4(int tiles, int nk, int fill_pct = 0) {
    // slots the split-K work items are sized for (VIT_G4_SLOTS, A/B): 512 = both workgroups of every CU
    static const int slots = [] {
        const char* e = getenv("VIT_G4_SLOTS");
        const int v = e ? atoi(e) : 512;
        return v >= 64 && v <= 2048 ? v : 512;
    }();
    // r06 rule: the smallest split whose work items fill >= `fill` of the slots in ONE round.  The weight
    // gradients run on their own stream beside the micro-batch streams, so a partly idle round costs
    // less than the slab bytes (and the fixed-order reduce) of more splits: ViT-B/16 splits 9/26/7/7 ->
    // 8/23/6/6 (qkv/proj/fc/fcproj), ViT-H/14 qkv 10 -> 3 (profiles/r06_g4_slots.txt).  VIT_G4_RULE=0:
    // the round-5 rule below alone (best fill, multi-round allowed, first >= 90 %)
    static const bool one_round = [] {
        const char* e = getenv("VIT_G4_RULE");
        return !(e && e[0] == '0');
    }();
    // fill target 45 % (VIT_G4_FILL), as the fp8 engine's: 80 -> 45 % ViT-B/16 +0.2 / +0.4 %, ViT-H/14 bf16
    // +2.2 %, ViT-L/16 -0.6 % (interleaved bench rounds, profiles/r06_g4_slots.txt)
    static const double fill = [] {
        const char* e = getenv("VIT_G4_FILL");
        const int v = e ? atoi(e) : 45;
        return (v >= 20 && v <= 100 ? v : 45) / 100.0;
    }();
    if (one_round) {
        const double f = fill_pct > 0 ? fill_pct / 100.0 : fill;
        const int s1 = (int)((f * slots + tiles - 1) / tiles);
        if (s1 >= 1 && (long long)tiles * s1 <= slots && nk / s1 >= 32) return s1;
    }
    int best = 1;
    double best_eff = 0.0;
    for (int s = 1; s <= 64 && nk / s >= 32; s++) {
        const int blocks = tiles * s;
        const int rounds = (blocks + slots - 1) / slots;
        const double eff = (double)blocks / (rounds * (double)slots) * (blocks >= slots / 2 ? 1.0 : blocks / (slots / 2.0));
        if (eff > best_eff + 1e-9) { best_eff = eff; best = s; }
        if (eff >= 0.9) break;
    }
    return best;
}

static void gemm_bf16_g4(const GemmArgs& a, hipStream_t s) {
    const int tiles = cdiv(a.M, g4::BM) * cdiv(a.N, g4::BN);
    int split = 1;
    if (a.epi == EPI_F32_ATOMIC) split = a.splitk > 0 ? a.splitk : choose_split_g4(tiles, a.K / g4::KTILE, a.fill_pct);
    int kchunk = cdiv(cdiv(a.K, split), g4::KTILE) * g4::KTILE;
    split = cdiv(a.K, kchunk);
    GemmArgs b = a;
    float* slab = nullptr;
    if (a.epi == EPI_F32_ATOMIC) {
        // split-K partials go to fp32 slabs + one reduce (no float atomics in the GEMM); a single
        // split accumulates in place
        if (split > 1) {
            if (!(slab = slab_buffer(a, split))) return;
            b.epi = EPI_F32_SLAB;
            b.C = slab;
            b.ldc = a.N;
        } else {
            b.epi = EPI_F32_ACC;
        }
    }
    GemmParams p = make_gemm_params(b, kchunk);
    p.tiles = tiles;
    float* cs_rows = colsum_rows_begin(a);
    if ((a.colsum_out || a.colsum_part) && epi_aux16(a.epi) && !cs_rows) return;
    p.colsum_out = cs_rows;
    dim3 grid(tiles, split);
    if (a.a_kcontig && a.b_kcontig) launch_g4<true, true>(b, p, grid, s);
    else if (a.a_kcontig && !a.b_kcontig) launch_g4<true, false>(b, p, grid, s);
    else if (!a.a_kcontig && !a.b_kcontig) launch_g4<false, false>(b, p, grid, s);
    else launch_g4<false, true>(b, p, grid, s);
    after_launch("gemm_bf16_256x128");
    count_hit(VIT_HIT_GEMM_256x128 + b.epi);
    if (slab) slab_reduce(a, slab, split, s);
    colsum_rows_end(a, cs_rows, s);
    // bias gradient of a wgrad (M-contig A = dout^T): column sums of dout over the K rows (the
    // thread workspace may be the slab just reduced: stream-ordered after the reduce)
    if (a.dbias && !a.a_kcontig) colsum_bf16(a.dbias, (const bf16_t*)a.A, a.K, a.M, a.lda, s);
}

void gemm_bf16(const GemmArgs& a, hipStream_t s) {
    if (a.M <= 0 || a.N <= 0) return;
    if (a.mx_q || a.mxc_q) {
        set_error("gemm_bf16: the fused MX output is an fp8-engine feature");
        return;
    }
    if (!gemm_bf16_supported(a)) {
        set_error("gemm_bf16: unsupported shape/alignment M=%d N=%d K=%d lda=%lld ldb=%lld",
                  a.M, a.N, a.K, a.lda, a.ldb);
        return;
    }
    if ((gemm_variant() == 4 || gemm_variant() == 5) && a.K % g4::KTILE == 0 && a.M >= 256 && a.N >= 128 &&
        (a.epi != EPI_F32_ATOMIC || a.N % 4 == 0)) {
        gemm_bf16_g4(a, s);
        return;
    }
    // split-K weight gradients (M/N-contiguous operands, K = the token count) run on the 256x128
    // two-per-CU engine: 3-9 % faster than 256x256 on every ViT-B/16 wgrad shape (r02,
    // tools/bench_gemm.py), the other GEMMs are faster on 256x256
    if ((gemm_variant() == 2 || gemm_variant() == 7 || gemm_variant() == 9 || gemm_variant() == 10 || gemm_variant() == 11) &&
        a.epi == EPI_F32_ATOMIC && !a.a_kcontig && !a.b_kcontig &&
        a.K % g4::KTILE == 0 && a.M >= 256 && a.N >= 128 && a.N % 4 == 0 &&
        (a.splitk > 0 || !a.ws ||
         (size_t)choose_split_g4(cdiv(a.M, g4::BM) * cdiv(a.N, g4::BN), a.K / g4::KTILE) * a.M * a.N * sizeof(float) <=
             a.ws_bytes)) {
        gemm_bf16_g4(a, s);
        return;
    }
    const bool big = a.K % g2::KTILE == 0 && a.M >= 256 && a.N >= 256 && gemm_variant() != 1;
    if (big) {
        const int tiles = cdiv(a.M, g2::BM) * cdiv(a.N, g2::BN);
        int split = 1;
        if (a.epi == EPI_F32_ATOMIC) split = a.splitk > 0 ? a.splitk : choose_split_waves(tiles, a.K / g2::KTILE);
        int kchunk = cdiv(cdiv(a.K, split), g2::KTILE) * g2::KTILE;
        split = cdiv(a.K, kchunk);
        GemmArgs b = a;
        float* slab = nullptr;
        if (a.epi == EPI_F32_ATOMIC) {  // split-K partials to fp32 slabs + one reduce (no atomics)
            if (split > 1) {
                if (!(slab = slab_buffer(a, split))) return;
                b.epi = EPI_F32_SLAB;
                b.C = slab;
                b.ldc = a.N;
            } else {
                b.epi = EPI_F32_ACC;
            }
        }
        GemmParams p = make_gemm_params(b, kchunk);
        p.tiles = tiles;
        float* cs_rows = colsum_rows_begin(a);
        if ((a.colsum_out || a.colsum_part) && epi_aux16(a.epi) && !cs_rows) return;
        p.colsum_out = cs_rows;
        // fused bias gradient: one add per (column block, K-split), deterministic with one split
        const bool late_db = a.dbias && !a.a_kcontig && split > 1;
        if (late_db) p.dbias = nullptr;
        if (split == 1 && pp_taken(b)) {  // variant 11: the ping-pong engine (gemm_pp.hip)
            gemm_bf16_pp(b, p, s);
            after_launch("gemm_bf16_pp");
            count_hit(VIT_HIT_GEMM_256x256 + b.epi);
            count_hit(VIT_HIT_GEMM_PP);
            colsum_rows_end(a, cs_rows, s);
            return;
        }
        dim3 grid(tiles, split);
        if (a.a_kcontig && a.b_kcontig) launch_g2<true, true>(b, p, grid, s);
        else if (a.a_kcontig && !a.b_kcontig) launch_g2<true, false>(b, p, grid, s);
        else if (!a.a_kcontig && !a.b_kcontig) launch_g2<false, false>(b, p, grid, s);
        else launch_g2<false, true>(b, p, grid, s);
        after_launch("gemm_bf16_256");
        count_hit(VIT_HIT_GEMM_256x256 + b.epi);
        if (slab) slab_reduce(a, slab, split, s);
        colsum_rows_end(a, cs_rows, s);
        if (late_db) colsum_bf16(a.dbias, (const bf16_t*)a.A, a.K, a.M, a.lda, s);
        return;
    }
    const int tiles = cdiv(a.M, bf::BM) * cdiv(a.N, bf::BN);
    int split = 1;
    if (a.epi == EPI_F32_ATOMIC) split = a.splitk > 0 ? a.splitk : choose_split(tiles, a.K, bf::BK, 512);
    int kchunk = cdiv(cdiv(a.K, split), bf::BK) * bf::BK;
    if (kchunk <= 0) kchunk = bf::BK;
    split = cdiv(a.K > 0 ? a.K : 1, kchunk);
    GemmArgs b = a;
    float* slab = nullptr;
    if (a.epi == EPI_F32_ATOMIC) {  // split-K partials to fp32 slabs + one reduce (no atomics)
        if (split > 1) {
            if (!(slab = slab_buffer(a, split))) return;
            b.epi = EPI_F32_SLAB; b.C = slab; b.ldc = a.N;
        } else {
            b.epi = EPI_F32_ACC;
        }
    }
    GemmParams p = make_gemm_params(b, kchunk);
    // the kernel's fused bias gradient adds once per (column block, K-split): deterministic with
    // one split only; otherwise the column sums run after the GEMM
    const bool late_db = a.dbias && !a.a_kcontig && split > 1;
    if (late_db) p.dbias = nullptr;
    dim3 grid(tiles, split);
    if (a.a_kcontig && a.b_kcontig) launch_bf16<true, true>(b, p, grid, s);
    else if (a.a_kcontig && !a.b_kcontig) launch_bf16<true, false>(b, p, grid, s);
    else if (!a.a_kcontig && !a.b_kcontig) launch_bf16<false, false>(b, p, grid, s);
    else launch_bf16<false, true>(b, p, grid, s);
    after_launch("gemm_bf16");
    count_hit(VIT_HIT_GEMM_128 + b.epi);
    if (slab) slab_reduce(a, slab, split, s);
    if (late_db) colsum_bf16(a.dbias, (const bf16_t*)a.A, a.K, a.M, a.lda, s);
    // the 128x128 kernel has no fused column sums: partial rows of its output, then the same
    // fixed-order reduce as the fused epilogues
    if ((a.colsum_out || a.colsum_part) && epi_aux16(a.epi)) {
        float* rows = colsum_rows_begin(a);
        if (!rows) return;
        colsum_part_k<bf16_t><<<dim3(cdiv(a.N, 256), cdiv(a.M, 128)), 256, 0, s>>>(
            rows, (const bf16_t*)a.C, a.M, a.N, a.ldc, 128, 0);
        after_launch("colsum_rows");
        colsum_rows_end(a, rows, s);
    }
}

void colsum_f32(float* dbias, const float* X, int M, int N, long long ld, hipStream_t s, float* ws) {
    colsum_any(dbias, X, M, N, ld, s, ws);
}
void colsum_bf16(float* dbias, const bf16_t* X, int M, int N, long long ld, hipStream_t s, float* ws) {
    colsum_any(dbias, X, M, N, ld, s, ws);
}

}  // namespace vit
