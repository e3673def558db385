// gemm_fp8.hip — MXFP8 GEMM for the fp8 mode of matmul_forward / matmul_backward's input gradient
// (train_vit.rs:384-398, 530-541) and the MX block quantizer that feeds it.
//
// Operands are OCP fp8 e4m3 with one E8M0 scale per 32 consecutive k-elements of a row (the OCP
// MX block scaling), multiplied on v_mfma_scale_f32_32x32x64_f8f6f4 (twice the bf16 MFMA rate,
// fp32 accumulate, the block scales applied in hardware).  Both operands are K-contiguous byte
// rows: A [M][K] (activations or output gradients) and B [N][K] (W[n][k] for the forward; the
// transposed weight copy WT[n][k] for the input gradient).
//
// Engine: the bf16 256x256 pipeline of gemm.hip (g2) with bytes in place of bf16.  One LDS slot
// holds a 64-deep k-step of both 256-row operands (16 KiB each, 64-B rows) = exactly one
// 32x32x64 MFMA k-step, so the slot cadence, the ring of 4 slots (LDS-DMA 2 steps ahead), the
// counted vmcnt waits and the staggered wave halves carry over unchanged: per slot and wave,
// 2 phases x 4 MFMAs of 64 cycles (= g2's 2 x 16 x 16).  8 waves (2 M x 4 N), 128 x 64 per wave =
// 4 x 2 tiles of 32x32.  MFMA lane layout (tools/probe_mx.hip, measured): lane (r = l&31,
// h = l>>5) carries k [16h, 16h+16) in bytes 0..15 and k [32+16h, 48+16h) in bytes 16..31 of the
// step, i.e. 16-B chunks h and 2+h of the 64-B row; its scale byte scales row r, k-block h.
// LDS images are lane-linear (LDS-DMA); chunk' = chunk ^ ((row >> 2) & 3) on the global source
// address makes the 32-row fragment reads conflict free.
//
// Scales, "lane-native" layout: S[K/64][Rpad/32][64] bytes, Rpad = rows rounded up to 256; byte
// h*32 + r of row group g at step s is the scale of row 32g + r, k-block 2s + h.  Per slot the
// tile's scales are 512 contiguous bytes per operand, staged by one 4-byte LDS-DMA per wave;
// each MFMA reads its lane's byte with one ds_read_u8.  Padding rows carry scale 0 (2^-127).
#include <algorithm>
#include <cstdlib>

#include "gemm_common.h"
#include "ln_common.h"
#include "ops_internal.h"

#ifndef VIT_F8_TRACE
#define VIT_F8_TRACE 0
#endif
// one phase per K-step in the streaming engine (two barriers per step instead of four): faster alone
// (ViT-H/14 micro-batch GEMMs, tools/f8_trace.py: qkv fwd 146 -> 128 us, fc dgrad 187 -> 170, qkv dgrad
// 152 -> 137) but slower in the sustained train step (117.0 vs 115.7 ms/step, two interleaved rounds;
// profiles/r06_onephase.txt), so off
#ifndef VIT_F8_ONEPHASE
#define VIT_F8_ONEPHASE 0
#endif

namespace vit {
namespace f8 {
constexpr int BM = 256, BN = 256, NT = 512;
constexpr int KB = 64;                           // k bytes (= fp8 elements) per slot
constexpr int IMG_BYTES = 256 * KB;              // 16 KiB per operand image
constexpr int SC_BYTES = 1024;                   // scales of one slot: A 512 B | B 512 B
constexpr int SLOT_BYTES = 2 * IMG_BYTES + SC_BYTES;
constexpr int DEPTH = 2, NS = DEPTH + 2;
constexpr int SMEM = NS * SLOT_BYTES > 8 * STG_WAVE_BYTES ? NS * SLOT_BYTES : 8 * STG_WAVE_BYTES;
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int swz(int row) { return (row >> 2) & 3; }

// this wave's 2 data pieces of one operand image (piece blk = 8j + wave: rows 16blk .. 16blk+15)
__device__ __forceinline__ void stage(const uint8_t* __restrict__ base, long long ld, int row0,
                                      int rows_lim, int k0, char* img, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int blk = j * 8 + wave;
        const int row = blk * 16 + (lane >> 2);
        const int c = (lane & 3) ^ swz(row);
        const int gr = min(row0 + row, rows_lim - 1);
        const uint8_t* src = base + (long long)gr * ld + k0 + c * 16;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(img + blk * 1024),
                                         16, 0, 0);
    }
}
// this wave's 128 B of the slot's scales: waves 0-3 the A tile's 8 row groups, 4-7 the B tile's;
// 4-byte LDS-DMA on lanes 0-31 (every wave issues the same one instruction, so the counted vmcnt
// waits stay uniform; sub-dword LDS-DMA does not pack lanes at their byte size)
__device__ __forceinline__ void stage_scales(const uint8_t* __restrict__ sa, const uint8_t* __restrict__ sb,
                                             int rga, int rgb, int ks, int rga_tot, int rgb_tot,
                                             char* sc, int wave, int lane) {
    const bool isb = wave >= 4;
    const int w4 = wave & 3;
    const uint8_t* src = isb ? sb + ((long long)ks * rgb_tot + rgb + 2 * w4) * 64
                             : sa + ((long long)ks * rga_tot + rga + 2 * w4) * 64;
    if (lane < 32)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 4 * lane),
                                         (__attribute__((address_space(3))) void*)(sc + (isb ? 512 : 0) + w4 * 128),
                                         4, 0, 0);
}
// rows [r0, r0+32) of an image: chunks h and 2+h of the lane's row
__device__ __forceinline__ v8i frag(const char* img, int r0, int lane) {
    const int r = r0 + (lane & 31), h = lane >> 5, sw = swz(r);
    const u32x4 lo = *reinterpret_cast<const u32x4*>(img + r * KB + ((h ^ sw) << 4));
    const u32x4 hi = *reinterpret_cast<const u32x4*>(img + r * KB + (((2 + h) ^ sw) << 4));
    return v8i{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}
__device__ __forceinline__ int scale_of(const char* sc, int grp, int lane) {
    return *reinterpret_cast<const uint8_t*>(sc + grp * 64 + lane);
}
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

struct F8Params {
    GemmParams p;
    const uint8_t* sa;
    const uint8_t* sb;
    int rga_tot, rgb_tot;  // scale row groups (Rpad / 32) of A and B
};

// Pipeline (as g2): every 64-deep k-step is two phases of 4 MFMAs per wave; each phase is
// [LDS fragment reads + LDS-DMA] barrier [MFMAs] barrier; waves 4-7 run one barrier behind.
// Per step and wave 5 DMA instructions: A half (2 data + 1 scale) in phase 0, B half (2) in
// phase 1, for step kt + DEPTH into the slot read at step kt - 2.
template <int EPI>
__global__ __launch_bounds__(NT, 1) void gemm_kernel(F8Params fp) {
    const GemmParams& p = fp.p;
    __shared__ __attribute__((aligned(1024))) char smem[SMEM];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int ntn = cdiv(p.N, BN);
    int wg, split;
    split_remap(p.tiles, wg, split);
    const int tm0 = (wg / ntn) * BM, tn0 = (wg % ntn) * BN;
    // K-split `split` (EPI_F32_SLAB) covers k [kbeg, kend); kchunk % KB == 0
    const int kbeg = split * p.kchunk;
    const int nk = (min(p.K, kbeg + p.kchunk) - kbeg) / KB;
    const int ks0 = kbeg / KB;  // first scale k-step of the split
    const uint8_t* A = (const uint8_t*)p.A + kbeg;
    const uint8_t* B = (const uint8_t*)p.B + kbeg;

    v16f acc[4][2];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = v16f{};

    auto slot_of = [&](int st) { return smem + (st % NS) * SLOT_BYTES; };
    auto issue_a = [&](int st) {  // A image pieces + this wave's scale piece of step st
        if (st < nk) {
            stage(A, p.lda, tm0, p.M, st * KB, slot_of(st), wave, lane);
            stage_scales(fp.sa, fp.sb, tm0 / 32, tn0 / 32, ks0 + st, fp.rga_tot, fp.rgb_tot,
                         slot_of(st) + 2 * IMG_BYTES, wave, lane);
        }
    };
    auto issue_b = [&](int st) {
        if (st < nk) stage(B, p.ldb, tn0, p.N, st * KB, slot_of(st) + IMG_BYTES, wave, lane);
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };
    // instruction A = the B fragment (rows = output columns), instruction B = the A fragment, so a
    // lane's accumulator registers run along output columns of one output row (as g2)
    auto mfma_half = [&](int half, const v8i (&fa)[2], const int (&sa)[2], const v8i (&fb)[2], const int (&sb)[2]) {
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 2; b++)
                acc[half * 2 + a][b] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                    fb[b], fa[a], acc[half * 2 + a][b], 0, 0, 0, sb[b], 0, sa[a]);
    };

    const bool lagging = wave >= 4;
    if (nk > 0) {
#pragma unroll
        for (int st = 0; st < DEPTH; st++) { issue_a(st); issue_b(st); }
        wait_vm(5 * (min(DEPTH, nk) - 1));  // own pieces of step 0
        bar();
        if (lagging) {
            __builtin_amdgcn_s_setprio(1);  // static priority for the younger half
            bar();                          // stagger: one barrier behind waves 0-3
        }
    }
    v8i fb[2], fa0[2], fa1[2];
    int sb_[2], sa0[2], sa1[2];
    for (int kt = 0; kt < nk; kt++) {
        const char* img = slot_of(kt);
        const char* sc = img + 2 * IMG_BYTES;
        // ---- phase 0: B fragments, A tiles 0-1 (rows 0-63 of the wave tile)
#pragma unroll
        for (int b = 0; b < 2; b++) {
            fb[b] = frag(img + IMG_BYTES, wn * 64 + b * 32, lane);
            sb_[b] = scale_of(sc + 512, wn * 2 + b, lane);
        }
#pragma unroll
        for (int a = 0; a < 2; a++) {
            fa0[a] = frag(img, wm * 128 + a * 32, lane);
            sa0[a] = scale_of(sc, wm * 4 + a, lane);
        }
        issue_a(kt + DEPTH);
        bar();
        mfma_half(0, fa0, sa0, fb, sb_);
        bar();
        // ---- phase 1: A tiles 2-3
#pragma unroll
        for (int a = 0; a < 2; a++) {
            fa1[a] = frag(img, wm * 128 + (2 + a) * 32, lane);
            sa1[a] = scale_of(sc, wm * 4 + 2 + a, lane);
        }
        // own pieces of step kt+1 landed: the younger ones are the A half of step kt+DEPTH (3)
        wait_vm(kt + DEPTH < nk ? 3 : 0);
        issue_b(kt + DEPTH);
        bar();
        mfma_half(1, fa1, sa1, fb, sb_);
        bar();
    }
    if (nk > 0 && !lagging) bar();  // balance the stagger barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(0);

    if (p.no_epi & 1) {  // diagnostic: main loop only; keep the accumulators live (in 16-B pieces: a
                     // 64-B "v" asm operand makes hipcc drop the host stubs of the other instances)
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int q = 0; q < 4; q++)
                    asm volatile("" ::"v"(f32x4_t{acc[a][b][4 * q], acc[a][b][4 * q + 1], acc[a][b][4 * q + 2],
                                                   acc[a][b][4 * q + 3]}));
        return;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // 32x32 accumulators -> the row-staged epilogue: lane l of tile (a,b) holds output row
    // 32a + (l&31), columns 32b + 8q + 4(l>>5) + 0..3 in registers 4q..4q+3
    float* st = reinterpret_cast<float*>(smem + wave * STG_WAVE_BYTES);
    const int m0 = tm0 + wm * 128, n0 = tn0 + wn * 64;
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const bool interior = staged_interior<EPI>(p, m0, n0);
    const int r = lane & 31, h = lane >> 5;
#pragma unroll
    for (int pass = 0; pass < 2; pass++) {
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const v16f& v = acc[pass * 2 + a][b];
                    *reinterpret_cast<f32x4_t*>(st + (a * 32 + r) * STG_LD + b * 32 + 8 * q + 4 * h) =
                        f32x4_t{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
                }
        staged_pass<EPI>(p, st, lane, m0, n0, pass, interior, cs);
        if constexpr (epi_mx(EPI)) {
            if (p.mxc_q) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                mx_cols_pass(p, st, lane, m0 + pass * 64, n0);
            }
        }
    }
    staged_colsum<EPI>(p, lane, m0, n0, cs);
}

// Persistent streaming form (as g2::gemm_kernel_s): one workgroup per CU walks its
// tiles with the LDS-DMA ring (data and scale pieces) streaming across tile boundaries, the next
// tile's first two K-steps landing under the epilogue, which stages through the tile's last two
// slots in 32-row passes (8 KiB per wave; the column-wise MX pass quantizes one 32-token block per
// pass).  Same MFMAs in the same order and the same epilogue arithmetic: bit-identical outputs.
template <int EPI>
__global__ __launch_bounds__(NT, 1) void gemm_kernel_s(F8Params fp) {
    const GemmParams& p = fp.p;
    __shared__ __attribute__((aligned(1024))) char smem[NS * SLOT_BYTES];
    static_assert(4 * 8192 <= SLOT_BYTES, "epilogue staging: four waves per slot");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int ntn = cdiv(p.N, BN), tiles = p.tiles;
    const int nblk = gridDim.x;
    const int my_tiles = (tiles - (int)blockIdx.x + nblk - 1) / nblk;
    const int nk = p.K / KB;
    const char* A = (const char*)p.A;
    const char* B = (const char*)p.B;
    const bool isb = wave >= 4;
    const int w4 = wave & 3;
    const char* S = (const char*)(isb ? fp.sb : fp.sa);
    const int rg_tot = isb ? fp.rgb_tot : fp.rga_tot;
    v16f acc[4][2];
    auto zero_acc = [&]() {
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 2; b++) acc[a][b] = v16f{};
    };
    zero_acc();
    if (my_tiles <= 0) return;
    struct TileSrc {
        int tm0, tn0;
        uint32_t a[2], b[2], sc;
    };
    auto tile_src = [&](int j, TileSrc& ts) {
        const int t = xcd_remap(j * nblk + (int)blockIdx.x, tiles);
        if (p.gm > 0) {  // grouped order, as g2::gemm_kernel_s
            const int ntm = cdiv(p.M, BM), per = p.gm * ntn, g = t / per, r = t - g * per,
                      rows = min(p.gm, ntm - g * p.gm);
            ts.tm0 = (g * p.gm + r % rows) * BM;
            ts.tn0 = (r / rows) * BN;
        } else {
            ts.tm0 = (t / ntn) * BM;
            ts.tn0 = (t % ntn) * BN;
        }
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int row = (q * 8 + wave) * 16 + (lane >> 2);
            const int c = (lane & 3) ^ swz(row);
            ts.a[q] = (uint32_t)((long long)min(ts.tm0 + row, p.M - 1) * p.lda + c * 16);
            ts.b[q] = (uint32_t)((long long)min(ts.tn0 + row, p.N - 1) * p.ldb + c * 16);
        }
        ts.sc = (uint32_t)((((isb ? ts.tn0 : ts.tm0) / 32) + 2 * w4) * 64 + 4 * lane);
    };
    TileSrc cur, nxt;
    tile_src(0, cur);
    nxt = cur;
    if (my_tiles > 1) tile_src(1, nxt);
    auto glds16 = [&](const char* src, char* dst) {
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    };
    // A pieces + this wave's scale piece of step kt2 of the current tile (kt2 >= nk: the next one's)
    auto issue_a = [&](int kt2, int sl, bool more) {
        if (kt2 >= nk && !more) return;
        const bool c = kt2 < nk;
        const int k = c ? kt2 : kt2 - nk;
        char* dst = smem + sl * SLOT_BYTES;
#pragma unroll
        for (int q = 0; q < 2; q++) glds16(A + (long long)k * KB + (c ? cur.a[q] : nxt.a[q]), dst + (q * 8 + wave) * 1024);
        if (lane < 32)
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(S + (long long)k * rg_tot * 64 + (c ? cur.sc : nxt.sc)),
                (__attribute__((address_space(3))) void*)(dst + 2 * IMG_BYTES + (isb ? 512 : 0) + w4 * 128), 4, 0, 0);
    };
    auto issue_b = [&](int kt2, int sl, bool more) {
        if (kt2 >= nk && !more) return;
        const bool c = kt2 < nk;
        const int k = c ? kt2 : kt2 - nk;
        char* dst = smem + sl * SLOT_BYTES + IMG_BYTES;
#pragma unroll
        for (int q = 0; q < 2; q++) glds16(B + (long long)k * KB + (c ? cur.b[q] : nxt.b[q]), dst + (q * 8 + wave) * 1024);
    };
#if VIT_F8_TRACE
    // diagnostic build (tools/f8_trace.py): lane 0 of every wave of workgroups 0..7 sums the shader
    // cycles (s_memtime, sampled at issue) spent waiting for LDS reads before each barrier, in the
    // barrier, in the counted vmcnt waits of the main loop, in main loops and in epilogues
    unsigned long long tr_lgk = 0, tr_bar = 0, tr_vm = 0, tr_main = 0, tr_epi = 0, tr_t = 0;
    const unsigned long long tr_mt0 = __builtin_amdgcn_s_memtime(), tr_rt0 = __builtin_amdgcn_s_memrealtime();
#define F8T(x) x
#else
#define F8T(x)
#endif
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        F8T(const unsigned long long t0 = __builtin_amdgcn_s_memtime();)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        F8T(const unsigned long long t1 = __builtin_amdgcn_s_memtime();)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        F8T(const unsigned long long t2 = __builtin_amdgcn_s_memtime(); tr_lgk += t1 - t0; tr_bar += t2 - t1;)
        __builtin_amdgcn_sched_barrier(0);
    };
    auto wait_vm_t = [&](int n) {
        F8T(const unsigned long long t0 = __builtin_amdgcn_s_memtime();)
        wait_vm(n);
        F8T(tr_vm += __builtin_amdgcn_s_memtime() - t0;)
    };
    auto mfma_half = [&](int half, const v8i (&fa)[2], const int (&sa)[2], const v8i (&fb)[2], const int (&sb)[2]) {
#pragma unroll
        for (int a = 0; a < 2; a++)
#pragma unroll
            for (int b = 0; b < 2; b++)
                acc[half * 2 + a][b] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(
                    fb[b], fa[a], acc[half * 2 + a][b], 0, 0, 0, sb[b], 0, sa[a]);
        // keep the phase's MFMAs in front of the barrier that closes it (as g2::gemm_kernel_s)
        asm volatile("" ::"v"(acc[half * 2][0]), "v"(acc[half * 2][1]), "v"(acc[half * 2 + 1][0]),
                     "v"(acc[half * 2 + 1][1]));
    };
    const bool lagging = wave >= 4;
    issue_a(0, 0, false); issue_b(0, 0, false);
    issue_a(1, 1, my_tiles > 1); issue_b(1, 1, my_tiles > 1);  // nk >= 1; a missing step 1 issues nothing
    if (nk > 1 || my_tiles > 1) wait_vm(5);
    else wait_vm(0);
    int sl = 0;
    v8i fb[2], fa0[2], fa1[2];
    int sb_[2], sa0[2], sa1[2];
    for (int j = 0; j < my_tiles; j++) {
        const bool more = j + 1 < my_tiles;
        F8T(tr_t = __builtin_amdgcn_s_memtime();)
        bar();
        if (lagging) {
            __builtin_amdgcn_s_setprio(1);
            bar();
        }
        for (int kt = 0; kt < nk; kt++) {
            const char* img = smem + sl * SLOT_BYTES;
            const char* sc = img + 2 * IMG_BYTES;
            const int sl2 = (sl + 2) & 3;
#pragma unroll
            for (int b = 0; b < 2; b++) {
                fb[b] = frag(img + IMG_BYTES, wn * 64 + b * 32, lane);
                sb_[b] = scale_of(sc + 512, wn * 2 + b, lane);
            }
#pragma unroll
            for (int a = 0; a < 2; a++) {
                fa0[a] = frag(img, wm * 128 + a * 32, lane);
                sa0[a] = scale_of(sc, wm * 4 + a, lane);
            }
#if VIT_F8_ONEPHASE
            // one phase per step: every fragment of the step read before one barrier, the 8 MFMAs
            // after it (two barriers per step instead of four; 48 fragment VGPRs live at once)
#pragma unroll
            for (int a = 0; a < 2; a++) {
                fa1[a] = frag(img, wm * 128 + (2 + a) * 32, lane);
                sa1[a] = scale_of(sc, wm * 4 + 2 + a, lane);
            }
            issue_a(kt + 2, sl2, more);
            issue_b(kt + 2, sl2, more);
            // own pieces of the next step landed (the one after, 5 pieces, in flight); in a later
            // tile's first step they were retired before the previous epilogue
            if (kt > 0 || j == 0) {
                if (kt + 2 < nk || more) wait_vm_t(5);
                else wait_vm_t(0);
            }
            bar();
            mfma_half(0, fa0, sa0, fb, sb_);
            mfma_half(1, fa1, sa1, fb, sb_);
            bar();
            sl = (sl + 1) & 3;
            continue;
#endif
            issue_a(kt + 2, sl2, more);
            bar();
            mfma_half(0, fa0, sa0, fb, sb_);
            bar();
#pragma unroll
            for (int a = 0; a < 2; a++) {
                fa1[a] = frag(img, wm * 128 + (2 + a) * 32, lane);
                sa1[a] = scale_of(sc, wm * 4 + 2 + a, lane);
            }
            // own pieces of the next step landed (the A half of the one after, 3 pieces, in flight);
            // in a later tile's first step they were retired before the previous epilogue
            if (kt > 0 || j == 0) {
                if (kt + 2 < nk || more) wait_vm_t(3);
                else wait_vm_t(0);
            }
            issue_b(kt + 2, sl2, more);
            bar();
            mfma_half(1, fa1, sa1, fb, sb_);
            bar();
            sl = (sl + 1) & 3;
        }
        if (!lagging) bar();  // balance the stagger barrier
        F8T(const unsigned long long te = __builtin_amdgcn_s_memtime(); tr_main += te - tr_t; tr_t = te;)
        float bpre[8];
        staged_bias_prefetch<EPI>(p, lane, cur.tn0 + wn * 64, bpre);
        // through the builtin so hipcc knows no LDS-DMA is pending afterwards (as g2::gemm_kernel_s)
#if VIT_F8_EPI_WAIT_ASM
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#else
        __builtin_amdgcn_s_waitcnt(0x0070);
#endif
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // this tile's last two steps were in slots sl - 1, sl - 2 (mod 4); nk == 1: slot sl - 1 and
        // slot sl + 2, the next tile's step 2 slot, which nothing fills before the next barrier
        float* st = reinterpret_cast<float*>(smem + ((wave < 4 ? sl + 2 : sl + 3) & 3) * SLOT_BYTES + (wave & 3) * 8192);
        const int r = lane & 31, h = lane >> 5;
        auto stage_pass = [&](int pass) {
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const v16f& v = acc[pass][b];
                    *reinterpret_cast<f32x4_t*>(st + sq_off(r, b * 32 + 8 * q + 4 * h)) =
                        f32x4_t{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
                }
        };
        staged_epilogue_q_any<EPI, true>(p, stage_pass, st, lane, cur.tm0 + wm * 128, cur.tn0 + wn * 64, bpre);
        F8T(tr_epi += __builtin_amdgcn_s_memtime() - tr_t;)
        zero_acc();
        // recomputed rather than carried: nothing of the next tiles' sources stays live through the epilogue
        if (more) tile_src(j + 1, cur);
        if (j + 2 < my_tiles) tile_src(j + 2, nxt);
    }
#if VIT_F8_TRACE
    if (p.trace && blockIdx.x < 8 && lane == 0) {
        unsigned long long* r = p.trace + (blockIdx.x * 8 + wave) * 16;
        r[0] = tr_main; r[1] = tr_lgk; r[2] = tr_bar; r[3] = tr_vm; r[4] = tr_epi;
        r[5] = (unsigned long long)my_tiles; r[6] = (unsigned long long)nk;
        // the in-kernel shader clock: shader cycles over 100 MHz real-time ticks (MI355X guide, DVFS item 6)
        r[8] = __builtin_amdgcn_s_memtime() - tr_mt0; r[9] = __builtin_amdgcn_s_memrealtime() - tr_rt0;
    }
#endif
#undef F8T
}

// ------------------------------------------------------------------------------- quantizer
// MX block quantization of a [R][K] fp32 / bf16 matrix (row stride ldx elements) into fp8 e4m3
// rows (stride ldq bytes) + lane-native scales.  One wave per (32-row group, 64-deep k-step):
// lane (r, h) owns row 32g + r, k-block 2s + h (32 elements): amax -> the smallest power of two
// 2^X with amax / 2^X <= 448 (the e4m3 maximum; v_cvt_pk_fp8_f32 does not saturate) -> E8M0 byte
// X + 127 -> x * 2^-X (exact) rounded to nearest even by v_cvt_pk_fp8_f32.  Rows >= R get scale 0.
// One wave per (32-row group, 64-k step) was the round-1 form: a wave instruction moved 32 rows x
// 16 B (partial lines); the row-major form below replaced it (ViT-H/14 fp8: 18.8 -> 14.2 ms/step).
// blockIdx.y: matrix of a batch (x, q, sl advance by xs elements, qs bytes, ss bytes).
// Row-major: 8 consecutive elements per lane, 4 lanes per 32-element MX
// block (amax by two xor-shuffles), so a wave instruction moves 512 consecutive elements of a row
// (1 KiB of bf16 in, 512 B of fp8 out).  Rows R .. Rpad-1 write scale 0 and no data.
template <typename TX>
__global__ __launch_bounds__(256) void quantize_mx_rows_k(uint8_t* __restrict__ q, uint8_t* __restrict__ sl,
                                                          const TX* __restrict__ x, int R, int Rpad, int K,
                                                          long long ldx, long long ldq, int rg_tot, long long xs,
                                                          long long qs, long long ss) {
    x += blockIdx.y * xs;
    q += blockIdx.y * qs;
    sl += blockIdx.y * ss;
    const int kc = K / 8;  // granules per row (K % 64 == 0: a block's 4 granules never straddle rows)
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
    if (gid >= (long long)Rpad * kc) return;  // whole 4-lane groups (Rpad * kc % 4 == 0)
    const int row = (int)(gid / kc), g8 = (int)(gid - (long long)row * kc), col = g8 * 8;
    float v[8];
    if (row < R) {
        const TX* src = x + (long long)row * ldx + col;
        if constexpr (sizeof(TX) == 2) {
            const u32x4 w = *reinterpret_cast<const u32x4*>(src);
#pragma unroll
            for (int e = 0; e < 4; e++) {
                v[2 * e] = __uint_as_float(w[e] << 16);
                v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
            }
        } else {
            const float4 a = reinterpret_cast<const float4*>(src)[0], b = reinterpret_cast<const float4*>(src)[1];
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = 0.f;
    }
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 8; j++) amax = fmaxf(amax, fabsf(v[j]));
    amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
    amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
    const int sb = row < R ? mx_scale_byte(amax) : 0;
    if ((g8 & 3) == 0) {
        const int kb = col >> 5, ks = kb >> 1, h = kb & 1;
        sl[((long long)ks * rg_tot + (row >> 5)) * 64 + h * 32 + (row & 31)] = (uint8_t)sb;
    }
    if (row >= R) return;
    const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);  // 2^(127 - sb), exact
    int t0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, 0, false);
    t0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, t0, true);
    int t1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, 0, false);
    t1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, t1, true);
    *reinterpret_cast<uint2*>(q + (long long)row * ldq + col) = make_uint2((uint32_t)t0, (uint32_t)t1);
}

// Column-wise MX quantization for the weight gradients (dW = dout^T . inp reduces over the token
// axis, so both operands need MX blocks of 32 consecutive TOKENS): x [R tokens][C] bf16 (row
// stride ldx) -> q [C][Kp] e4m3 (row c = column c of x, Kp = R rounded up to 64; tokens R..Kp-1
// are zeros) + lane-native scales for C rows and K = Kp.  Equal, byte for byte, to
// quantize_mx_bf16 of the zero-padded transpose.  A workgroup takes 128 tokens x 64 columns: the
// tile is read with 16-B row loads into LDS (one 128-B line per token row), then lane c of wave w
// gathers column c over tokens 32w..32w+31 (a wave reads one 128-B LDS row per step: no bank
// conflicts), computes the block's scale and writes the 32 bytes of its block (the 4 waves fill
// one 128-B line of output row c).  Workgroups past column C write the padding rows' zero scales.
template <int TOK>  // tokens per workgroup (TOK / 32 waves)
__global__ __launch_bounds__(TOK * 2) void quantize_mx_cols_k(uint8_t* __restrict__ q, uint8_t* __restrict__ sl,
                                                             const uint16_t* __restrict__ x, int R, int C,
                                                             long long ldx, int Kp, int rg_tot, long long xs,
                                                             long long qs, long long ss) {
    constexpr int NT = TOK * 2;
    x += blockIdx.z * xs;  // blockIdx.z: matrix of a batch (the L layers of one weight kind)
    q += blockIdx.z * qs;
    sl += blockIdx.z * ss;
    __shared__ __attribute__((aligned(16))) uint16_t tile[TOK * 64];
    const int tok0 = blockIdx.x * TOK, col0 = blockIdx.y * 64;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int c = col0 + lane, tb = tok0 + 32 * wave;  // this lane's output row and token block
    if (col0 >= C) {  // padding rows of the scale layout (C .. Rpad-1): scale 0, no data
        if (tb < Kp) {
            const int kb = tb >> 5;
            sl[((long long)(kb >> 1) * rg_tot + (c >> 5)) * 64 + (kb & 1) * 32 + (c & 31)] = 0;
        }
        return;
    }
    u32x4 vl[4];  // all four pieces requested first (clamped rows: unconditional loads)
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int idx = i * NT + tid, row = idx >> 3, ch = idx & 7;
        vl[i] = *reinterpret_cast<const u32x4*>(x + (long long)min(tok0 + row, R - 1) * ldx + col0 + ch * 8);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int idx = i * NT + tid, row = idx >> 3, ch = idx & 7;
        *reinterpret_cast<u32x4*>(tile + row * 64 + ch * 8) = tok0 + row < R ? vl[i] : u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();
    if (tb >= Kp) return;
    float v[32];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        v[i] = __uint_as_float((uint32_t)tile[(32 * wave + i) * 64 + lane] << 16);
        amax = fmaxf(amax, fabsf(v[i]));
    }
    const int sb = mx_scale_byte(amax), kb = tb >> 5;
    sl[((long long)(kb >> 1) * rg_tot + (c >> 5)) * 64 + (kb & 1) * 32 + (c & 31)] = (uint8_t)sb;
    const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);  // 2^(127 - sb), exact
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        int t = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * j] * inv, v[4 * j + 1] * inv, 0, false);
        t = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * j + 2] * inv, v[4 * j + 3] * inv, t, true);
        w[j] = (uint32_t)t;
    }
    uint8_t* dst = q + (long long)c * Kp + tb;
    *reinterpret_cast<u32x4*>(dst) = u32x4{w[0], w[1], w[2], w[3]};
    *reinterpret_cast<u32x4*>(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
}

// Row- and column-wise MX in one pass over x (the fp8 trainer quantizes its GEMM inputs ln1, atty,
// ln2 and the output gradients dres3, dres2, dqkv both ways: row-wise for the forward / input-
// gradient GEMM, column-wise for the weight gradient; one read of x instead of two).  Same tile
// as quantize_mx_cols_k; while a lane holds its 8 elements of a token row on their way into LDS it
// also forms the row-wise block (4 lanes per 32-column block, as quantize_mx_rows_k), so both
// outputs equal the two separate quantizers byte for byte.  The column form covers tokens
// [tok_off, tok_off + ntok) of a [C][ldqc] matrix (one micro-batch of a larger token axis;
// tok_off % 64 == 0, tokens R .. ntok-1 are zero padding); the row form is [R][C] with its own
// Rpad (grid.x = Rpad / TOK covers the padding rows' zero scales).
// COLS = 128: two column groups per workgroup (8 waves), so every token row's row-form bytes
// leave as one full 128-B line (64 columns wrote half lines from two workgroups far apart).
template <int TOK, int COLS>
__global__ __launch_bounds__(TOK * 2 * (COLS / 64)) void quantize_mx_rowcol_k(uint8_t* __restrict__ qr, uint8_t* __restrict__ slr,
                                                               uint8_t* __restrict__ qc, uint8_t* __restrict__ slc,
                                                               const uint16_t* __restrict__ x, int R, int C,
                                                               long long ldx, int rgr_tot, long long ldqc, int tok_off,
                                                               int ntok, int rgc_tot) {
    constexpr int NT = TOK * 2 * (COLS / 64), G8 = COLS / 8;
    __shared__ __attribute__((aligned(16))) uint16_t tile[TOK * COLS];
    const int tok0 = blockIdx.x * TOK, col0 = blockIdx.y * COLS;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int cg = wave / (TOK / 32);  // the column phase: wave -> (64-column group, token block)
    const int c = col0 + 64 * cg + lane, tb = tok0 + 32 * (wave % (TOK / 32));
    if (col0 >= C) {  // padding rows of the column form's scale layout
        if (tb < ntok) {
            const int kb = (tok_off + tb) >> 5;
            slc[((long long)(kb >> 1) * rgc_tot + (c >> 5)) * 64 + (kb & 1) * 32 + (c & 31)] = 0;
        }
        return;
    }
    // every row piece requested before the first is used (the clamped row keeps the load unconditional;
    // a "zero, then load if in range" form made each iteration wait for its own load)
    constexpr int NI = TOK * G8 / NT;
    u32x4 wl[NI];
#pragma unroll
    for (int i = 0; i < NI; i++) {
        const int idx = i * NT + tid, row = idx / G8, ch = idx % G8;
        wl[i] = *reinterpret_cast<const u32x4*>(x + (long long)min(tok0 + row, R - 1) * ldx + col0 + ch * 8);
    }
#pragma unroll
    for (int i = 0; i < NI; i++) {
        const int idx = i * NT + tid, row = idx / G8, ch = idx % G8, tok = tok0 + row;
        const u32x4 w = tok < R ? wl[i] : u32x4{0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4*>(tile + row * COLS + ch * 8) = w;
        float v[8];
        float amax = 0.f;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            v[2 * e] = __uint_as_float(w[e] << 16);
            v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
            amax = fmaxf(amax, fmaxf(fabsf(v[2 * e]), fabsf(v[2 * e + 1])));
        }
        amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
        amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
        const int sb = tok < R ? mx_scale_byte(amax) : 0;
        if ((ch & 3) == 0) {
            const int kb = (col0 + ch * 8) >> 5;
            slr[((long long)(kb >> 1) * rgr_tot + (tok >> 5)) * 64 + (kb & 1) * 32 + (tok & 31)] = (uint8_t)sb;
        }
        if (tok < R) {
            const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);
            int t0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, 0, false);
            t0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, t0, true);
            int t1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, 0, false);
            t1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, t1, true);
            *reinterpret_cast<uint2*>(qr + (long long)tok * C + col0 + ch * 8) = make_uint2((uint32_t)t0, (uint32_t)t1);
        }
    }
    __syncthreads();
    if (tb >= ntok) return;
    float v[32];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        v[i] = __uint_as_float((uint32_t)tile[(tb - tok0 + i) * COLS + 64 * cg + lane] << 16);
        amax = fmaxf(amax, fabsf(v[i]));
    }
    const int sb = mx_scale_byte(amax), kb = (tok_off + tb) >> 5;
    slc[((long long)(kb >> 1) * rgc_tot + (c >> 5)) * 64 + (kb & 1) * 32 + (c & 31)] = (uint8_t)sb;
    const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);
    uint32_t w[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        int t = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * j] * inv, v[4 * j + 1] * inv, 0, false);
        t = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * j + 2] * inv, v[4 * j + 3] * inv, t, true);
        w[j] = (uint32_t)t;
    }
    uint8_t* dst = qc + (long long)c * ldqc + tok_off + tb;
    *reinterpret_cast<u32x4*>(dst) = u32x4{w[0], w[1], w[2], w[3]};
    *reinterpret_cast<u32x4*>(dst + 16) = u32x4{w[4], w[5], w[6], w[7]};
}

// LayerNorm forward straight into both MX forms.  In the fp8 trainer ln1 / ln2 feed only the qkv /
// fc GEMM (row form) and the qkv / fc weight gradients (column form), so the bf16 tensor that
// ln_forward_bf16 stored and quantize_mx_rowcol_bf16 read back (4 B per element) never exists.
// A workgroup takes 32 tokens (8 waves x 4 rows; C = 256 NV): each wave normalises its rows with
// ln_vec_stats / ln_vec_y (ln_common.h, the arithmetic of ln_fwd_vec_k), rounds to bf16, writes the row form
// (8 lanes per 32-channel block: 3 xor-shuffles for the block amax; 256 consecutive bytes per wave
// store) and puts the bf16 row into an LDS tile; after one barrier each thread takes a channel and
// writes its column block of the 32 tokens (as quantize_mx_cols_k).  Both forms equal
// ln_forward_bf16 + quantize_mx_rowcol_bf16 byte for byte.  Rows R .. Rpad-1 write zero row-form
// scales; tokens R .. ntok-1 of the column form are zero padding (as quantize_mx_rowcol_k).
// (two rows of loads in flight per wave: <= 128 VGPRs up to C = 1280, where two 80-KiB workgroups share a CU)
// WB: the lane's LN weight / bias float4s held in registers for the wave's 4 rows (else re-read per row)
// RPW: rows per wave (4: 8 waves, 512 threads, the default; 2: 16 waves, 1024 threads, every row's loads
// issued at once: VIT_LNMX_RPW=2, measured 39.1 vs 36.4 us at 16448 x 1280, tools/bench_lnmx.py).
// Standalone it is at par with the pair it replaces (36.4 vs 37.5 us per ViT-H/14 micro-batch; 64.6 vs
// 67.7 us for B = 128): a 32-token tile holds 80 KiB of LDS, so two workgroups per CU and 514 tiles
// for 512 slots; in the train step the other micro-batch stream fills the gaps.
template <int NV, bool WB, int RPW>
__global__ __launch_bounds__(64 * 32 / RPW, (RPW == 2 || NV <= 5 ? 4 : 2)) void ln_fwd_mx_k(uint8_t* __restrict__ qr, uint8_t* __restrict__ slr,
                                                   uint8_t* __restrict__ qc, uint8_t* __restrict__ slc,
                                                   float* __restrict__ mean, float* __restrict__ rstd,
                                                   const float* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ b, int R, int rgr_tot, long long ldqc,
                                                   int tok_off, int ntok, int rgc_tot, int xmap, int nmain,
                                                   int ntiles, uint16_t* __restrict__ ybf) {
    constexpr int C = 256 * NV, TOK = 32, NT = 64 * TOK / RPW;
    __shared__ __attribute__((aligned(16))) uint16_t tile[TOK * C];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    if ((int)blockIdx.x >= nmain) {
        // the rows of the last, partial round of tiles (one per wave; no tile): row form, mean /
        // rstd, and the bf16 row into ybf for the launcher's follow-up column quantize
        const int q = nmain * TOK + ((int)blockIdx.x - nmain) * (NT / 64) + wave;
        if (q >= ntiles * TOK) return;
        if (q >= R) {
#pragma unroll
            for (int j = 0; j < NV; j++) {
                const int kb = (lane + 64 * j) >> 3;
                if ((lane & 7) == 0) slr[((long long)(kb >> 1) * rgr_tot + (q >> 5)) * 64 + (kb & 1) * 32 + (q & 31)] = 0;
            }
            return;
        }
        float4 xv[NV];
        const float4* x4 = reinterpret_cast<const float4*>(x + (long long)q * C);
#pragma unroll
        for (int j = 0; j < NV; j++) xv[j] = x4[lane + 64 * j];
        float m, rs;
        ln_vec_stats<NV>(xv, C, m, rs);
#pragma unroll
        for (int j = 0; j < NV; j++) {
            const int k = lane + 64 * j, kb = k >> 3;
            const float4 y = ln_vec_y(xv[j], reinterpret_cast<const float4*>(w)[k], reinterpret_cast<const float4*>(b)[k], m, rs);
            const uint2 h = make_uint2(pack_bf16x2(y.x, y.y), pack_bf16x2(y.z, y.w));
            reinterpret_cast<uint2*>(ybf + (long long)(q - nmain * TOK) * C)[k] = h;
            const float f0 = __uint_as_float(h.x << 16), f1 = __uint_as_float(h.x & 0xffff0000u);
            const float f2 = __uint_as_float(h.y << 16), f3 = __uint_as_float(h.y & 0xffff0000u);
            float amax = fmaxf(fmaxf(fabsf(f0), fabsf(f1)), fmaxf(fabsf(f2), fabsf(f3)));
            amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
            amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
            amax = fmaxf(amax, __shfl_xor(amax, 4, 64));
            const int sb = mx_scale_byte(amax);
            if ((lane & 7) == 0)
                slr[((long long)(kb >> 1) * rgr_tot + (q >> 5)) * 64 + (kb & 1) * 32 + (q & 31)] = (uint8_t)sb;
            const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);
            int t8 = __builtin_amdgcn_cvt_pk_fp8_f32(f0 * inv, f1 * inv, 0, false);
            t8 = __builtin_amdgcn_cvt_pk_fp8_f32(f2 * inv, f3 * inv, t8, true);
            reinterpret_cast<uint32_t*>(qr + (long long)q * C)[k] = (uint32_t)t8;
        }
        if (lane == 0) {
            mean[q] = m;
            rstd[q] = rs;
        }
        return;
    }
    // xmap: within each group of 32 workgroups, the 4 tiles of one 128-token span go to workgroups
    // 8 apart (the same XCD, dispatched together), so the column form's 32-B pieces of a 128-B line
    // meet in one L2 instead of leaving four L2s as partial lines
    int t = blockIdx.x;
    if (xmap && (int)(blockIdx.x | 31) < nmain) t = (blockIdx.x & ~31) + (blockIdx.x & 7) * 4 + ((blockIdx.x >> 3) & 3);
    const int tok0 = t * TOK;
    // row i + 1 in flight while row i reduces, row i + 2 requested once row i's inputs are dead
    // (clamped rows: unconditional loads).  A branch-free form (zero-selects, buffer stores that drop
    // rows >= R, every lane storing the scale bytes) let hipcc count the waits per row instead of
    // vmcnt(0), but spilled at 4 rows per wave and measured slower at 2 (39.1 vs 36.4 us, 16448 x 1280)
    float4 v[2][NV];
    auto load = [&](int i) {
        const float4* x4 = reinterpret_cast<const float4*>(x + (long long)min(tok0 + wave * RPW + i, R - 1) * C);
#pragma unroll
        for (int j = 0; j < NV; j++) v[i & 1][j] = x4[lane + 64 * j];
    };
    load(0);
    if (RPW > 1) load(1);
    // the LN weight / bias float4s of this lane, once per wave (not a dependent load per row)
    float4 w4[NV], b4[NV];
    if constexpr (WB) {
#pragma unroll
        for (int j = 0; j < NV; j++) {
            w4[j] = reinterpret_cast<const float4*>(w)[lane + 64 * j];
            b4[j] = reinterpret_cast<const float4*>(b)[lane + 64 * j];
        }
    }
#pragma unroll
    for (int i = 0; i < RPW; i++) {
        const int r = wave * RPW + i, tok = tok0 + r;
        uint2* trow = reinterpret_cast<uint2*>(tile + r * C);
        if (tok >= R) {  // padding row: zero tile row (the column form's padding tokens), scale 0
            if (i + 2 < RPW) load(i + 2);
#pragma unroll
            for (int j = 0; j < NV; j++) {
                const int k = lane + 64 * j, kb = k >> 3;
                trow[k] = make_uint2(0u, 0u);
                if ((lane & 7) == 0)
                    slr[((long long)(kb >> 1) * rgr_tot + (tok >> 5)) * 64 + (kb & 1) * 32 + (tok & 31)] = 0;
            }
            continue;
        }
        float m, rs;
        ln_vec_stats<NV>(v[i & 1], C, m, rs);
        uint2 hv[NV];
#pragma unroll
        for (int j = 0; j < NV; j++) {
            const int k = lane + 64 * j;
            const float4 y = WB ? ln_vec_y(v[i & 1][j], w4[j], b4[j], m, rs)
                                : ln_vec_y(v[i & 1][j], reinterpret_cast<const float4*>(w)[k],
                                           reinterpret_cast<const float4*>(b)[k], m, rs);
            hv[j] = make_uint2(pack_bf16x2(y.x, y.y), pack_bf16x2(y.z, y.w));
        }
        if (i + 2 < RPW) load(i + 2);  // row i's inputs are dead: its buffer takes row i + 2
#pragma unroll
        for (int j = 0; j < NV; j++) {
            const int k = lane + 64 * j, kb = k >> 3;  // channels 4k .. 4k+3, MX block 4k / 32
            const uint2 h = hv[j];
            trow[k] = h;
            const float f0 = __uint_as_float(h.x << 16), f1 = __uint_as_float(h.x & 0xffff0000u);
            const float f2 = __uint_as_float(h.y << 16), f3 = __uint_as_float(h.y & 0xffff0000u);
            float amax = fmaxf(fmaxf(fabsf(f0), fabsf(f1)), fmaxf(fabsf(f2), fabsf(f3)));
            amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
            amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
            amax = fmaxf(amax, __shfl_xor(amax, 4, 64));
            const int sb = mx_scale_byte(amax);
            if ((lane & 7) == 0)
                slr[((long long)(kb >> 1) * rgr_tot + (tok >> 5)) * 64 + (kb & 1) * 32 + (tok & 31)] = (uint8_t)sb;
            const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);  // 2^(127 - sb), exact
            int t = __builtin_amdgcn_cvt_pk_fp8_f32(f0 * inv, f1 * inv, 0, false);
            t = __builtin_amdgcn_cvt_pk_fp8_f32(f2 * inv, f3 * inv, t, true);
            reinterpret_cast<uint32_t*>(qr + (long long)tok * C)[k] = (uint32_t)t;
        }
        if (lane == 0) {
            mean[tok] = m;
            rstd[tok] = rs;
        }
    }
    __syncthreads();
    if (tok0 >= ntok) return;
    const int kb = (tok_off + tok0) >> 5;
    for (int c = tid; c < C; c += NT) {
        float cv[TOK];
        float amax = 0.f;
#pragma unroll
        for (int t = 0; t < TOK; t++) {
            cv[t] = __uint_as_float((uint32_t)tile[t * C + c] << 16);
            amax = fmaxf(amax, fabsf(cv[t]));
        }
        const int sb = mx_scale_byte(amax);
        slc[((long long)(kb >> 1) * rgc_tot + (c >> 5)) * 64 + (kb & 1) * 32 + (c & 31)] = (uint8_t)sb;
        const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);
        uint32_t wd[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            int t = __builtin_amdgcn_cvt_pk_fp8_f32(cv[4 * j] * inv, cv[4 * j + 1] * inv, 0, false);
            t = __builtin_amdgcn_cvt_pk_fp8_f32(cv[4 * j + 2] * inv, cv[4 * j + 3] * inv, t, true);
            wd[j] = (uint32_t)t;
        }
        uint8_t* dst = qc + (long long)c * ldqc + tok_off + tok0;
        *reinterpret_cast<u32x4*>(dst) = u32x4{wd[0], wd[1], wd[2], wd[3]};
        *reinterpret_cast<u32x4*>(dst + 16) = u32x4{wd[4], wd[5], wd[6], wd[7]};
    }
}

// LayerNorm backward of the residual-gradient stream straight into both MX forms of its bf16 plane
// (fp8 trainer: dres3 / dres2 feed the fcproj / attproj input-gradient GEMMs (row form) and weight
// gradients (column form), so the row + column quantizer's read of the bf16 plane goes away; the
// bf16 + lo8 planes are still written, the next LayerNorm backward reads them).  Per row exactly
// ln_bwd_vec_k<NV, bf16, true> (ln_bwd_row, ln_common.h): dres_out = dres_in + LN'(dy) as bf16 + lo8.
// A persistent workgroup (8 waves) walks 32-token tiles (4 rows per wave, the next row's loads in
// flight); each wave keeps its dW / db column partials in its LDS rows and its dres column sums in
// registers (the lane's 4 NV columns),
// writes the row form of each row (8 lanes per 32-channel block) and the bf16 row into an LDS tile,
// and after the tile's barrier every thread writes a channel's 32-token column block (as
// ln_fwd_mx_k).  At the end the 8 waves' partials are summed in wave order into the workgroup's
// partial row part[blockIdx.x][2C | 3C] (dw | db | dsum); rows gridDim.x .. nparts-1 are zeroed, so
// the caller reduces the same nparts rows as for ln_bwd_vec_k.  hi / lo and both MX forms equal
// ln_backward_bf16_stream + quantize_mx_rowcol_bf16 byte for byte; the partial sums group rows
// differently (a deterministic fixed order, not the same fp32 association).
struct LnbMx {
    bf16_t* hi_out;
    uint8_t* lo_out;
    const bf16_t* hi_in;
    const uint8_t* lo_in;
    const bf16_t* dout;
    const float* inp;
    const float* w;
    const float* mean;
    const float* rstd;
    float* part;
    int nsum, nparts;
    uint8_t *qr, *slr, *qc, *slc;
    int R, ntiles, nmain, rgr_tot, tok_off, ntok, rgc_tot;
    long long ldqc;
};
__device__ __forceinline__ float4 bf4_f32(uint2 u) {
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xffff0000u));
}
template <int NV>
__global__ __launch_bounds__(512, 2) void ln_bwd_mx_k(LnbMx a) {
    constexpr int C = 256 * NV, TOK = 32, RPW = 4, NT = 512;
    __shared__ __attribute__((aligned(16))) uint16_t tile[TOK * C];  // 80 KiB at C = 1280 (ps partials at the end)
    // dW / db column partials per wave in LDS (lane-owned entries: no synchronisation until the end),
    // dres column sums in registers: 80 + 80 KiB = the whole LDS at C = 1280
    __shared__ __attribute__((aligned(16))) float4 sp[8][2][NV * 64];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    float4 ps[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) {
        ps[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        sp[wave][0][lane + 64 * j] = sp[wave][1][lane + 64 * j] = ps[j];
    }
    // the wave's row sequence: tile t = blockIdx.x + n * gridDim.x, rows t * 32 + wave * 4 + i
    uint2 pdy[NV], pri[NV];
    float4 px[NV];
    uint32_t plo[NV];
    float pmu = 0.f, prs = 0.f;
    auto fetch = [&](int row) {
        const int r = min(row, a.R - 1);
        const long long o = (long long)r * C;
#pragma unroll
        for (int j = 0; j < NV; j++) {
            const int k = lane + 64 * j;
            pdy[j] = reinterpret_cast<const uint2*>(a.dout + o)[k];
            px[j] = reinterpret_cast<const float4*>(a.inp + o)[k];
            pri[j] = reinterpret_cast<const uint2*>(a.hi_in + o)[k];
            plo[j] = reinterpret_cast<const uint32_t*>(a.lo_in + o)[k];
        }
        pmu = a.mean[r];
        prs = a.rstd[r];
    };
    // one row from the fetched registers (fetch() for the next row is issued by the caller's `next`
    // before this row's arithmetic); trow: the row's LDS tile row, or nullptr (leftover rows)
    auto do_row = [&](int tok, uint2* trow, int next) {
        float4 dy[NV], xr[NV], ri[NV];
#pragma unroll
        for (int j = 0; j < NV; j++) {
            dy[j] = bf4_f32(pdy[j]);
            xr[j] = px[j];
            const float4 h = bf4_f32(pri[j]);
            const uint32_t q = plo[j];
            ri[j] = make_float4(lo8_decode(h.x, q), lo8_decode(h.y, q >> 8), lo8_decode(h.z, q >> 16),
                                lo8_decode(h.w, q >> 24));
        }
        const float mu = pmu, rs = prs;
        if (next >= 0) fetch(next);
        __builtin_amdgcn_sched_barrier(0);
        if (tok >= a.R) {  // padding row: zero tile row, zero row-form scales, no outputs
#pragma unroll
            for (int j = 0; j < NV; j++) {
                const int k = lane + 64 * j, kb = k >> 3;
                if (trow) trow[k] = make_uint2(0u, 0u);
                if ((lane & 7) == 0)
                    a.slr[((long long)(kb >> 1) * a.rgr_tot + (tok >> 5)) * 64 + (kb & 1) * 32 + (tok & 31)] = 0;
            }
            return;
        }
        float4 nr[NV], dv[NV], w4[NV];  // the LN weight re-read per row (L1): registers go to the partials
#pragma unroll
        for (int j = 0; j < NV; j++) w4[j] = reinterpret_cast<const float4*>(a.w)[lane + 64 * j];
        ln_bwd_row<NV>(dy, xr, w4, mu, rs, C, nr, dv);
        const long long o = (long long)tok * C;
#pragma unroll
        for (int j = 0; j < NV; j++) {
            const int k = lane + 64 * j, kb = k >> 3;
            {
                float4 b = sp[wave][1][k], w = sp[wave][0][k];
                b.x += dy[j].x; b.y += dy[j].y; b.z += dy[j].z; b.w += dy[j].w;
                w.x += nr[j].x * dy[j].x; w.y += nr[j].y * dy[j].y;
                w.z += nr[j].z * dy[j].z; w.w += nr[j].w * dy[j].w;
                sp[wave][1][k] = b;
                sp[wave][0][k] = w;
            }
            const float4 tv = make_float4(ri[j].x + dv[j].x, ri[j].y + dv[j].y, ri[j].z + dv[j].z, ri[j].w + dv[j].w);
            ps[j].x += tv.x; ps[j].y += tv.y; ps[j].z += tv.z; ps[j].w += tv.w;
            const uint2 h = make_uint2(pack_bf16x2(tv.x, tv.y), pack_bf16x2(tv.z, tv.w));
            reinterpret_cast<uint2*>(a.hi_out + o)[k] = h;
            reinterpret_cast<uint32_t*>(a.lo_out + o)[k] =
                lo8_encode(tv.x, __uint_as_float(h.x << 16)) | (lo8_encode(tv.y, __uint_as_float(h.x & 0xffff0000u)) << 8) |
                (lo8_encode(tv.z, __uint_as_float(h.y << 16)) << 16) |
                (lo8_encode(tv.w, __uint_as_float(h.y & 0xffff0000u)) << 24);
            if (trow) trow[k] = h;
            const float4 f = bf4_f32(h);
            float amax = fmaxf(fmaxf(fabsf(f.x), fabsf(f.y)), fmaxf(fabsf(f.z), fabsf(f.w)));
            amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
            amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
            amax = fmaxf(amax, __shfl_xor(amax, 4, 64));
            const int sb = mx_scale_byte(amax);
            if ((lane & 7) == 0)
                a.slr[((long long)(kb >> 1) * a.rgr_tot + (tok >> 5)) * 64 + (kb & 1) * 32 + (tok & 31)] = (uint8_t)sb;
            const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);
            int q8 = __builtin_amdgcn_cvt_pk_fp8_f32(f.x * inv, f.y * inv, 0, false);
            q8 = __builtin_amdgcn_cvt_pk_fp8_f32(f.z * inv, f.w * inv, q8, true);
            reinterpret_cast<uint32_t*>(a.qr + o)[k] = (uint32_t)q8;
        }
    };
    // whole tiles: the first nmain (a multiple of gridDim.x: every workgroup takes the same number)
    int t = blockIdx.x;
    if (t < a.nmain) fetch(t * TOK + wave * RPW);
    for (; t < a.nmain; t += gridDim.x) {
        const int tok0 = t * TOK;
#pragma unroll
        for (int i = 0; i < RPW; i++) {
            const int r = wave * RPW + i, tok = tok0 + r;
            // the next row of the sequence (the last one re-fetches itself: every load unconditional)
            const int nt = i + 1 < RPW ? t : t + (int)gridDim.x;
            const int nr_ = i + 1 < RPW ? i + 1 : 0;
            do_row(tok, reinterpret_cast<uint2*>(tile + r * C), nt < a.nmain ? nt * TOK + wave * RPW + nr_ : tok);
        }
        __syncthreads();
        if (tok0 < a.ntok) {
            const int kb = (a.tok_off + tok0) >> 5;
            for (int c = tid; c < C; c += NT) {
                float cv[TOK];
                float amax = 0.f;
#pragma unroll
                for (int u = 0; u < TOK; u++) {
                    cv[u] = __uint_as_float((uint32_t)tile[u * C + c] << 16);
                    amax = fmaxf(amax, fabsf(cv[u]));
                }
                const int sb = mx_scale_byte(amax);
                a.slc[((long long)(kb >> 1) * a.rgc_tot + (c >> 5)) * 64 + (kb & 1) * 32 + (c & 31)] = (uint8_t)sb;
                const float inv = __uint_as_float((uint32_t)(254 - sb) << 23);
                uint32_t wd[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    int q8 = __builtin_amdgcn_cvt_pk_fp8_f32(cv[4 * j] * inv, cv[4 * j + 1] * inv, 0, false);
                    q8 = __builtin_amdgcn_cvt_pk_fp8_f32(cv[4 * j + 2] * inv, cv[4 * j + 3] * inv, q8, true);
                    wd[j] = (uint32_t)q8;
                }
                uint8_t* dst = a.qc + (long long)c * a.ldqc + a.tok_off + tok0;
                *reinterpret_cast<u32x4*>(dst) = u32x4{wd[0], wd[1], wd[2], wd[3]};
                *reinterpret_cast<u32x4*>(dst + 16) = u32x4{wd[4], wd[5], wd[6], wd[7]};
            }
        }
        __syncthreads();  // the tile is rewritten by the next one
    }
    // the rows of the last, partial round of tiles: one row per wave across all workgroups (their
    // column form is written by the launcher's follow-up quantize over these rows)
    for (int q = a.nmain * TOK + (int)blockIdx.x * 8 + wave; q < a.ntiles * TOK; q += (int)gridDim.x * 8) {
        fetch(q);
        do_row(q, nullptr, -1);
    }
    // the 8 waves' column partials -> the workgroup's partial row, waves added in order 0 .. 7
    float4* sps = reinterpret_cast<float4*>(tile);  // dres sums [8][NV * 64] (the tile is free after the loop)
#pragma unroll
    for (int j = 0; j < NV; j++) sps[wave * NV * 64 + lane + 64 * j] = ps[j];
    __syncthreads();
    float* prow = a.part + (long long)blockIdx.x * a.nsum;
    for (int k = tid; k < NV * 64; k += NT) {
        float4 w = sp[0][0][k], b = sp[0][1][k], z = sps[k];
#pragma unroll
        for (int u = 1; u < 8; u++) {
            const float4 w2 = sp[u][0][k], b2 = sp[u][1][k], z2 = sps[u * NV * 64 + k];
            w.x += w2.x; w.y += w2.y; w.z += w2.z; w.w += w2.w;
            b.x += b2.x; b.y += b2.y; b.z += b2.z; b.w += b2.w;
            z.x += z2.x; z.y += z2.y; z.z += z2.z; z.w += z2.w;
        }
        reinterpret_cast<float4*>(prow)[k] = w;
        reinterpret_cast<float4*>(prow + C)[k] = b;
        if (a.nsum == 3 * C) reinterpret_cast<float4*>(prow + 2 * C)[k] = z;
    }
    // the partial rows no workgroup owns (gridDim.x .. nparts-1) are zeros
    for (int rr = (int)gridDim.x + (int)blockIdx.x; rr < a.nparts; rr += gridDim.x)
        for (int i = tid; i < a.nsum; i += NT) a.part[(long long)rr * a.nsum + i] = 0.f;
}
}  // namespace f8

long long mx_rows_padded(long long rows) { return (rows + 255) / 256 * 256; }
size_t mx_scale_bytes(long long rows, int K) { return (size_t)mx_rows_padded(rows) / 32 * (K / 64) * 64; }

bool gemm_fp8_supported(const GemmArgs& a) {
    auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    return a.a_kcontig && a.b_kcontig && a.K % 64 == 0 && a.lda % 16 == 0 && a.ldb % 16 == 0 &&
           a.N % 4 == 0 && a.ldc % 4 == 0 && al16(a.A) && al16(a.B) && a.a_scale && a.b_scale &&
           a.epi != EPI_F32_SLAB && (a.epi != EPI_F32_ATOMIC || a.N % 4 == 0) &&
           // fused MX output: whole 32-column blocks, GELU/GELU'/product epilogues only (4 lanes per block)
           (!a.mx_q || (a.mx_s && a.N % 32 == 0 && epi_mx(a.epi))) &&
           (!a.mxc_q || (a.mxc_s && epi_mx(a.epi) && a.M % 64 == 0 && a.N % 64 == 0 && a.mxc_off % 64 == 0 &&
                         a.mxc_off >= 0 && a.mxc_ld % 16 == 0 && a.mxc_off + a.M <= a.mxc_ld && al16(a.mxc_q))) &&
           // an omitted bf16 output needs an MX copy in its place
           (a.C2 || !(a.epi == EPI_BF16_GELU || a.epi == EPI_BF16_GELU_D) || a.mx_q || a.mxc_q) &&
           (a.C || !epi_aux16(a.epi) || a.mx_q || a.mxc_q);
}

void gemm_fp8(const GemmArgs& a, hipStream_t s) {
    if (a.M <= 0 || a.N <= 0) return;
    if (!gemm_fp8_supported(a)) {
        set_error("gemm_fp8: unsupported shape/layout M=%d N=%d K=%d lda=%lld ldb=%lld epi=%d", a.M, a.N,
                  a.K, a.lda, a.ldb, a.epi);
        return;
    }
    const int tiles = cdiv(a.M, f8::BM) * cdiv(a.N, f8::BN);
    // EPI_F32_ATOMIC (the weight gradients, K = the token count): K-split partials into fp32 slabs
    // + one fixed-order reduce (no atomics; deterministic), a single split accumulates in place
    int split = 1;
    GemmArgs b = a;
    float* slab = nullptr;
    if (a.epi == EPI_F32_ATOMIC) {
        // the bf16 weight gradients' r06 rule (gemm.hip choose_split_g4): the smallest split filling
        // >= 80 % of the 256 slots in one round, before the round-5 rule (ViT-H/14 fp8 qkv wgrad 10 -> 3
        // splits, proj 10 -> 9: 1094 / 1091 vs 1081 / 1075 img/s, two interleaved rounds,
        // profiles/r06_g4_slots.txt); VIT_F8_SPLIT_RULE=0: the round-5 rule alone
        static const bool one_round = [] {
            const char* e = getenv("VIT_F8_SPLIT_RULE");
            return !(e && e[0] == '0');
        }();
        // fill target 45 % (VIT_F8_FILL): ViT-H/14 fp8 80 -> 60 -> 45 -> 35 -> 25 %: 1091 -> 1103 -> 1108 ->
        // 1103 -> 1092 img/s (interleaved rounds, profiles/r06_f8_fill.txt): half-filled rounds of fewer
        // splits, the micro-batch streams' kernels beside them
        static const double fill = [] {
            const char* e = getenv("VIT_F8_FILL");
            const int v = e ? atoi(e) : 45;
            return (v >= 20 && v <= 100 ? v : 45) / 100.0;
        }();
        split = 0;
        if (a.splitk <= 0 && one_round) {
            const double f = a.fill_pct > 0 ? a.fill_pct / 100.0 : fill;
            const int nk = a.K / f8::KB, s1 = (int)((f * 256 + tiles - 1) / tiles);
            if (s1 >= 1 && tiles * s1 <= 256 && nk / s1 >= 16) split = s1;
        }
        if (!split) split = a.splitk > 0 ? a.splitk : choose_split_waves(tiles, a.K / f8::KB);
        if (split < 1) split = 1;
        const int kchunk = cdiv(cdiv(a.K, split), f8::KB) * f8::KB;
        split = cdiv(a.K, kchunk);
        if (split > 1) {
            if (!(slab = slab_buffer(a, split))) return;
            b.epi = EPI_F32_SLAB; b.C = slab; b.ldc = a.N;
        } else {
            b.epi = EPI_F32_ACC;
        }
    }
    f8::F8Params fp;
    fp.p = make_gemm_params(b, cdiv(cdiv(a.K, split), f8::KB) * f8::KB);
    float* cs_rows = colsum_rows_begin(a);
    if ((a.colsum_out || a.colsum_part) && !cs_rows) return;
    fp.p.colsum_out = cs_rows;
    fp.p.tiles = tiles;
    // tile order: make_gemm_params' rule (grouped for K <= 768).  Extending it to the fp8 A panels'
    // byte size (K <= 1536) measured 1059 / 1060 vs 1062 / 1064 img/s on ViT-H/14 fp8: not taken
    fp.sa = (const uint8_t*)a.a_scale;
    fp.sb = (const uint8_t*)a.b_scale;
    fp.rga_tot = (int)(mx_rows_padded(a.M) / 32);
    fp.rgb_tot = (int)(mx_rows_padded(a.N) / 32);
    // persistent streaming engine (production GEMM variant, gemm_streaming()): no split-K, 32-bit
    // DMA offsets; not for the aux x product epilogues (6 / 9: with both MX outputs their epilogue
    // outgrows the registers the streaming state leaves and spills; measured 8 % slower than the
    // one-tile kernel on the ViT-H/14 fcproj input gradient)
    // (its DMA ring fetches two K-steps ahead across one tile boundary: K >= 2 steps)
    if (split == 1 && gemm_streaming() && b.epi != EPI_F32_ACC && !epi_aux16(b.epi) && a.K >= 2 * f8::KB &&
        (long long)a.M * a.lda < (1LL << 31) &&
        (long long)a.N * a.ldb < (1LL << 31)) {
        const int cus = gemm_persist_grid();
        const dim3 pg(tiles < cus ? tiles : cus);
        switch (b.epi) {
#define VIT_CASE(E) \
    case E: f8::gemm_kernel_s<E><<<pg, f8::NT, 0, s>>>(fp); break;
            VIT_CASE(EPI_F32_STORE)
            VIT_CASE(EPI_BF16_STORE)
            VIT_CASE(EPI_BF16_GELU)
            VIT_CASE(EPI_F32_RESID)
            VIT_CASE(EPI_BF16_DGELU)
            VIT_CASE(EPI_BF16_GELU_D)
            VIT_CASE(EPI_BF16_MUL)
#undef VIT_CASE
            default: set_error("gemm_fp8: unsupported epilogue %d", b.epi); return;
        }
        after_launch("gemm_fp8");
        count_hit(VIT_HIT_GEMM_FP8 + b.epi);
        colsum_rows_end(a, cs_rows, s);
        return;
    }
    switch (b.epi) {
#define VIT_CASE(E) \
    case E: f8::gemm_kernel<E><<<dim3(tiles, split), f8::NT, 0, s>>>(fp); break;
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
        default: set_error("gemm_fp8: unsupported epilogue %d", a.epi); return;
    }
    after_launch("gemm_fp8");
    count_hit(VIT_HIT_GEMM_FP8 + b.epi);
    if (slab) slab_reduce(a, slab, split, s);
    colsum_rows_end(a, cs_rows, s);
}

template <typename TX>
static void quantize_mx(uint8_t* q, uint8_t* sl, const TX* x, long long R, int K, long long ldx,
                        long long ldq, int count, long long xs, long long qs, long long ss, hipStream_t s) {
    if (R <= 0 || count <= 0) return;
    if (K % 64 || ldx % (16 / sizeof(TX)) || ldq % 16 || xs % (16 / sizeof(TX)) || qs % 16 ||
        ((uintptr_t)x & 15) || ((uintptr_t)q & 15) || R >= (1LL << 31)) {
        set_error("quantize_mx: K %% 64 and 16-B aligned rows required (K=%d)", K);
        return;
    }
    const long long rp = mx_rows_padded(R);
    const int rg = (int)(rp / 32);
    f8::quantize_mx_rows_k<TX><<<dim3(cdiv(rp * (K / 8), 256), count), 256, 0, s>>>(q, sl, x, (int)R, (int)rp, K, ldx,
                                                                                      ldq, rg, xs, qs, ss);
    after_launch("quantize_mx");
}
void quantize_mx_bf16(uint8_t* q, uint8_t* sl, const bf16_t* x, long long R, int K, long long ldx,
                      long long ldq, hipStream_t s) {
    quantize_mx<bf16_t>(q, sl, x, R, K, ldx, ldq, 1, 0, 0, 0, s);
}
void quantize_mx_f32(uint8_t* q, uint8_t* sl, const float* x, long long R, int K, long long ldx,
                     long long ldq, hipStream_t s) {
    quantize_mx<float>(q, sl, x, R, K, ldx, ldq, 1, 0, 0, 0, s);
}
long long mx_cols_kp(long long R) { return (R + 63) / 64 * 64; }
void quantize_mx_cols_batched_bf16(uint8_t* q, uint8_t* sl, const bf16_t* x, long long R, int C, long long ldx,
                                   int count, long long xs, long long qs, long long ss, hipStream_t s) {
    if (R <= 0 || C <= 0 || count <= 0) return;
    if (C % 64 || ldx % 8 || xs % 8 || qs % 16 || ((uintptr_t)x & 15) || ((uintptr_t)q & 15) || R >= (1LL << 30)) {
        set_error("quantize_mx_cols: C %% 64 == 0 and 16-B aligned rows required (C=%d)", C);
        return;
    }
    const int kp = (int)mx_cols_kp(R);
    const int cpad = (int)mx_rows_padded(C);
    // 128 tokens per workgroup (256 measured within 2 %, r03)
    f8::quantize_mx_cols_k<128><<<dim3(cdiv(kp, 128), cpad / 64, count), 256, 0, s>>>(
        q, sl, (const uint16_t*)x, (int)R, C, ldx, kp, cpad / 32, xs, qs, ss);
    after_launch("quantize_mx_cols");
}
void quantize_mx_cols_bf16(uint8_t* q, uint8_t* sl, const bf16_t* x, long long R, int C, long long ldx, hipStream_t s) {
    quantize_mx_cols_batched_bf16(q, sl, x, R, C, ldx, 1, 0, 0, 0, s);
}
bool quantize_mx_rowcol_bf16(uint8_t* qr, uint8_t* slr, uint8_t* qc, uint8_t* slc, const bf16_t* x, long long R,
                             int C, long long ldx, long long ldqc, long long tok_off, long long ntok, hipStream_t s) {
    if (R <= 0 || C <= 0) return true;
    if (C % 64 || ldx % 8 || ldqc % 16 || tok_off % 64 || tok_off < 0 || ntok < R || ntok > mx_cols_kp(R) ||
        tok_off + ntok > ldqc || ((uintptr_t)x & 15) || ((uintptr_t)qr & 15) || ((uintptr_t)qc & 15) ||
        R >= (1LL << 30) || ldqc >= (1LL << 31)) {
        set_error("quantize_mx_rowcol: C %% 64, tok_off %% 64, R <= ntok <= R rounded to 64 and 16-B aligned rows "
                  "required (C=%d R=%lld tok_off=%lld ntok=%lld ldqc=%lld)", C, R, tok_off, ntok, ldqc);
        return false;
    }
    const long long rp = mx_rows_padded(R);
    const int cpad = (int)mx_rows_padded(C);
    // 128 columns from C = 2048 (ViT-H/14 micro-batch, tools/bench_quant.py: 3840 columns 64 -> 50 us,
    // 5120: 88 -> 78 us; 1280: 17.0 vs 17.5 us, kept at 64); VIT_ROWCOL_COLS=64|128 forces one
    static const int force = [] {
        const char* e = getenv("VIT_ROWCOL_COLS");
        return e ? atoi(e) : 0;
    }();
    const int cols = force == 64 || force == 128 ? force : (C >= 2048 ? 128 : 64);
    if (cols == 128 && C % 128 == 0)
        f8::quantize_mx_rowcol_k<128, 128><<<dim3((unsigned)(rp / 128), cpad / 128), 512, 0, s>>>(
            qr, slr, qc, slc, (const uint16_t*)x, (int)R, C, ldx, (int)(rp / 32), ldqc, (int)tok_off, (int)ntok, cpad / 32);
    else
        f8::quantize_mx_rowcol_k<128, 64><<<dim3((unsigned)(rp / 128), cpad / 64), 256, 0, s>>>(
            qr, slr, qc, slc, (const uint16_t*)x, (int)R, C, ldx, (int)(rp / 32), ldqc, (int)tok_off, (int)ntok, cpad / 32);
    after_launch("quantize_mx_rowcol");
    count_hit(VIT_HIT_QUANT_ROWCOL);
    return true;
}
// the leftover rows of the LayerNorm -> MX kernels (< 2 rounds of tiles on 2 workgroups per CU): their
// bf16 rows (forward), the follow-up quantize's discarded row form and its scales
static long long ln_mx_scratch_rows() { return 4LL * gemm_cu_count() * 32; }
size_t ln_mx_scratch_bytes(int C) {
    const long long r = ln_mx_scratch_rows();
    return (size_t)(2 * r * C + 256) + (size_t)(r * C + 256) + mx_scale_bytes(r, C) + 256;
}
bool ln_forward_mx_supported(int C) { return C % 256 == 0 && C >= 256 && C <= 2048 && C != 1792; }
bool ln_forward_mx(uint8_t* qr, uint8_t* slr, uint8_t* qc, uint8_t* slc, float* mean, float* rstd, const float* x,
                   const float* w, const float* b, long long R, int C, long long ldqc, long long tok_off, long long ntok,
                   hipStream_t s, uint8_t* scratch) {
    if (R <= 0) return true;
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (!ln_forward_mx_supported(C) || ldqc % 16 || tok_off % 64 || tok_off < 0 || ntok < R ||
        ntok > mx_cols_kp(R) || tok_off + ntok > ldqc || !al16(x) || !al16(w) || !al16(b) || !al16(qr) ||
        !al16(qc) || R >= (1LL << 30) || ldqc >= (1LL << 31)) {
        set_error("ln_forward_mx: C in 256 .. 2048 (multiple of 256), tok_off %% 64, R <= ntok <= R rounded to 64 "
                  "and 16-B aligned operands required (C=%d R=%lld tok_off=%lld ntok=%lld ldqc=%lld)",
                  C, R, tok_off, ntok, ldqc);
        return false;
    }
    const long long rp = mx_rows_padded(R);
    const int rgr = (int)(rp / 32), rgc = (int)(mx_rows_padded(C) / 32);
    // whole rounds of tiles only (two 80-KiB workgroups per CU at 4 rows per wave, one at 2): 16 448 rows
    // are 514 tiles for 512 slots, and the 2 of a second round would cost a whole tile time; the rows of
    // a last partial round go one per wave to extra workgroups (row form, bf16 row into the scratch) and
    // their column form comes from a follow-up quantize of those rows
    static const int rpw_env = [] {
        const char* e = getenv("VIT_LNMX_RPW");
        return e && atoi(e) == 2 ? 2 : 4;
    }();
    const int ntiles = (int)(rp / 32), slots = gemm_cu_count() * (rpw_env == 2 ? 1 : 2);
    int nmain = ntiles <= slots || !scratch ? ntiles : ntiles / slots * slots;
    if (nmain < ntiles && (long long)nmain * 32 >= R && ntok > (long long)nmain * 32) nmain -= slots;
    const long long r_left = (long long)nmain * 32;  // leftover rows: < 2 rounds of tiles <= ln_mx_scratch_rows()
    uint16_t* ybf = reinterpret_cast<uint16_t*>(scratch);
    const dim3 g((unsigned)(nmain + (ntiles - nmain) * 32 / (64 * 32 / rpw_env / 64)));
    static const int xmap = [] {
        const char* e = getenv("VIT_LNMX_XMAP");
        return e ? atoi(e) : 1;
    }();
    static const bool wb = [] {
        const char* e = getenv("VIT_LNMX_WB");
        return !(e && e[0] == '0');
    }();
    const int rpw = rpw_env;
    switch (C / 256) {
#define VIT_LAUNCH(NV, WB, RPW) \
    f8::ln_fwd_mx_k<NV, WB, RPW><<<g, 64 * 32 / RPW, 0, s>>>(qr, slr, qc, slc, mean, rstd, x, w, b, (int)R, rgr, ldqc, \
                                                             (int)tok_off, (int)ntok, rgc, xmap, nmain, ntiles, ybf)
#define VIT_CASE(NV) \
    case NV: \
        if (rpw == 2) { if (wb) VIT_LAUNCH(NV, true, 2); else VIT_LAUNCH(NV, false, 2); } \
        else { if (wb) VIT_LAUNCH(NV, true, 4); else VIT_LAUNCH(NV, false, 4); } \
        break;
        VIT_CASE(1) VIT_CASE(2) VIT_CASE(3) VIT_CASE(4) VIT_CASE(5) VIT_CASE(6) VIT_CASE(8)
#undef VIT_CASE
#undef VIT_LAUNCH
        default: break;
    }
    after_launch("ln_forward_mx");
    count_hit(VIT_HIT_LN_MX);
    if (r_left < R && r_left < ntok) {  // column form of the leftover rows (their row form again into the scratch)
        const long long rs = R - r_left;
        uint8_t* sq = scratch + ((2 * rs * C + 255) / 256 * 256);
        if (!quantize_mx_rowcol_bf16(sq, sq + ((rs * C + 255) / 256 * 256), qc, slc, reinterpret_cast<bf16_t*>(ybf), rs,
                                     C, C, ldqc, tok_off + r_left, ntok - r_left, s))
            return false;
    }
    return true;
}
bool ln_backward_mx_supported(int C) { return C % 256 == 0 && C >= 256 && C <= 1280; }
size_t ln_backward_mx_scratch_bytes(int C) { return ln_mx_scratch_bytes(C); }
bool ln_backward_bf16_stream_mx(bf16_t* dres_out, uint8_t* lo_out, const bf16_t* dres_in, const uint8_t* lo_in,
                                float* dw, float* db, float* dres_colsum, const bf16_t* dout, const float* inp,
                                const float* w, const float* mean, const float* rstd, long long R, int C,
                                hipStream_t s, float* part, uint8_t* qr, uint8_t* slr, uint8_t* qc, uint8_t* slc,
                                long long ldqc, long long tok_off, long long ntok, uint8_t* scratch) {
    if (R <= 0) return true;
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (!ln_backward_mx_supported(C) || !dres_out || !lo_out || !dres_in || !lo_in || ldqc % 16 || tok_off % 64 ||
        tok_off < 0 || ntok < R || ntok > mx_cols_kp(R) || tok_off + ntok > ldqc || !al16(dres_out) || !al16(dres_in) ||
        !al16(dout) || !al16(inp) || !al16(w) || !al16(qr) || !al16(qc) || (((uintptr_t)lo_in | (uintptr_t)lo_out) & 3) ||
        R >= (1LL << 30) || ldqc >= (1LL << 31)) {
        set_error("layernorm_backward_mx: C in 256 .. 1280 (multiple of 256), tok_off %% 64, R <= ntok <= R rounded "
                  "to 64, aligned planes required (C=%d R=%lld tok_off=%lld ntok=%lld ldqc=%lld)", C, R, tok_off, ntok, ldqc);
        return false;
    }
    const int nsum = dres_colsum ? 3 * C : 2 * C, nparts = ln_bwd_blocks(R);
    const bool reduce = part == nullptr;
    const size_t part_bytes = ((size_t)nparts * nsum * sizeof(float) + 255) / 256 * 256;
    if (reduce || !scratch) {  // the C-ABI path: partial rows and / or the scratch from the thread workspace
        char* ws = (char*)workspace(part_bytes + (scratch ? 0 : ln_backward_mx_scratch_bytes(C)));
        if (!ws) return false;
        if (reduce) part = (float*)ws;
        if (!scratch) scratch = (uint8_t*)(ws + part_bytes);
    }
    f8::LnbMx a;
    a.hi_out = dres_out; a.lo_out = lo_out; a.hi_in = dres_in; a.lo_in = lo_in;
    a.dout = dout; a.inp = inp; a.w = w; a.mean = mean; a.rstd = rstd;
    a.part = part; a.nsum = nsum; a.nparts = nparts;
    a.qr = qr; a.slr = slr; a.qc = qc; a.slc = slc;
    const long long rp = mx_rows_padded(R);
    a.R = (int)R; a.ntiles = (int)(rp / 32); a.rgr_tot = (int)(rp / 32);
    a.tok_off = (int)tok_off; a.ntok = (int)ntok; a.rgc_tot = (int)(mx_rows_padded(C) / 32); a.ldqc = ldqc;
    // one 8-wave workgroup per CU (160 KiB of LDS at C = 1280), persistent over the 32-token tiles.
    // Whole rounds of tiles only (nmain, a multiple of g): the tiles of a last partial round would
    // leave every other CU idle for a tile time (16 448 rows: 514 tiles on 256 CUs), so their rows are
    // spread one per wave over all workgroups and their column form comes from a follow-up quantize.
    const int g = std::min(std::min(a.ntiles, gemm_cu_count()), nparts);
    int nmain = a.ntiles / g * g;
    // the follow-up needs at least one real row (it writes the padding tokens' zero blocks only then)
    if (nmain < a.ntiles && (long long)nmain * 32 >= R && ntok > (long long)nmain * 32) nmain -= g;
    a.nmain = nmain;
    const long long r_left = (long long)nmain * 32;
    switch (C / 256) {
        case 1: f8::ln_bwd_mx_k<1><<<g, 512, 0, s>>>(a); break;
        case 2: f8::ln_bwd_mx_k<2><<<g, 512, 0, s>>>(a); break;
        case 3: f8::ln_bwd_mx_k<3><<<g, 512, 0, s>>>(a); break;
        case 4: f8::ln_bwd_mx_k<4><<<g, 512, 0, s>>>(a); break;
        default: f8::ln_bwd_mx_k<5><<<g, 512, 0, s>>>(a); break;
    }
    after_launch("layernorm_backward_mx");
    count_hit(VIT_HIT_LNB_MX);
    if (r_left < R && r_left < ntok) {  // column form of the leftover rows (row form into the scratch)
        if (R - r_left > ln_mx_scratch_rows()) {
            set_error("layernorm_backward_mx: %lld leftover rows exceed the scratch", R - r_left);
            return false;
        }
        const long long rs = R - r_left;
        if (!quantize_mx_rowcol_bf16(scratch, scratch + ((rs * C + 255) / 256 * 256), qc, slc, dres_out + r_left * C, rs,
                                     C, C, ldqc, tok_off + r_left, ntok - r_left, s))
            return false;
    }
    if (reduce) {
        const RowsJob jobs[3] = {{dw, part, nparts, nsum, C}, {db, part + C, nparts, nsum, C},
                                 {dres_colsum, part + 2 * C, nparts, nsum, C}};
        rows_reduce_add(jobs, dres_colsum ? 3 : 2, s);
    }
    return true;
}
void quantize_mx_batched_bf16(uint8_t* q, uint8_t* sl, const bf16_t* x, long long R, int K, int count,
                              long long xs, long long qs, long long ss, hipStream_t s) {
    quantize_mx<bf16_t>(q, sl, x, R, K, K, K, count, xs, qs, ss, s);
}
void quantize_mx_batched_f32(uint8_t* q, uint8_t* sl, const float* x, long long R, int K, int count,
                             long long xs, long long qs, long long ss, hipStream_t s) {
    quantize_mx<float>(q, sl, x, R, K, K, K, count, xs, qs, ss, s);
}

}  // namespace vit

// ============================================================================ C ABI (vit_ops.h)
using namespace vit;
extern "C" {
long long mx_scale_size(long long rows, int K) { return (long long)mx_scale_bytes(rows, K); }
void quantize_mx_bf16_ex(uint8_t* q, uint8_t* scales, const uint16_t* x, long long R, int K, long long ldx,
                         long long ldq) {
    quantize_mx_bf16(q, scales, x, R, K, ldx, ldq, stream());
}
void quantize_mx_f32_ex(uint8_t* q, uint8_t* scales, const float* x, long long R, int K, long long ldx,
                        long long ldq) {
    quantize_mx_f32(q, scales, x, R, K, ldx, ldq, stream());
}
long long mx_cols_padded(long long R) { return mx_cols_kp(R); }
void quantize_mx_cols_bf16_ex(uint8_t* q, uint8_t* scales, const uint16_t* x, long long R, int C, long long ldx) {
    quantize_mx_cols_bf16(q, scales, (const bf16_t*)x, R, C, ldx, stream());
}
void quantize_mx_rowcol_bf16_ex(uint8_t* qr, uint8_t* scales_r, uint8_t* qc, uint8_t* scales_c, const uint16_t* x,
                                long long R, int C, long long ldx, long long ldqc, long long tok_off, long long ntok) {
    quantize_mx_rowcol_bf16(qr, scales_r, qc, scales_c, (const bf16_t*)x, R, C, ldx, ldqc, tok_off, ntok, stream());
}
void layernorm_backward_stream(uint16_t* dres_out, uint8_t* lo_out, const uint16_t* dres_in, const uint8_t* lo_in,
                               float* dweight, float* dbias, float* dres_colsum, const uint16_t* dout, const float* inp,
                               const float* weight, const float* mean, const float* rstd, long long R, int C) {
    ln_backward_bf16_stream((bf16_t*)dres_out, lo_out, (const bf16_t*)dres_in, lo_in, dweight, dbias, dres_colsum,
                            (const bf16_t*)dout, inp, weight, mean, rstd, R, C, stream());
}
void layernorm_backward_stream_mx(uint16_t* dres_out, uint8_t* lo_out, const uint16_t* dres_in, const uint8_t* lo_in,
                                  float* dweight, float* dbias, float* dres_colsum, const uint16_t* dout,
                                  const float* inp, const float* weight, const float* mean, const float* rstd,
                                  long long R, int C, uint8_t* qr, uint8_t* scales_r, uint8_t* qc, uint8_t* scales_c,
                                  long long ldqc, long long tok_off, long long ntok) {
    ln_backward_bf16_stream_mx((bf16_t*)dres_out, lo_out, (const bf16_t*)dres_in, lo_in, dweight, dbias, dres_colsum,
                               (const bf16_t*)dout, inp, weight, mean, rstd, R, C, stream(), nullptr, qr, scales_r, qc,
                               scales_c, ldqc, tok_off, ntok, nullptr);
}
void layernorm_forward_mx(uint8_t* qr, uint8_t* scales_r, uint8_t* qc, uint8_t* scales_c, float* mean, float* rstd,
                          const float* inp, const float* weight, const float* bias, long long R, int C, long long ldqc,
                          long long tok_off, long long ntok) {
    ln_forward_mx(qr, scales_r, qc, scales_c, mean, rstd, inp, weight, bias, R, C, ldqc, tok_off, ntok, stream(),
                  (uint8_t*)workspace(ln_mx_scratch_bytes(C)));
}
void gemm_fp8_fused_mx(void* C, void* C2, long long ldc, const void* aux, long long ldaux, const uint8_t* A,
                       const uint8_t* a_scale, long long lda, const uint8_t* B, const uint8_t* b_scale,
                       long long ldb, const float* bias, float* colsum_out, int M, int N, int K, int epi,
                       uint8_t* mx_q, uint8_t* mx_s) {
    GemmArgs a;
    a.C = C; a.C2 = C2; a.ldc = ldc; a.aux = aux; a.ldaux = ldaux;
    a.A = A; a.a_scale = a_scale; a.lda = lda; a.B = B; a.b_scale = b_scale; a.ldb = ldb;
    a.bias = bias; a.colsum_out = colsum_out; a.M = M; a.N = N; a.K = K; a.epi = epi;
    a.mx_q = mx_q; a.mx_s = mx_s;
    if (mx_q && !epi_mx(epi)) {
        set_error("gemm_fp8_fused_mx: the MX output needs epi 4 / 8 (GELU pairs) or 6 / 9 (GELU', product)");
        return;
    }
    gemm_fp8(a, stream());
}
void gemm_fp8_fused_mxc(void* C, void* C2, long long ldc, const void* aux, long long ldaux, const uint8_t* A,
                        const uint8_t* a_scale, long long lda, const uint8_t* B, const uint8_t* b_scale,
                        long long ldb, const float* bias, float* colsum_out, int M, int N, int K, int epi,
                        uint8_t* mx_q, uint8_t* mx_s, uint8_t* mxc_q, uint8_t* mxc_s, long long mxc_ld,
                        long long mxc_off) {
    GemmArgs a;
    a.C = C; a.C2 = C2; a.ldc = ldc; a.aux = aux; a.ldaux = ldaux;
    a.A = A; a.a_scale = a_scale; a.lda = lda; a.B = B; a.b_scale = b_scale; a.ldb = ldb;
    a.bias = bias; a.colsum_out = colsum_out; a.M = M; a.N = N; a.K = K; a.epi = epi;
    a.mx_q = mx_q; a.mx_s = mx_s;
    a.mxc_q = mxc_q; a.mxc_s = mxc_s; a.mxc_ld = mxc_ld; a.mxc_off = mxc_off;
    gemm_fp8(a, stream());
}
void gemm_fp8_fused(void* C, void* C2, long long ldc, const void* aux, long long ldaux, const uint8_t* A,
                    const uint8_t* a_scale, long long lda, const uint8_t* B, const uint8_t* b_scale,
                    long long ldb, const float* bias, float* colsum_out, int M, int N, int K, int epi) {
    GemmArgs a;
    a.C = C; a.C2 = C2; a.ldc = ldc; a.aux = aux; a.ldaux = ldaux;
    a.A = A; a.a_scale = a_scale; a.lda = lda; a.B = B; a.b_scale = b_scale; a.ldb = ldb;
    a.bias = bias; a.colsum_out = colsum_out; a.M = M; a.N = N; a.K = K; a.epi = epi;
    gemm_fp8(a, stream());
}
}
