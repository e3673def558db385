// attention.hip — attention_forward / attention_backward (train_vit.rs:400-451, 559-601;
// attention.rs:1-57), fixes D1 (offsets by T), D2 (full normalisation), D3 (non-causal).
//
// Drop-in fp32 kernels (reference signature): materialise preatt/att [B,T,NH,T] exactly like the
// reference; one wave per (b,t,h) row, scores in LDS.
//
// Fused bf16 kernels (trainer fast path, head size 64, T <= 256): one workgroup per (b,h) holds
// the head's K and V (and Q, dO for backward) in LDS; scores never touch HBM.
//   forward : per 16-query tile, S^T = K.Q^T with v_mfma_f32_16x16x32_bf16 so each lane owns one
//             query column (lane&15) -> row max/sum need only two cross-lane shuffles; the fp32
//             score accumulators convert in place into the B operand of O^T = V^T.P^T (the
//             shared k permutation of gemm.hip: k = 4g+j | 16+4g+j), V read with
//             ds_read_b64_tr_b16.  Writes O (bf16) and lse (log2 domain) per query.
//   backward: recomputes P from lse (no T x T storage).  Phase 1 (key tiles per wave):
//             S = Q.K^T and dP = dO.V^T with the key on the lane, dS = P*(dP - delta),
//             dV^T += dO^T.P and dK^T += Q^T.dS (accumulators used directly as B operands).
//             Phase 2 (query tiles per wave): S^T, dP^T with the query on the lane,
//             dQ^T += K^T.dS^T.  No atomics: dQ, dK, dV are each owned by one wave.
//             delta = rowsum(dO*O) is the O(T^2) form of the reference's O(T^3) softmax
//             Jacobian loop (train_vit.rs:583-589).
#include "ops_internal.h"

namespace vit {

// ======================================================================= fp32 drop-in kernels
__global__ __launch_bounds__(256) void attn_fwd_f32_k(float* __restrict__ out,
                                                      float* __restrict__ preatt,
                                                      float* __restrict__ att,
                                                      const float* __restrict__ inp, int B, int T,
                                                      int C, int NH) {
    extern __shared__ float sc[];  // [4][T]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long nrows = (long long)B * T * NH;
    const long long bth = blockIdx.x * 4LL + w;
    const bool valid = bth < nrows;
    const int hs = C / NH;
    const long long C3 = 3LL * C;
    const float scale = 1.0f / sqrtf((float)hs);
    float* s = sc + w * T;
    long long b = 0, t = 0, h = 0;
    if (valid) {
        b = bth / ((long long)T * NH);
        t = (bth / NH) % T;
        h = bth % NH;
        const float* q = inp + (b * T + t) * C3 + h * hs;
        float mx = -INFINITY;
        for (int t2 = lane; t2 < T; t2 += 64) {
            const float* k = inp + (b * T + t2) * C3 + h * hs + C;
            float v = 0.f;
            for (int i = 0; i < hs; i++) v += q[i] * k[i];
            v *= scale;
            s[t2] = v;
            preatt[bth * T + t2] = v;
            mx = fmaxf(mx, v);
        }
        mx = warp_max(mx);
        float sum = 0.f;
        for (int t2 = lane; t2 < T; t2 += 64) {
            const float e = expf(s[t2] - mx);
            s[t2] = e;
            sum += e;
        }
        const float inv = 1.0f / warp_sum(sum);
        for (int t2 = lane; t2 < T; t2 += 64) {
            const float a = s[t2] * inv;
            s[t2] = a;
            att[bth * T + t2] = a;
        }
    }
    __syncthreads();
    if (valid) {
        for (int d = lane; d < hs; d += 64) {
            float o = 0.f;
            for (int t2 = 0; t2 < T; t2++) o += s[t2] * inp[(b * T + t2) * C3 + h * hs + 2 * C + d];
            out[(b * T + t) * C + h * hs + d] = o;
        }
    }
}

// per query row: datt += V.dout (accumulated scratch), dpreatt += att*(datt - sum(att*datt)),
// dq += K^T dpreatt * scale
__global__ __launch_bounds__(256) void attn_bwd_q_f32_k(float* __restrict__ dinp,
                                                        float* __restrict__ dpreatt,
                                                        float* __restrict__ datt,
                                                        const float* __restrict__ dout,
                                                        const float* __restrict__ inp,
                                                        const float* __restrict__ att, int B,
                                                        int T, int C, int NH) {
    extern __shared__ float sc[];  // [4][T]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long nrows = (long long)B * T * NH;
    const long long bth = blockIdx.x * 4LL + w;
    const bool valid = bth < nrows;
    const int hs = C / NH;
    const long long C3 = 3LL * C;
    const float scale = 1.0f / sqrtf((float)hs);
    float* s = sc + w * T;
    long long b = 0, t = 0, h = 0;
    if (valid) {
        b = bth / ((long long)T * NH);
        t = (bth / NH) % T;
        h = bth % NH;
        const float* dy = dout + (b * T + t) * C + h * hs;
        const float* a = att + bth * T;
        float dsum = 0.f;
        for (int t2 = lane; t2 < T; t2 += 64) {
            const float* v = inp + (b * T + t2) * C3 + h * hs + 2 * C;
            float d = 0.f;
            for (int i = 0; i < hs; i++) d += v[i] * dy[i];
            const float dn = datt[bth * T + t2] + d;
            datt[bth * T + t2] = dn;
            s[t2] = dn;
            dsum += a[t2] * dn;
        }
        dsum = warp_sum(dsum);
        for (int t2 = lane; t2 < T; t2 += 64) {
            const float dp = dpreatt[bth * T + t2] + a[t2] * (s[t2] - dsum);
            dpreatt[bth * T + t2] = dp;
            s[t2] = dp;
        }
    }
    __syncthreads();
    if (valid) {
        float* dq = dinp + (b * T + t) * C3 + h * hs;
        for (int d = lane; d < hs; d += 64) {
            float acc = 0.f;
            for (int t2 = 0; t2 < T; t2++) acc += inp[(b * T + t2) * C3 + h * hs + C + d] * s[t2] * scale;
            dq[d] += acc;
        }
    }
}

// per key row (b,t2,h): dk += sum_t q[t]*dpreatt[t,t2]*scale ; dv += sum_t att[t,t2]*dout[t]
__global__ __launch_bounds__(256) void attn_bwd_kv_f32_k(float* __restrict__ dinp,
                                                         const float* __restrict__ dpreatt,
                                                         const float* __restrict__ dout,
                                                         const float* __restrict__ inp,
                                                         const float* __restrict__ att, int B,
                                                         int T, int C, int NH) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long nrows = (long long)B * T * NH;
    const long long r = blockIdx.x * 4LL + w;
    if (r >= nrows) return;
    const int hs = C / NH;
    const long long C3 = 3LL * C;
    const float scale = 1.0f / sqrtf((float)hs);
    const long long b = r / ((long long)T * NH), t2 = (r / NH) % T, h = r % NH;
    float* dk = dinp + (b * T + t2) * C3 + h * hs + C;
    float* dv = dinp + (b * T + t2) * C3 + h * hs + 2 * C;
    for (int d = lane; d < hs; d += 64) {
        float ak = 0.f, av = 0.f;
        for (int t = 0; t < T; t++) {
            const long long row = ((b * T + t) * NH + h) * T + t2;
            ak += inp[(b * T + t) * C3 + h * hs + d] * dpreatt[row] * scale;
            av += att[row] * dout[(b * T + t) * C + h * hs + d];
        }
        dk[d] += ak;
        dv[d] += av;
    }
}

void attn_forward_f32(float* out, float* preatt, float* att, const float* inp, int B, int T, int C,
                      int NH, hipStream_t s) {
    const long long rows = (long long)B * T * NH;
    if (rows <= 0) return;
    if (T > 4096) { set_error("attention_forward: T=%d > 4096", T); return; }
    attn_fwd_f32_k<<<cdiv(rows, 4), 256, 4 * T * sizeof(float), s>>>(out, preatt, att, inp, B, T, C, NH);
    after_launch("attention_forward");
}

void attn_backward_f32(float* dinp, float* dpreatt, float* datt, const float* dout,
                       const float* inp, const float* att, int B, int T, int C, int NH,
                       hipStream_t s) {
    const long long rows = (long long)B * T * NH;
    if (rows <= 0) return;
    if (T > 4096) { set_error("attention_backward: T=%d > 4096", T); return; }
    if (!dpreatt || !datt) {
        const size_t n = (size_t)rows * T;
        float* ws = (float*)workspace(2 * n * sizeof(float));
        if (!ws) return;
        VIT_HIP(hipMemsetAsync(ws, 0, 2 * n * sizeof(float), s));
        if (!dpreatt) dpreatt = ws;
        if (!datt) datt = ws + n;
    }
    attn_bwd_q_f32_k<<<cdiv(rows, 4), 256, 4 * T * sizeof(float), s>>>(dinp, dpreatt, datt, dout,
                                                                        inp, att, B, T, C, NH);
    after_launch("attention_backward(q)");
    attn_bwd_kv_f32_k<<<cdiv(rows, 4), 256, 0, s>>>(dinp, dpreatt, dout, inp, att, B, T, C, NH);
    after_launch("attention_backward(kv)");
}

// ======================================================================= fused bf16 kernels
namespace fa {
constexpr int HS = 64;
constexpr int TMAX = 256;
constexpr int SK = 72;  // row-read image stride (144 B)
constexpr int SV = 80;  // tr-read-only image stride (160 B): 8 consecutive rows hit 8 slots
constexpr float LOG2E = 1.4426950408889634f;
constexpr int NWB = 8;   // waves per backward workgroup (one workgroup per (b,h), LDS-bound to 1/CU)

// rows r0+i, k over the head dim with the shared permutation (d = 32s+4g+j | 32s+16+4g+j-4)
__device__ __forceinline__ bf16x8_t frag_row(const bf16_t* img, int stride, int r0, int s, int lane) {
    const int i = lane & 15, g = lane >> 4;
    const bf16_t* p = img + (r0 + i) * stride + 32 * s + 4 * g;
    const bf16x4_t lo = *reinterpret_cast<const bf16x4_t*>(p);
    const bf16x4_t hi = *reinterpret_cast<const bf16x4_t*>(p + 16);
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
__device__ __forceinline__ f32x4_t mfma(bf16x8_t a, bf16x8_t b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// rows of 64 bf16 (8 x 16 B each, rows >= T zero-filled) of NOP operands into their LDS images.
// Every global load of the thread is issued before its first LDS store, so the whole staging is
// one memory round trip (a load -> store loop serialised one round trip per 16-B chunk row).
template <int TP, int NTHR, int NOP>
__device__ __forceinline__ void load_images(bf16_t* const (&img)[NOP], const int (&stride)[NOP],
                                            const bf16_t* const (&src)[NOP],
                                            const long long (&ld)[NOP], int T) {
    constexpr int PER = (TP * 8 + NTHR - 1) / NTHR;
    uint4 v[NOP][PER];
#pragma unroll
    for (int o = 0; o < NOP; o++)
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int idx = j * NTHR + (int)threadIdx.x, t = idx >> 3, c = idx & 7;
            v[o][j] = make_uint4(0, 0, 0, 0);
            if (idx < TP * 8 && t < T) v[o][j] = *reinterpret_cast<const uint4*>(src[o] + (long long)t * ld[o] + c * 8);
        }
#pragma unroll
    for (int o = 0; o < NOP; o++)
#pragma unroll
        for (int j = 0; j < PER; j++) {
            const int idx = j * NTHR + (int)threadIdx.x, t = idx >> 3, c = idx & 7;
            if (idx < TP * 8) *reinterpret_cast<uint4*>(img[o] + t * stride[o] + c * 8) = v[o][j];
        }
}
__device__ __forceinline__ void store4(bf16_t* dst, f32x4_t v, float mul) {
    *reinterpret_cast<uint2*>(dst) =
        make_uint2(pack_bf16x2(v[0] * mul, v[1] * mul), pack_bf16x2(v[2] * mul, v[3] * mul));
}

template <int NKT>  // key tiles of 16 covering Tpad = 16*NKT (multiple of 32)
__global__ __launch_bounds__(256) void attn_fwd_fused_k(bf16_t* __restrict__ out,
                                                        float* __restrict__ lse,
                                                        const bf16_t* __restrict__ qkv, int T,
                                                        int C, int NH) {
    constexpr int TP = NKT * 16;
    __shared__ __attribute__((aligned(16))) bf16_t Ks[TP * SK];
    __shared__ __attribute__((aligned(16))) bf16_t Vs[TP * SV];
    const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
    const long long C3 = 3LL * C;
    const bf16_t* base = qkv + (long long)b * T * C3 + h * HS;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
    // Q fragments of a 16-query tile straight from HBM (rows >= T -> 0); the next tile's are
    // requested while the current one computes, the first ones before the K/V staging
    auto load_q = [&](int qt, bf16x8_t (&qf)[2]) {
        const int q = qt * 16 + i;
#pragma unroll
        for (int s = 0; s < 2; s++) {
            bf16x4_t lo = {}, hi = {};
            if (q < T) {
                const bf16_t* p = base + (long long)q * C3 + 32 * s + 4 * g;
                lo = *reinterpret_cast<const bf16x4_t*>(p);
                hi = *reinterpret_cast<const bf16x4_t*>(p + 16);
            }
            qf[s] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
    };
    const int nqt = (T + 15) / 16;
    bf16x8_t qn[2];
    load_q(w, qn);
    {
        bf16_t* const img[2] = {Ks, Vs};
        const int st[2] = {SK, SV};
        const bf16_t* const src[2] = {base + C, base + 2 * C};
        const long long ld[2] = {C3, C3};
        load_images<TP, 256, 2>(img, st, src, ld, T);
    }
    __syncthreads();
    const float c = LOG2E / sqrtf((float)HS);
    for (int qt = w; qt < nqt; qt += 4) {
        const int q = qt * 16 + i;
        const bf16x8_t qf[2] = {qn[0], qn[1]};
        if (qt + 4 < nqt) load_q(qt + 4, qn);
        f32x4_t sacc[NKT];
#pragma unroll
        for (int kt = 0; kt < NKT; kt++) {
            f32x4_t a = {0.f, 0.f, 0.f, 0.f};
            a = mfma(frag_row(Ks, SK, kt * 16, 0, lane), qf[0], a);
            a = mfma(frag_row(Ks, SK, kt * 16, 1, lane), qf[1], a);
            sacc[kt] = a;
        }
        // lane (i,g) holds S^T[key = 16kt+4g+r][q]
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < NKT; kt++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int key = kt * 16 + 4 * g + r;
                const float x = key < T ? sacc[kt][r] * c : -INFINITY;
                sacc[kt][r] = x;
                mx = fmaxf(mx, x);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        float l = 0.f;
#pragma unroll
        for (int kt = 0; kt < NKT; kt++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const float p = fexp2(sacc[kt][r] - mx);
                sacc[kt][r] = p;
                l += p;
            }
        l += __shfl_xor(l, 16, 64);
        l += __shfl_xor(l, 32, 64);
        f32x4_t o[4];
#pragma unroll
        for (int dt = 0; dt < 4; dt++) o[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKT / 2; ks++) {
            const bf16x8_t pb = pack_acc(sacc[2 * ks], sacc[2 * ks + 1]);
#pragma unroll
            for (int dt = 0; dt < 4; dt++) o[dt] = mfma(frag_tr(Vs, SV, 32 * ks, 16 * dt, lane), pb, o[dt]);
        }
        if (q < T) {
            const float inv = 1.0f / l;
            bf16_t* dst = out + ((long long)b * T + q) * C + h * HS + 4 * g;
#pragma unroll
            for (int dt = 0; dt < 4; dt++) store4(dst + 16 * dt, o[dt], inv);
            if (g == 0) lse[(long long)bh * T + q] = mx + log2f(l);
        }
    }
}

template <int NKT>
__global__ __launch_bounds__(512) void attn_bwd_fused_k(bf16_t* __restrict__ dqkv,
                                                        const bf16_t* __restrict__ dout,
                                                        const bf16_t* __restrict__ qkv,
                                                        const bf16_t* __restrict__ out,
                                                        const float* __restrict__ lse, int T,
                                                        int C, int NH, float* __restrict__ dsum) {
    __shared__ __attribute__((aligned(16))) bf16_t Qs[TMAX * SK];
    __shared__ __attribute__((aligned(16))) bf16_t Ks[TMAX * SK];
    __shared__ __attribute__((aligned(16))) bf16_t Vs[TMAX * SK];
    __shared__ __attribute__((aligned(16))) bf16_t Ds[TMAX * SK];
    __shared__ float lse_s[TMAX];
    __shared__ float del_s[TMAX];
    __shared__ float csum_s[NWB * 3 * HS];  // fused bias gradient: per-wave column sums dQ|dK|dV
    constexpr int TP = NKT * 16;
    const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
    const long long C3 = 3LL * C;
    const bf16_t* base = qkv + (long long)b * T * C3 + h * HS;
    const bf16_t* dbase = dout + (long long)b * T * C + h * HS;
    for (int t = threadIdx.x; t < NWB * 3 * HS; t += blockDim.x) csum_s[t] = 0.f;
    const bf16_t* obase = out + (long long)b * T * C + h * HS;
    {
        bf16_t* const img[4] = {Qs, Ks, Vs, Ds};
        const int st[4] = {SK, SK, SK, SK};
        const bf16_t* const src[4] = {base, base + C, base + 2 * C, dbase};
        const long long ld[4] = {C3, C3, C3, C};
        load_images<TP, 512, 4>(img, st, src, ld, T);
    }
    for (int t = threadIdx.x; t < TP; t += blockDim.x) {
        float dl = 0.f, ls = INFINITY;
        if (t < T) {
            ls = lse[(long long)bh * T + t];
            const bf16_t* orow = obase + (long long)t * C;
            const bf16_t* drow = dbase + (long long)t * C;
#pragma unroll
            for (int cch = 0; cch < 8; cch++) {
                const uint4 ov = *reinterpret_cast<const uint4*>(orow + cch * 8);
                const uint4 dv = *reinterpret_cast<const uint4*>(drow + cch * 8);
                const uint32_t* o32 = reinterpret_cast<const uint32_t*>(&ov);
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
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
    const float scale = 1.0f / sqrtf((float)HS);
    const float c = LOG2E * scale;
    const int nt_valid = (T + 15) / 16;

    // ---- phase 1: dK, dV for key tiles owned by this wave
    f32x4_t ck[4] = {}, cv[4] = {};  // this lane's share of the dK / dV column sums
    for (int kt = w; kt < nt_valid; kt += NWB) {
        const int key0 = kt * 16;
        const bool key_ok = key0 + i < T;
        const bf16x8_t kf0 = frag_row(Ks, SK, key0, 0, lane), kf1 = frag_row(Ks, SK, key0, 1, lane);
        const bf16x8_t vf0 = frag_row(Vs, SK, key0, 0, lane), vf1 = frag_row(Vs, SK, key0, 1, lane);
        f32x4_t dv[4], dk[4];
#pragma unroll
        for (int dt = 0; dt < 4; dt++) dv[dt] = dk[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int qs = 0; qs < TP / 32; qs++) {
            f32x4_t P[2], dS[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int qt0 = (2 * qs + u) * 16;
                f32x4_t s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
                s = mfma(frag_row(Qs, SK, qt0, 0, lane), kf0, s);
                s = mfma(frag_row(Qs, SK, qt0, 1, lane), kf1, s);
                dp = mfma(frag_row(Ds, SK, qt0, 0, lane), vf0, dp);
                dp = mfma(frag_row(Ds, SK, qt0, 1, lane), vf1, dp);
                // lane (i,g): [q = qt0+4g+r][key = key0+i]
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int qq = qt0 + 4 * g + r;
                    const float p = key_ok ? exp2f(s[r] * c - lse_s[qq]) : 0.f;
                    P[u][r] = p;
                    dS[u][r] = p * (dp[r] - del_s[qq]);
                }
            }
            const bf16x8_t pb = pack_acc(P[0], P[1]);
            const bf16x8_t db = pack_acc(dS[0], dS[1]);
#pragma unroll
            for (int dt = 0; dt < 4; dt++) {
                dv[dt] = mfma(frag_tr(Ds, SK, 32 * qs, 16 * dt, lane), pb, dv[dt]);
                dk[dt] = mfma(frag_tr(Qs, SK, 32 * qs, 16 * dt, lane), db, dk[dt]);
            }
        }
        if (key_ok) {
            bf16_t* dst = dqkv + ((long long)b * T + key0 + i) * C3 + h * HS + 4 * g;
#pragma unroll
            for (int dt = 0; dt < 4; dt++) {
                store4(dst + C + 16 * dt, dk[dt], scale);
                store4(dst + 2 * C + 16 * dt, dv[dt], 1.0f);
            }
        }
        if (dsum) {  // rows past T hold exact zeros (P = 0 there)
#pragma unroll
            for (int dt = 0; dt < 4; dt++) {
                ck[dt] += dk[dt] * scale;
                cv[dt] += dv[dt];
            }
        }
    }
    if (dsum) {  // reduce over the 16 key lanes once, one LDS row per wave
#pragma unroll
        for (int dt = 0; dt < 4; dt++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float tk = ck[dt][r], tv = cv[dt][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    tk += __shfl_xor(tk, o, 64);
                    tv += __shfl_xor(tv, o, 64);
                }
                if (i == 0) {
                    csum_s[(w * 3 + 1) * HS + 16 * dt + 4 * g + r] = tk;
                    csum_s[(w * 3 + 2) * HS + 16 * dt + 4 * g + r] = tv;
                }
            }
    }

    // ---- phase 2: dQ for query tiles owned by this wave
    f32x4_t cq[4] = {};
    for (int qt = w; qt < nt_valid; qt += NWB) {
        const int q0 = qt * 16;
        const bf16x8_t qf0 = frag_row(Qs, SK, q0, 0, lane), qf1 = frag_row(Qs, SK, q0, 1, lane);
        const bf16x8_t df0 = frag_row(Ds, SK, q0, 0, lane), df1 = frag_row(Ds, SK, q0, 1, lane);
        const float ls = lse_s[q0 + i], dl = del_s[q0 + i];
        f32x4_t dq[4];
#pragma unroll
        for (int dt = 0; dt < 4; dt++) dq[dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int ks = 0; ks < TP / 32; ks++) {
            f32x4_t dS[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int kt0 = (2 * ks + u) * 16;
                f32x4_t s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
                s = mfma(frag_row(Ks, SK, kt0, 0, lane), qf0, s);
                s = mfma(frag_row(Ks, SK, kt0, 1, lane), qf1, s);
                dp = mfma(frag_row(Vs, SK, kt0, 0, lane), df0, dp);
                dp = mfma(frag_row(Vs, SK, kt0, 1, lane), df1, dp);
                // lane (i,g): [key = kt0+4g+r][q = q0+i]
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int key = kt0 + 4 * g + r;
                    const float p = key < T ? exp2f(s[r] * c - ls) : 0.f;
                    dS[u][r] = p * (dp[r] - dl);
                }
            }
            const bf16x8_t db = pack_acc(dS[0], dS[1]);
#pragma unroll
            for (int dt = 0; dt < 4; dt++) dq[dt] = mfma(frag_tr(Ks, SK, 32 * ks, 16 * dt, lane), db, dq[dt]);
        }
        if (q0 + i < T) {
            bf16_t* dst = dqkv + ((long long)b * T + q0 + i) * C3 + h * HS + 4 * g;
#pragma unroll
            for (int dt = 0; dt < 4; dt++) store4(dst + 16 * dt, dq[dt], scale);
        }
        if (dsum) {
#pragma unroll
            for (int dt = 0; dt < 4; dt++) cq[dt] += dq[dt] * scale;
        }
    }
    if (dsum) {
#pragma unroll
        for (int dt = 0; dt < 4; dt++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float tq = cq[dt][r];
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) tq += __shfl_xor(tq, o, 64);
                if (i == 0) csum_s[(w * 3 + 0) * HS + 16 * dt + 4 * g + r] = tq;
            }
    }
    if (dsum) {  // per-(b,h) partial column sums -> dsum[bh][3*64] (reduced over b by a second kernel)
        __syncthreads();
        for (int t = threadIdx.x; t < 3 * HS; t += blockDim.x) {
            float acc = 0.f;
#pragma unroll
            for (int ww = 0; ww < NWB; ww++) acc += csum_s[ww * 3 * HS + t];
            dsum[(long long)bh * 3 * HS + t] = acc;
        }
    }
}

// ----------------------------------------------------------------------------------------------
// Backward as two roles of one launch with 32-row register tiles (attn_bwd_pair_k: bwd_kv_body
// and bwd_q_body), a 256-thread workgroup per (b,h) and role, two workgroups per CU (LDS ~66 KB).  The single-kernel
// form above holds Q, K, V and dO in 147 KB of LDS (one workgroup per CU) and reads four LDS
// fragments per two MFMAs; here each fragment read from LDS feeds two 16-row MFMA tiles:
//   kv: wave owns 32 keys (K, V fragments in registers, dK^T / dV^T accumulators); per 32-query
//       chunk: S, dP (8 + 8 MFMA, Q / dO rows from LDS), P = exp2(S c - lse), dS = P (dP - delta),
//       dV^T += dO^T P, dK^T += Q^T dS (8 + 8 MFMA, transposed reads).  delta = rowsum(dO * O)
//       (the O(T^2) form of train_vit.rs:583-589) is computed by each role for the rows it needs.
//   q:  wave owns 32 queries (Q, dO fragments in registers, dQ^T accumulators); per 32-key chunk:
//       S^T, dP^T (8 + 8, K / V rows from LDS), dQ^T += K^T dS^T (8).
// Rows >= T are zero-filled, so padded keys contribute nothing to dQ; padded queries have
// lse = +inf (P = 0).  P of padded keys is zeroed for the fused bias column sums.
template <int NKT>
constexpr int bwd_lds_bytes() { return 2 * NKT * 16 * SK * 2 + 2 * NKT * 16 * 4 + 4 * 2 * HS * 4; }

template <int NKT>
__device__ __forceinline__ void bwd_kv_body(char* lds, int bh, bf16_t* __restrict__ dqkv,
                                            const bf16_t* __restrict__ dout,
                                            const bf16_t* __restrict__ qkv,
                                            const bf16_t* __restrict__ out,
                                            const float* __restrict__ lse, int T, int C, int NH,
                                            float* __restrict__ dsum) {
    constexpr int TP = NKT * 16;  // padded length, multiple of 32
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
    auto load_kv = [&](int kt, bf16x8_t (&kf)[2][2], bf16x8_t (&vf)[2][2]) {
#pragma unroll
        for (int kk = 0; kk < 2; kk++) {
            const int key = kt * 32 + kk * 16 + i;
#pragma unroll
            for (int s = 0; s < 2; s++) {
                bf16x4_t klo = {}, khi = {}, vlo = {}, vhi = {};
                if (key < T) {
                    const bf16_t* pk = base + (long long)key * C3 + C + 32 * s + 4 * g;
                    klo = *reinterpret_cast<const bf16x4_t*>(pk);
                    khi = *reinterpret_cast<const bf16x4_t*>(pk + 16);
                    vlo = *reinterpret_cast<const bf16x4_t*>(pk + C);
                    vhi = *reinterpret_cast<const bf16x4_t*>(pk + C + 16);
                }
                kf[kk][s] = __builtin_shufflevector(klo, khi, 0, 1, 2, 3, 4, 5, 6, 7);
                vf[kk][s] = __builtin_shufflevector(vlo, vhi, 0, 1, 2, 3, 4, 5, 6, 7);
            }
        }
    };
    bf16x8_t kf[2][2], vf[2][2];
    if (w < TP / 32) load_kv(w, kf, vf);
    {
        bf16_t* const img[2] = {Qs, Ds};
        const int st[2] = {SK, SK};
        const bf16_t* const src[2] = {base, dbase};
        const long long ld[2] = {C3, C};
        load_images<TP, 256, 2>(img, st, src, ld, T);
    }
    __syncthreads();
    // delta = rowsum(dO * O) per query (O from HBM, dO from the image), lse staged
    for (int t = tid; t < TP; t += 256) {
        float dl = 0.f, ls = INFINITY;
        if (t < T) {
            ls = lse[(long long)bh * T + t];
            uint4 ov[8];
#pragma unroll
            for (int c = 0; c < 8; c++) ov[c] = *reinterpret_cast<const uint4*>(obase + (long long)t * C + c * 8);
#pragma unroll
            for (int c = 0; c < 8; c++) {
                const uint4 dv = *reinterpret_cast<const uint4*>(Ds + t * SK + c * 8);
                const uint32_t* o32 = reinterpret_cast<const uint32_t*>(&ov[c]);
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
    f32x4_t ck[4] = {}, cv[4] = {};  // this lane's share of the dK / dV column sums
    for (int kt = w; kt < TP / 32; kt += 4) {
        const int key0 = kt * 32;
        if (kt != w) load_kv(kt, kf, vf);
        const bool kok[2] = {key0 + i < T, key0 + 16 + i < T};
        f32x4_t dv[2][4], dk[2][4];
#pragma unroll
        for (int kk = 0; kk < 2; kk++)
#pragma unroll
            for (int dt = 0; dt < 4; dt++) dv[kk][dt] = dk[kk][dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int qs = 0; qs < TP / 32; qs++) {
            f32x4_t P[2][2], dS[2][2];  // [kk][u]: lane (i,g) -> [q = 32qs+16u+4g+r][key = 16kk+i]
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int qt0 = qs * 32 + u * 16;
                const bf16x8_t q0 = frag_row(Qs, SK, qt0, 0, lane), q1 = frag_row(Qs, SK, qt0, 1, lane);
                const bf16x8_t d0 = frag_row(Ds, SK, qt0, 0, lane), d1 = frag_row(Ds, SK, qt0, 1, lane);
                float lq[4], dq[4];
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    lq[r] = lse_s[qt0 + 4 * g + r];
                    dq[r] = del_s[qt0 + 4 * g + r];
                }
#pragma unroll
                for (int kk = 0; kk < 2; kk++) {
                    f32x4_t s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
                    s = mfma(q0, kf[kk][0], s);
                    s = mfma(q1, kf[kk][1], s);
                    dp = mfma(d0, vf[kk][0], dp);
                    dp = mfma(d1, vf[kk][1], dp);
                    // padded keys (K, V rows zero) get P != 0 here; they only reach dK / dV rows
                    // that are neither stored nor summed
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const float pv = fexp2(s[r] * c - lq[r]);
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
            for (int dt = 0; dt < 4; dt++) {
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
            for (int dt = 0; dt < 4; dt++) {
                store4(dst + C + 16 * dt, dk[kk][dt], scale);
                store4(dst + 2 * C + 16 * dt, dv[kk][dt], 1.0f);
            }
        }
        if (dsum) {
#pragma unroll
            for (int kk = 0; kk < 2; kk++) {
                if (!kok[kk]) continue;
#pragma unroll
                for (int dt = 0; dt < 4; dt++) {
                    ck[dt] += dk[kk][dt] * scale;
                    cv[dt] += dv[kk][dt];
                }
            }
        }
    }
    if (dsum) {  // per-(b,h) column sums of dK, dV -> dsum[bh][64..191]
#pragma unroll
        for (int dt = 0; dt < 4; dt++)
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

template <int NKT>
__device__ __forceinline__ void bwd_q_body(char* lds, int bh, bf16_t* __restrict__ dqkv,
                                           const bf16_t* __restrict__ dout,
                                           const bf16_t* __restrict__ qkv,
                                           const bf16_t* __restrict__ out,
                                           const float* __restrict__ lse, int T, int C, int NH,
                                           float* __restrict__ dsum) {
    constexpr int TP = NKT * 16;
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
    auto load_tile = [&](int qt, bf16x8_t (&qf)[2][2], bf16x8_t (&df)[2][2], float (&lq)[2], float (&dl)[2]) {
        const int q0 = qt * 32;
        float part[2] = {0.f, 0.f};
#pragma unroll
        for (int qq = 0; qq < 2; qq++) {
            const int q = q0 + qq * 16 + i;
#pragma unroll
            for (int s = 0; s < 2; s++) {
                bf16x4_t a0 = {}, a1 = {}, b0 = {}, b1 = {}, o0 = {}, o1 = {};
                if (q < T) {
                    const bf16_t* pq = base + (long long)q * C3 + 32 * s + 4 * g;
                    const bf16_t* pd = dbase + (long long)q * C + 32 * s + 4 * g;
                    const bf16_t* po = obase + (long long)q * C + 32 * s + 4 * g;
                    a0 = *reinterpret_cast<const bf16x4_t*>(pq);
                    a1 = *reinterpret_cast<const bf16x4_t*>(pq + 16);
                    b0 = *reinterpret_cast<const bf16x4_t*>(pd);
                    b1 = *reinterpret_cast<const bf16x4_t*>(pd + 16);
                    o0 = *reinterpret_cast<const bf16x4_t*>(po);
                    o1 = *reinterpret_cast<const bf16x4_t*>(po + 16);
                }
                qf[qq][s] = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
                df[qq][s] = __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7);
                // delta = rowsum(dO * O): this lane's 16 of the query's 64 columns
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    part[qq] += (float)b0[e] * (float)o0[e];
                    part[qq] += (float)b1[e] * (float)o1[e];
                }
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
    bf16x8_t qn[2][2], dn[2][2];
    float lqn[2], dln[2];
    if (w < TP / 32) load_tile(w, qn, dn, lqn, dln);
    {
        bf16_t* const img[2] = {Ks, Vs};
        const int st[2] = {SK, SK};
        const bf16_t* const src[2] = {base + C, base + 2 * C};
        const long long ld[2] = {C3, C3};
        load_images<TP, 256, 2>(img, st, src, ld, T);
    }
    __syncthreads();
    const float scale = 1.0f / sqrtf((float)HS);
    const float c = LOG2E * scale;
    f32x4_t cq[4] = {};
    for (int qt = w; qt < TP / 32; qt += 4) {
        const int q0 = qt * 32;
        bf16x8_t qf[2][2], df[2][2];
        float lq[2], dl[2];
#pragma unroll
        for (int qq = 0; qq < 2; qq++) {
            lq[qq] = lqn[qq];
            dl[qq] = dln[qq];
#pragma unroll
            for (int s = 0; s < 2; s++) {
                qf[qq][s] = qn[qq][s];
                df[qq][s] = dn[qq][s];
            }
        }
        if (qt + 4 < TP / 32) load_tile(qt + 4, qn, dn, lqn, dln);
        f32x4_t dq[2][4];
#pragma unroll
        for (int qq = 0; qq < 2; qq++)
#pragma unroll
            for (int dt = 0; dt < 4; dt++) dq[qq][dt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int ks = 0; ks < TP / 32; ks++) {
            f32x4_t dS[2][2];  // [qq][u]: lane (i,g) -> [key = 32ks+16u+4g+r][q = 16qq+i]
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int kt0 = ks * 32 + u * 16;
                const bf16x8_t k0 = frag_row(Ks, SK, kt0, 0, lane), k1 = frag_row(Ks, SK, kt0, 1, lane);
                const bf16x8_t v0 = frag_row(Vs, SK, kt0, 0, lane), v1 = frag_row(Vs, SK, kt0, 1, lane);
#pragma unroll
                for (int qq = 0; qq < 2; qq++) {
                    f32x4_t s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
                    s = mfma(k0, qf[qq][0], s);
                    s = mfma(k1, qf[qq][1], s);
                    dp = mfma(v0, df[qq][0], dp);
                    dp = mfma(v1, df[qq][1], dp);
#pragma unroll
                    for (int r = 0; r < 4; r++) dS[qq][u][r] = fexp2(s[r] * c - lq[qq]) * (dp[r] - dl[qq]);
                }
            }
            bf16x8_t db[2];
#pragma unroll
            for (int qq = 0; qq < 2; qq++) db[qq] = pack_acc(dS[qq][0], dS[qq][1]);
#pragma unroll
            for (int dt = 0; dt < 4; dt++) {
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
            for (int dt = 0; dt < 4; dt++) store4(dst + 16 * dt, dq[qq][dt], scale);
        }
        if (dsum) {  // padded queries: dS = exp2(-inf) * ... = 0
#pragma unroll
            for (int qq = 0; qq < 2; qq++)
#pragma unroll
                for (int dt = 0; dt < 4; dt++) cq[dt] += dq[qq][dt] * scale;
        }
    }
    if (dsum) {
#pragma unroll
        for (int dt = 0; dt < 4; dt++)
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
template <int NKT>
__global__ __launch_bounds__(256, 2) void attn_bwd_pair_k(bf16_t* __restrict__ dqkv,
                                                          const bf16_t* __restrict__ dout,
                                                          const bf16_t* __restrict__ qkv,
                                                          const bf16_t* __restrict__ out,
                                                          const float* __restrict__ lse, int T,
                                                          int C, int NH, int BH,
                                                          float* __restrict__ dsum) {
    __shared__ __attribute__((aligned(16))) char lds[bwd_lds_bytes<NKT>()];
    const int x = blockIdx.x & 7, grp = blockIdx.x >> 3;
    const int role = grp & 1, bh = (grp >> 1) * 8 + x;
    if (bh >= BH) return;
    if (role == 0) bwd_kv_body<NKT>(lds, bh, dqkv, dout, qkv, out, lse, T, C, NH, dsum);
    else bwd_q_body<NKT>(lds, bh, dqkv, dout, qkv, out, lse, T, C, NH, dsum);
}

// out[s*C + h*64 + d] += sum_b part[(b*NH + h)][s*64 + d]; one 1024-thread block per (s, h):
// 16 batch lanes x 64 columns, fixed-order tree over the lanes (deterministic).
__global__ __launch_bounds__(1024) void attn_colsum_reduce_k(float* __restrict__ out,
                                                             const float* __restrict__ part, int B,
                                                             int NH, int C) {
    __shared__ float red[16][HS];
    const int sh = blockIdx.x;  // 0 .. 3*NH-1
    const int sct = sh / NH, h = sh - sct * NH;
    const int d = threadIdx.x & (HS - 1), lane_b = threadIdx.x >> 6;
    float t = 0.f;
#pragma unroll 4
    for (int b = lane_b; b < B; b += 16) t += part[((long long)b * NH + h) * 3 * HS + sct * HS + d];
    red[lane_b][d] = t;
    __syncthreads();
    if (lane_b == 0) {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < 16; i++) a += red[i][d];
        atomicAdd(out + sct * C + h * HS + d, a);  // micro-batches reduce into one bias concurrently
    }
}
}  // namespace fa


// ======================================================================= generic bf16 kernels
// Shapes outside the fused kernels' tiling (head size != 64 or T > 256, e.g. ViT-H/14: hs = 80,
// T = 257): the same math and the same outputs (O bf16, lse in the log2 domain, dqkv overwritten)
// on the VALU.  One workgroup per ((b,h), row chunk) stages the head's two streamed operands in
// LDS as bf16 (row stride hs+2 elements = an odd number of words, so lane-per-row reads are
// conflict-free); each wave owns one row at a time, lanes over keys for the scores and over
// head dims (d = lane, lane+64) for the products.  Correctness path, not the tuned one.
namespace gen {
// waves per workgroup: 16 for the forward up to hs 80 (123 VGPRs -> 4 waves/SIMD), 8 for the
// backward kernels (~210 VGPRs -> 2 waves/SIMD); one workgroup per CU (the staged operands take
// ~90 KiB of LDS at hs 80, T 257), so these wave counts are the latency hiding there is
__host__ __device__ constexpr int nw_fwd(int hs) { return hs <= 80 ? 16 : 8; }
__host__ __device__ constexpr int nw_bwd(int hs) { return hs <= 96 ? 8 : 4; }
constexpr int CHUNKS = 4;   // row chunks per (b,h)
using fa::LOG2E;

// LDS row stride (elements): HS + 8 = an odd number of 16-B units, so lane-per-row b128 reads
// are conflict-free
__host__ __device__ constexpr int stride(int hs) { return hs + 8; }
__host__ inline size_t lds_bytes(int T, int hs, int nw) {
    return (size_t)2 * T * stride(hs) * 2 + (size_t)nw * 2 * T * 4 + (size_t)2 * T * 4;
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// x[0..HS) (registers) . row[0..HS) (bf16, LDS or global), 8 elements per 16-B read
// orders one wave's LDS writes before its other lanes read them (no workgroup barrier: the row
// loops below have wave-dependent trip counts)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int HS>
__device__ __forceinline__ float dot_row(const bf16_t* row, const float (&x)[HS]) {
    float a = 0.f;
#pragma unroll
    for (int j = 0; j < HS / 8; j++) {
        const u32x4_t w = *reinterpret_cast<const u32x4_t*>(row + 8 * j);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            a += __uint_as_float(w[e] << 16) * x[8 * j + 2 * e];
            a += __uint_as_float(w[e] & 0xffff0000u) * x[8 * j + 2 * e + 1];
        }
    }
    return a;
}

template <int HS>
__device__ __forceinline__ void load_row(float (&x)[HS], const bf16_t* row, float scale) {
#pragma unroll
    for (int j = 0; j < HS / 8; j++) {
        const u32x4_t w = *reinterpret_cast<const u32x4_t*>(row + 8 * j);
#pragma unroll
        for (int e = 0; e < 4; e++) {
            x[8 * j + 2 * e] = __uint_as_float(w[e] << 16) * scale;
            x[8 * j + 2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u) * scale;
        }
    }
}

// stage rows [0,T) of two [T][HS] bf16 operands (row strides ld0/ld1) into LDS, 16 B per copy
template <int HS>
__device__ __forceinline__ void stage2(bf16_t* X0, bf16_t* X1, const bf16_t* b0, long long ld0,
                                       const bf16_t* b1, long long ld1, int T) {
    constexpr int st = stride(HS), pr = HS / 8;
    for (int e = threadIdx.x; e < T * pr; e += blockDim.x) {
        const int t = e / pr, i = e - t * pr;
        *reinterpret_cast<u32x4_t*>(X0 + t * st + 8 * i) = *reinterpret_cast<const u32x4_t*>(b0 + t * ld0 + 8 * i);
        *reinterpret_cast<u32x4_t*>(X1 + t * st + 8 * i) = *reinterpret_cast<const u32x4_t*>(b1 + t * ld1 + 8 * i);
    }
}

// lanes own four head dims (4p .. 4p+3) and a residue class of rows (g = lane / (HS/4)); the
// partial sums of the NG classes are combined with lane permutes.  out(d) = sum_t w[t] * X[t][d]
template <int HS>
struct Pairs {
    static constexpr int NQ = HS / 4;
    static constexpr int NG = 64 / NQ;  // row classes (3 at hs 80: lanes 60..63 idle)
    int p, g;
    bool on;
    __device__ Pairs(int lane) : p(lane % NQ), g(lane / NQ), on(lane < NQ * NG) {}
    __device__ __forceinline__ static void fma4(f32x4_t& a, float wt, uint2 v) {
        a[0] += wt * __uint_as_float(v.x << 16);
        a[1] += wt * __uint_as_float(v.x & 0xffff0000u);
        a[2] += wt * __uint_as_float(v.y << 16);
        a[3] += wt * __uint_as_float(v.y & 0xffff0000u);
    }
    // two rows per iteration into separate accumulators (independent LDS loads and FMA chains)
    __device__ __forceinline__ void acc(f32x4_t& a, const float* w, const bf16_t* X, int T) const {
        if (!on) return;
        constexpr int st = stride(HS);
        f32x4_t b = {0.f, 0.f, 0.f, 0.f};
        int t = g;
        for (; t + NG < T; t += 2 * NG) {
            const uint2 v0 = *reinterpret_cast<const uint2*>(X + t * st + 4 * p);
            const uint2 v1 = *reinterpret_cast<const uint2*>(X + (t + NG) * st + 4 * p);
            const float w0 = w[t], w1 = w[t + NG];
            fma4(a, w0, v0);
            fma4(b, w1, v1);
        }
        if (t < T) fma4(a, w[t], *reinterpret_cast<const uint2*>(X + t * st + 4 * p));
        a += b;
    }
    // a += sum_t wa[t] Xa[t], b += sum_t wb[t] Xb[t] in one pass (the key side's dK and dV)
    __device__ __forceinline__ void acc2(f32x4_t& a, const float* wa, const bf16_t* Xa, f32x4_t& b,
                                         const float* wb, const bf16_t* Xb, int T) const {
        if (!on) return;
        constexpr int st = stride(HS);
        for (int t = g; t < T; t += NG) {
            const uint2 va = *reinterpret_cast<const uint2*>(Xa + t * st + 4 * p);
            const uint2 vb = *reinterpret_cast<const uint2*>(Xb + t * st + 4 * p);
            fma4(a, wa[t], va);
            fma4(b, wb[t], vb);
        }
    }
    // after reduce, lanes with g == 0 hold the full sums
    __device__ __forceinline__ void reduce(f32x4_t& a, int lane) const {
        f32x4_t r = a;
#pragma unroll
        for (int k = 1; k < NG; k++) {
            const int src = (lane + k * NQ) & 63;
#pragma unroll
            for (int e = 0; e < 4; e++) r[e] += __shfl(a[e], src, 64);
        }
        a = r;
    }
    __device__ __forceinline__ bool writer() const { return on && g == 0; }
    __device__ __forceinline__ void store(bf16_t* dst, const f32x4_t& a, float scale) const {
        uint2 o;
        o.x = pack_bf16x2(a[0] * scale, a[1] * scale);
        o.y = pack_bf16x2(a[2] * scale, a[3] * scale);
        *reinterpret_cast<uint2*>(dst + 4 * p) = o;
    }
};

template <int HS, int NW = nw_fwd(HS)>
__global__ __launch_bounds__(NW * 64) void fwd_k(bf16_t* __restrict__ out, float* __restrict__ lse,
                                                  const bf16_t* __restrict__ qkv, int T, int C, int NH) {
    extern __shared__ char lds[];
    constexpr int st = stride(HS);
    const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long C3 = 3LL * C;
    bf16_t* Ks = reinterpret_cast<bf16_t*>(lds);
    bf16_t* Vs = Ks + T * st;
    float* ps = reinterpret_cast<float*>(Vs + T * st) + w * 2 * T;
    const bf16_t* base = qkv + (long long)b * T * C3 + h * HS;
    stage2<HS>(Ks, Vs, base + C, C3, base + 2 * C, C3, T);
    __syncthreads();
    const Pairs<HS> pr(lane);
    const float c = LOG2E / sqrtf((float)HS);
    for (int r0 = blockIdx.y * NW; r0 < T; r0 += CHUNKS * NW) {
        const int t = r0 + w;
        if (t >= T) break;  // no barriers below: the rest of the loop is wave-local
        float q[HS];
        load_row<HS>(q, base + (long long)t * C3, c);
        float mx = -INFINITY;
        for (int t2 = lane; t2 < T; t2 += 64) {
            const float sc = dot_row<HS>(Ks + t2 * st, q);
            ps[t2] = sc;
            mx = fmaxf(mx, sc);
        }
        mx = warp_max(mx);
        float sum = 0.f;
        for (int t2 = lane; t2 < T; t2 += 64) {
            const float p = exp2f(ps[t2] - mx);
            ps[t2] = p;
            sum += p;
        }
        sum = warp_sum(sum);
        wave_lds_sync();
        f32x4_t o = {0.f, 0.f, 0.f, 0.f};
        pr.acc(o, ps, Vs, T);
        pr.reduce(o, lane);
        if (pr.writer()) pr.store(out + ((long long)b * T + t) * C + h * HS, o, 1.f / sum);
        if (lane == 0) lse[(long long)bh * T + t] = mx + log2f(sum);
        wave_lds_sync();  // ps is rewritten by the next row
    }
}

// query side: delta = rowsum(dO*O) -> ws, dS row, dQ = scale * dS.K  (K, V staged)
template <int HS, int NW = nw_bwd(HS)>
__global__ __launch_bounds__(NW * 64) void bwd_q_k(bf16_t* __restrict__ dqkv, float* __restrict__ delta,
                                                    const bf16_t* __restrict__ dout,
                                                    const bf16_t* __restrict__ qkv,
                                                    const bf16_t* __restrict__ out,
                                                    const float* __restrict__ lse, int T, int C, int NH) {
    extern __shared__ char lds[];
    constexpr int st = stride(HS);
    const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long C3 = 3LL * C;
    bf16_t* Ks = reinterpret_cast<bf16_t*>(lds);
    bf16_t* Vs = Ks + T * st;
    float* ds = reinterpret_cast<float*>(Vs + T * st) + w * 2 * T;
    const bf16_t* base = qkv + (long long)b * T * C3 + h * HS;
    stage2<HS>(Ks, Vs, base + C, C3, base + 2 * C, C3, T);
    __syncthreads();
    const Pairs<HS> pr(lane);
    const float scale = 1.f / sqrtf((float)HS), c = LOG2E * scale;
    for (int r0 = blockIdx.y * NW; r0 < T; r0 += CHUNKS * NW) {
        const int t = r0 + w;
        if (t >= T) break;
        const long long row = (long long)b * T + t;
        float q[HS], g[HS];
        load_row<HS>(q, base + (long long)t * C3, c);
        load_row<HS>(g, dout + row * C + h * HS, 1.f);
        float dl = 0.f;
        for (int d = lane; d < HS; d += 64) dl += bf2f(dout[row * C + h * HS + d]) * bf2f(out[row * C + h * HS + d]);
        dl = warp_sum(dl);
        const float ls = lse[(long long)bh * T + t];
        for (int t2 = lane; t2 < T; t2 += 64) {
            const float p = exp2f(dot_row<HS>(Ks + t2 * st, q) - ls);
            const float dp = dot_row<HS>(Vs + t2 * st, g);
            ds[t2] = p * (dp - dl) * scale;
        }
        if (lane == 0) delta[(long long)bh * T + t] = dl;
        wave_lds_sync();
        f32x4_t a = {0.f, 0.f, 0.f, 0.f};
        pr.acc(a, ds, Ks, T);
        pr.reduce(a, lane);
        if (pr.writer()) pr.store(dqkv + row * C3 + h * HS, a, 1.f);
        wave_lds_sync();
    }
}

// key side: per key row t2, P and dS columns over all queries, dK = scale * dS^T.Q, dV = P^T.dO
// (Q, dO staged; lse and delta of the head in LDS)
template <int HS, int NW = nw_bwd(HS)>
__global__ __launch_bounds__(NW * 64) void bwd_kv_k(bf16_t* __restrict__ dqkv, const float* __restrict__ delta,
                                                     const bf16_t* __restrict__ dout,
                                                     const bf16_t* __restrict__ qkv,
                                                     const float* __restrict__ lse, int T, int C, int NH) {
    extern __shared__ char lds[];
    constexpr int st = stride(HS);
    const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long C3 = 3LL * C;
    bf16_t* Qs = reinterpret_cast<bf16_t*>(lds);
    bf16_t* Gs = Qs + T * st;
    float* ps = reinterpret_cast<float*>(Gs + T * st) + w * 2 * T;
    float* ds = ps + T;
    float* ls_s = reinterpret_cast<float*>(Gs + T * st) + NW * 2 * T;
    float* dl_s = ls_s + T;
    const bf16_t* base = qkv + (long long)b * T * C3 + h * HS;
    stage2<HS>(Qs, Gs, base, C3, dout + (long long)b * T * C + h * HS, C, T);
    for (int t = threadIdx.x; t < T; t += blockDim.x) {
        ls_s[t] = lse[(long long)bh * T + t];
        dl_s[t] = delta[(long long)bh * T + t];
    }
    __syncthreads();
    const Pairs<HS> pr(lane);
    const float scale = 1.f / sqrtf((float)HS), c = LOG2E * scale;
    for (int r0 = blockIdx.y * NW; r0 < T; r0 += CHUNKS * NW) {
        const int t2 = r0 + w;
        if (t2 >= T) break;
        const long long row = (long long)b * T + t2;
        float k[HS], v[HS];
        load_row<HS>(k, base + (long long)t2 * C3 + C, c);
        load_row<HS>(v, base + (long long)t2 * C3 + 2 * C, 1.f);
        for (int t = lane; t < T; t += 64) {
            const float p = exp2f(dot_row<HS>(Qs + t * st, k) - ls_s[t]);
            const float dp = dot_row<HS>(Gs + t * st, v);
            ps[t] = p;
            ds[t] = p * (dp - dl_s[t]) * scale;
        }
        wave_lds_sync();
        f32x4_t ka = {0.f, 0.f, 0.f, 0.f}, va = {0.f, 0.f, 0.f, 0.f};
        pr.acc2(ka, ds, Qs, va, ps, Gs, T);
        pr.reduce(ka, lane);
        pr.reduce(va, lane);
        if (pr.writer()) {
            pr.store(dqkv + row * C3 + C + h * HS, ka, 1.f);
            pr.store(dqkv + row * C3 + 2 * C + h * HS, va, 1.f);
        }
        wave_lds_sync();
    }
}
}  // namespace gen

bool attn_generic_supported(int T, int C, int NH) {
    if (NH <= 0 || C % NH || T < 1) return false;
    const int hs = C / NH;
    const bool inst = hs == 32 || hs == 64 || hs == 80 || hs == 96 || hs == 128;  // template instances
    return inst && C % 8 == 0 && gen::lds_bytes(T, hs, gen::nw_fwd(hs)) <= 160 * 1024 &&
           gen::lds_bytes(T, hs, gen::nw_bwd(hs)) <= 160 * 1024;
}

static bool gen_lds_attr(const void* k, size_t bytes) {
    return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) == hipSuccess;
}

bool attn_fused_supported(int T, int C, int NH) {
    return NH > 0 && C % NH == 0 && C / NH == fa::HS && T >= 1 && T <= fa::TMAX && C % 8 == 0;
}

#define VIT_NKT_DISPATCH(KERNEL, ...)                                                   \
    switch (nkt) {                                                                      \
        case 2: KERNEL<2><<<grid, 256, 0, s>>>(__VA_ARGS__); break;                     \
        case 4: KERNEL<4><<<grid, 256, 0, s>>>(__VA_ARGS__); break;                     \
        case 6: KERNEL<6><<<grid, 256, 0, s>>>(__VA_ARGS__); break;                     \
        case 8: KERNEL<8><<<grid, 256, 0, s>>>(__VA_ARGS__); break;                     \
        case 10: KERNEL<10><<<grid, 256, 0, s>>>(__VA_ARGS__); break;                   \
        case 12: KERNEL<12><<<grid, 256, 0, s>>>(__VA_ARGS__); break;                   \
        case 14: KERNEL<14><<<grid, 256, 0, s>>>(__VA_ARGS__); break;                   \
        case 16: KERNEL<16><<<grid, 256, 0, s>>>(__VA_ARGS__); break;                   \
        default: set_error("fused attention: unsupported key tile count %d", nkt); return; \
    }

#define VIT_NKT_DISPATCH_T(KERNEL, NTHR, ...)                                          \
    switch (nkt) {                                                                      \
        case 2: KERNEL<2><<<grid, NTHR, 0, s>>>(__VA_ARGS__); break;                    \
        case 4: KERNEL<4><<<grid, NTHR, 0, s>>>(__VA_ARGS__); break;                    \
        case 6: KERNEL<6><<<grid, NTHR, 0, s>>>(__VA_ARGS__); break;                    \
        case 8: KERNEL<8><<<grid, NTHR, 0, s>>>(__VA_ARGS__); break;                    \
        case 10: KERNEL<10><<<grid, NTHR, 0, s>>>(__VA_ARGS__); break;                  \
        case 12: KERNEL<12><<<grid, NTHR, 0, s>>>(__VA_ARGS__); break;                  \
        case 14: KERNEL<14><<<grid, NTHR, 0, s>>>(__VA_ARGS__); break;                  \
        case 16: KERNEL<16><<<grid, NTHR, 0, s>>>(__VA_ARGS__); break;                  \
        default: set_error("fused attention: unsupported key tile count %d", nkt); return; \
    }

void attn_forward_fused(bf16_t* out, float* lse, const bf16_t* qkv, int B, int T, int C, int NH,
                        hipStream_t s) {
    if (!attn_fused_supported(T, C, NH)) {
        if (!attn_generic_supported(T, C, NH)) {
            set_error("attention_forward_fused: unsupported shape (T=%d C=%d NH=%d)", T, C, NH);
            return;
        }
        const size_t lds = gen::lds_bytes(T, C / NH, gen::nw_fwd(C / NH));
        switch (C / NH) {
#define VIT_GEN_FWD(HS)                                                                              \
    case HS:                                                                                         \
        if (!gen_lds_attr((const void*)gen::fwd_k<HS>, lds)) { set_error("attention: LDS attribute"); return; } \
        gen::fwd_k<HS><<<dim3(B * NH, gen::CHUNKS), gen::nw_fwd(HS) * 64, lds, s>>>(out, lse, qkv, T, C, NH); \
        break;
            VIT_GEN_FWD(32) VIT_GEN_FWD(64) VIT_GEN_FWD(80) VIT_GEN_FWD(96) VIT_GEN_FWD(128)
#undef VIT_GEN_FWD
            default: set_error("attention: no generic kernel for head size %d", C / NH); return;
        }
        after_launch("attention_forward_generic");
        return;
    }
    const int nkt = cdiv(T, 32) * 2;
    dim3 grid(B * NH);
    VIT_NKT_DISPATCH(fa::attn_fwd_fused_k, out, lse, qkv, T, C, NH)
    after_launch("attention_forward_fused");
}

void attn_backward_fused(bf16_t* dqkv, const bf16_t* dout, const bf16_t* qkv, const bf16_t* out,
                         const float* lse, int B, int T, int C, int NH, hipStream_t s,
                         float* dqkv_colsum, float* ws) {
    if (!attn_fused_supported(T, C, NH)) {
        if (!attn_generic_supported(T, C, NH)) {
            set_error("attention_backward_fused: unsupported shape (T=%d C=%d NH=%d)", T, C, NH);
            return;
        }
        // ws: [B*NH*T] delta = rowsum(dO*O)
        const size_t need = (size_t)B * NH * T * sizeof(float);
        if (!ws) ws = (float*)workspace(need);
        if (!ws) return;
        const size_t lds = gen::lds_bytes(T, C / NH, gen::nw_bwd(C / NH));
        const dim3 g(B * NH, gen::CHUNKS);
        switch (C / NH) {
#define VIT_GEN_BWD(HS)                                                                            \
    case HS:                                                                                       \
        if (!gen_lds_attr((const void*)gen::bwd_q_k<HS>, lds) ||                                   \
            !gen_lds_attr((const void*)gen::bwd_kv_k<HS>, lds)) {                                  \
            set_error("attention: LDS attribute");                                                 \
            return;                                                                                \
        }                                                                                          \
        gen::bwd_q_k<HS><<<g, gen::nw_bwd(HS) * 64, lds, s>>>(dqkv, ws, dout, qkv, out, lse, T, C, NH);    \
        gen::bwd_kv_k<HS><<<g, gen::nw_bwd(HS) * 64, lds, s>>>(dqkv, ws, dout, qkv, lse, T, C, NH);        \
        break;
            VIT_GEN_BWD(32) VIT_GEN_BWD(64) VIT_GEN_BWD(80) VIT_GEN_BWD(96) VIT_GEN_BWD(128)
#undef VIT_GEN_BWD
            default: set_error("attention: no generic kernel for head size %d", C / NH); return;
        }
        after_launch("attention_backward_generic");
        if (dqkv_colsum) colsum_bf16(dqkv_colsum, dqkv, B * T, 3 * C, 3LL * C, s);
        return;
    }
    const int nkt = cdiv(T, 32) * 2;
    dim3 grid(B * NH);
    static const int one_kernel = getenv("VIT_ATTN_BWD") ? atoi(getenv("VIT_ATTN_BWD")) : 0;
    // ws: [B*NH*192] per-(b,h) bias partial sums
    const size_t need = (size_t)B * NH * 3 * fa::HS * sizeof(float);
    if (!ws) ws = (float*)workspace(need);
    if (!ws) return;
    float* part = dqkv_colsum ? ws : nullptr;
    if (one_kernel == 1) {
        VIT_NKT_DISPATCH_T(fa::attn_bwd_fused_k, 512, dqkv, dout, qkv, out, lse, T, C, NH, part)
    } else {
        grid = dim3(2 * cdiv(B * NH, 8) * 8);
        VIT_NKT_DISPATCH_T(fa::attn_bwd_pair_k, 256, dqkv, dout, qkv, out, lse, T, C, NH, B * NH, part)
    }
    after_launch("attention_backward_fused");
    if (dqkv_colsum) {
        fa::attn_colsum_reduce_k<<<3 * NH, 1024, 0, s>>>(dqkv_colsum, part, B, NH, C);
        after_launch("attention_colsum_reduce");
    }
}

}  // namespace vit

using namespace vit;
extern "C" {
void attention_forward(float* out, float* preatt, float* att, const float* inp, int B, int T, int C,
                       int NH) {
    if (!preatt || !att) {
        set_error("attention_forward: preatt/att are required in drop-in mode");
        return;
    }
    attn_forward_f32(out, preatt, att, inp, B, T, C, NH, stream());
}
void attention_backward(float* dinp, float* dpreatt, float* datt, const float* dout,
                        const float* inp, const float* att, int B, int T, int C, int NH) {
    attn_backward_f32(dinp, dpreatt, datt, dout, inp, att, B, T, C, NH, stream());
}
void attention_forward_fused_bf16(uint16_t* out, float* lse, const uint16_t* inp, int B, int T,
                                  int C, int NH) {
    attn_forward_fused(out, lse, inp, B, T, C, NH, stream());
}
void attention_backward_fused_bf16(uint16_t* dinp, const uint16_t* dout, const uint16_t* inp,
                                   const uint16_t* out, const float* lse, int B, int T, int C,
                                   int NH) {
    attn_backward_fused(dinp, dout, inp, out, lse, B, T, C, NH, stream());
}
}
