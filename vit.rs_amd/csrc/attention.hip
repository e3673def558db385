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
__device__ __forceinline__ f32x4_t mfma(bf16x8_t a, bf16x8_t b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void load_rows(bf16_t* img, int stride, const bf16_t* src, long long ld,
                                          int T, int Tp) {
    // rows of 64 bf16 = 8 x 16 B; rows >= T zero-filled
    for (int idx = threadIdx.x; idx < Tp * 8; idx += blockDim.x) {
        const int t = idx >> 3, c = idx & 7;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (t < T) v = *reinterpret_cast<const uint4*>(src + (long long)t * ld + c * 8);
        *reinterpret_cast<uint4*>(img + t * stride + c * 8) = v;
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
    __shared__ __attribute__((aligned(16))) bf16_t Ks[TMAX * SK];
    __shared__ __attribute__((aligned(16))) bf16_t Vs[TMAX * SV];
    constexpr int TP = NKT * 16;
    const int bh = blockIdx.x, b = bh / NH, h = bh % NH;
    const long long C3 = 3LL * C;
    const bf16_t* base = qkv + (long long)b * T * C3 + h * HS;
    load_rows(Ks, SK, base + C, C3, T, TP);
    load_rows(Vs, SV, base + 2 * C, C3, T, TP);
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
    const float c = LOG2E / sqrtf((float)HS);
    const int nqt = (T + 15) / 16;
    for (int qt = w; qt < nqt; qt += 4) {
        const int q = qt * 16 + i;
        bf16x8_t qf[2];
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
                const float p = exp2f(sacc[kt][r] - mx);
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
    load_rows(Qs, SK, base, C3, T, TP);
    load_rows(Ks, SK, base + C, C3, T, TP);
    load_rows(Vs, SK, base + 2 * C, C3, T, TP);
    load_rows(Ds, SK, dbase, C, T, TP);
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
        out[sct * C + h * HS + d] += a;
    }
}
}  // namespace fa

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
        set_error("attention_forward_fused: needs head size 64 and T<=256 (T=%d C=%d NH=%d)", T, C, NH);
        return;
    }
    const int nkt = cdiv(T, 32) * 2;
    dim3 grid(B * NH);
    VIT_NKT_DISPATCH(fa::attn_fwd_fused_k, out, lse, qkv, T, C, NH)
    after_launch("attention_forward_fused");
}

void attn_backward_fused(bf16_t* dqkv, const bf16_t* dout, const bf16_t* qkv, const bf16_t* out,
                         const float* lse, int B, int T, int C, int NH, hipStream_t s,
                         float* dqkv_colsum, float* part_ws) {
    if (!attn_fused_supported(T, C, NH)) {
        set_error("attention_backward_fused: needs head size 64 and T<=256 (T=%d C=%d NH=%d)", T, C, NH);
        return;
    }
    const int nkt = cdiv(T, 32) * 2;
    dim3 grid(B * NH);
#define VIT_BWD_THREADS 512
    if (dqkv_colsum && !part_ws) {
        set_error("attention_backward_fused: column sums need a [B*NH*192] workspace");
        return;
    }
    VIT_NKT_DISPATCH_T(fa::attn_bwd_fused_k, VIT_BWD_THREADS, dqkv, dout, qkv, out, lse, T, C, NH,
                       dqkv_colsum ? part_ws : nullptr)
    after_launch("attention_backward_fused");
    if (dqkv_colsum) {
        fa::attn_colsum_reduce_k<<<3 * NH, 1024, 0, s>>>(dqkv_colsum, part_ws, B, NH, C);
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
