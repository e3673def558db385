// attention.hip — attention_forward / attention_backward (train_vit.rs:400-451, 559-601;
// attention.rs:1-57), fixes D1 (offsets by T), D2 (full normalisation), D3 (non-causal).
//
// Drop-in fp32 kernels (reference signature): materialise preatt/att [B,T,NH,T] exactly like the
// reference (either may be NULL in fused use: the scores are then not stored); one wave per
// (b,t,h) row, scores in LDS.
//
// bf16 trainer path: the fused MFMA kernels of attn_fused.h (head sizes 32/64/80/96/128, T up to
// what LDS holds — 320 at every supported head size), instantiated per head size in attn_h*.hip,
// dispatched here.  Longer sequences fall back to the generic VALU kernels below (same outputs).
#include <string>

#include "attn_fused.h"

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
            if (preatt) preatt[bth * T + t2] = v;
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
            if (att) att[bth * T + t2] = a;
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



// ======================================================================= generic bf16 kernels
// Shapes outside the fused kernels' LDS range (T > 320 at the supported head sizes): the same math and the same outputs (O bf16, lse in the log2 domain, dqkv overwritten)
// on the VALU.  One workgroup per ((b,h), row chunk) stages the head's two streamed operands in
// LDS as bf16 (row stride hs+8 elements = an odd number of 16-B units, so lane-per-row b128 reads
// are conflict-free); each wave owns one row at a time, lanes over keys for the scores and over
// head dims (d = lane, lane+64) for the products.  Correctness path, not the tuned one.
namespace gen {
// waves per workgroup: 16 for the forward up to hs 80 (123 VGPRs -> 4 waves/SIMD), 8 for the
// backward kernels (~210 VGPRs -> 2 waves/SIMD); one workgroup per CU (the staged operands take
// ~90 KiB of LDS at hs 80, T 257), so these wave counts are the latency hiding there is
__host__ __device__ constexpr int nw_fwd(int hs) { return hs <= 80 ? 16 : 8; }
__host__ __device__ constexpr int nw_bwd(int hs) { return hs <= 96 ? 8 : 4; }
constexpr int CHUNKS = 4;   // row chunks per (b,h)
constexpr float LOG2E = 1.4426950408889634f;

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

int fa::attn_bwd_variant() {  // read per launch (host-side, cheap) so tests can A/B in one process
    const char* e = getenv("VIT_ATTN_BWD");
    if (!e) return 0;
    const std::string v(e);
    return v == "one" ? 1 : v == "pair" ? 2 : v == "p4" ? 4 : 0;
}
int fa::attn_cu_count() {
    static int n = [] {
        int dev = 0, cu = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
        return cu > 0 ? cu : 256;
    }();
    return n;
}

// head sizes with MFMA instantiations (attn_h*.hip) and the longest T their LDS images hold
static int fa_max_t(int hs) {
    switch (hs) {
        case 32: return fa_max_t_h32();
        case 64: return fa_max_t_h64();
        case 80: return fa_max_t_h80();
        case 96: return fa_max_t_h96();
        case 128: return fa_max_t_h128();
        default: return 0;
    }
}

bool attn_fused_supported(int T, int C, int NH) {
    return NH > 0 && C % NH == 0 && T >= 1 && T <= fa_max_t(C / NH) && C % 8 == 0 && !getenv("VIT_ATTN_GENERIC");
}

// Column sums of the fused backward's per-(row, h) partials, deterministic two-stage:
//   part_k : block (s*NH + h, chunk) sums its chunk of the R = B x rows partial rows
//            part[(r*NH + h)][s*HS + d] -> scratch[chunk][s*C + h*HS + d]
//   final_k: out[j] (+)= sum over chunks of scratch[chunk][j] (fixed order; the trainer stores one
//            row per micro-batch and reduces the rows after the layer)
// stage 1 of the deterministic qkv-bias column sums: workgroup (section*head, chunk) sums its
// chunk of the R partial rows for the head's HS columns.  16-B loads: HS/4 lanes cover a row
// segment, 256/(HS/4) rows are in flight per iteration, four independent accumulators per lane.
__global__ __launch_bounds__(256) void attn_colsum_part_k(float* __restrict__ scratch, const float* __restrict__ part,
                                                          int R, int NH, int C, int HS) {
    __shared__ float4 red[256];
    const int sh = blockIdx.x, sct = sh / NH, h = sh - sct * NH, ch = blockIdx.y, nch = gridDim.y;
    const int lpr = HS / 4, nb = 256 / lpr, d4 = threadIdx.x % lpr, lb = threadIdx.x / lpr;
    const int r0 = (int)((long long)R * ch / nch), r1 = (int)((long long)R * (ch + 1) / nch);
    float4 t[4] = {};
    const long long rs = (long long)NH * 3 * HS;  // floats between consecutive partial rows
    const float* base = part + (long long)h * 3 * HS + sct * HS + 4 * d4;
    int r = lb < nb ? r0 + lb : r1;  // lanes past nb * lpr (HS = 80, 96) take no rows
    for (; r + 3 * nb < r1; r += 4 * nb)
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const float4 v = *reinterpret_cast<const float4*>(base + (long long)(r + u * nb) * rs);
            t[u].x += v.x; t[u].y += v.y; t[u].z += v.z; t[u].w += v.w;
        }
    for (; r < r1; r += nb) {
        const float4 v = *reinterpret_cast<const float4*>(base + (long long)r * rs);
        t[0].x += v.x; t[0].y += v.y; t[0].z += v.z; t[0].w += v.w;
    }
    red[threadIdx.x] = make_float4(t[0].x + t[1].x + t[2].x + t[3].x, t[0].y + t[1].y + t[2].y + t[3].y,
                                   t[0].z + t[1].z + t[2].z + t[3].z, t[0].w + t[1].w + t[2].w + t[3].w);
    __syncthreads();
    if (lb == 0) {
        float4 a = red[d4];
        for (int j = 1; j < nb; j++) {
            const float4 b = red[j * lpr + d4];
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
        *reinterpret_cast<float4*>(scratch + (long long)ch * 3 * C + sct * C + h * HS + 4 * d4) = a;
    }
}
__global__ __launch_bounds__(256) void attn_colsum_final_k(float* __restrict__ out, const float* __restrict__ scratch,
                                                           int nch, int C3, int store) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= C3) return;
    float a = 0.f;
    for (int ch = 0; ch < nch; ch++) a += scratch[(long long)ch * C3 + j];
    out[j] = store ? a : out[j] + a;
}

size_t attn_backward_ws_floats(int B, int T, int C, int NH) {
    // partial rows (up to ATTN_PART_ROWS per (b,h)) + the colsum chunk sums (<= B rows of 3C)
    // (generic kernels: B*NH*T delta floats + the bias column sums' per-256-row partial rows)
    const size_t per_bh = std::max((size_t)T, (size_t)3 * (C / NH) * (fa::ATTN_PART_ROWS + 1));
    return (size_t)B * NH * per_bh + (size_t)cdiv((long long)B * T, 256) * 3 * C;
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
        count_hit(VIT_HIT_ATTN_GENERIC);
        return;
    }
    bool ok = false;
    switch (C / NH) {
        case 32: ok = fa_forward_h32(out, lse, qkv, B, T, C, NH, s); break;
        case 64: ok = fa_forward_h64(out, lse, qkv, B, T, C, NH, s); break;
        case 80: ok = fa_forward_h80(out, lse, qkv, B, T, C, NH, s); break;
        case 96: ok = fa_forward_h96(out, lse, qkv, B, T, C, NH, s); break;
        case 128: ok = fa_forward_h128(out, lse, qkv, B, T, C, NH, s); break;
    }
    if (!ok) { set_error("fused attention: no kernel for T=%d head size %d", T, C / NH); return; }
    after_launch("attention_forward_fused");
}

void attn_backward_fused(bf16_t* dqkv, const bf16_t* dout, const bf16_t* qkv, const bf16_t* out,
                         const float* lse, int B, int T, int C, int NH, hipStream_t s,
                         float* dqkv_colsum, float* ws, bool colsum_store) {
    if (!attn_fused_supported(T, C, NH)) {
        if (!attn_generic_supported(T, C, NH)) {
            set_error("attention_backward_fused: unsupported shape (T=%d C=%d NH=%d)", T, C, NH);
            return;
        }
        // ws: [B*NH*T] delta = rowsum(dO*O)
        if (!ws) ws = (float*)workspace(attn_backward_ws_floats(B, T, C, NH) * sizeof(float));
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
        count_hit(VIT_HIT_ATTN_GENERIC);
        if (dqkv_colsum) {
            if (colsum_store) VIT_HIP(hipMemsetAsync(dqkv_colsum, 0, 3 * (size_t)C * sizeof(float), s));
            colsum_bf16(dqkv_colsum, dqkv, B * T, 3 * C, 3LL * C, s, ws + (size_t)B * NH * T);
        }
        return;
    }
    const int HS = C / NH;
    // ws: per-(b,h) bias partial sums, up to ATTN_PART_ROWS rows of 3*HS each
    if (!ws) ws = (float*)workspace(attn_backward_ws_floats(B, T, C, NH) * sizeof(float));
    if (!ws) return;
    float* part = dqkv_colsum ? ws : nullptr;
    int rows = 0;
    switch (HS) {
        case 32: rows = fa_backward_h32(dqkv, dout, qkv, out, lse, B, T, C, NH, part, s); break;
        case 64: rows = fa_backward_h64(dqkv, dout, qkv, out, lse, B, T, C, NH, part, s); break;
        case 80: rows = fa_backward_h80(dqkv, dout, qkv, out, lse, B, T, C, NH, part, s); break;
        case 96: rows = fa_backward_h96(dqkv, dout, qkv, out, lse, B, T, C, NH, part, s); break;
        case 128: rows = fa_backward_h128(dqkv, dout, qkv, out, lse, B, T, C, NH, part, s); break;
    }
    if (!rows) { set_error("fused attention backward: no kernel for T=%d head size %d", T, HS); return; }
    after_launch("attention_backward_fused");
    if (dqkv_colsum) {  // the partial rows are laid out as B*rows batch entries; the chunk sums follow them
        const int nch = std::min(8, B);
        float* scratch = part + (size_t)B * rows * NH * 3 * HS;
        attn_colsum_part_k<<<dim3(3 * NH, nch), 256, 0, s>>>(scratch, part, B * rows, NH, C, HS);
        attn_colsum_final_k<<<cdiv(3 * C, 256), 256, 0, s>>>(dqkv_colsum, scratch, nch, 3 * C, colsum_store ? 1 : 0);
        after_launch("attention_colsum_reduce");
    }
}

}  // namespace vit

using namespace vit;
extern "C" {
void attention_forward(float* out, float* preatt, float* att, const float* inp, int B, int T, int C,
                       int NH) {
    attn_forward_f32(out, preatt, att, inp, B, T, C, NH, stream());
}
void attention_backward(float* dinp, float* dpreatt, float* datt, const float* dout,
                        const float* inp, const float* att, int B, int T, int C, int NH) {
    attn_backward_f32(dinp, dpreatt, datt, dout, inp, att, B, T, C, NH, stream());
}
int vit_attention_kernel_kind(int T, int C, int NH) {
    if (attn_fused_supported(T, C, NH)) return 1;
    if (attn_generic_supported(T, C, NH)) return 2;
    return 0;
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
void attention_backward_fused_bf16_ex(uint16_t* dinp, const uint16_t* dout, const uint16_t* inp,
                                      const uint16_t* out, const float* lse, int B, int T, int C, int NH,
                                      float* dqkv_bias) {
    attn_backward_fused(dinp, dout, inp, out, lse, B, T, C, NH, stream(), dqkv_bias);
}
}
