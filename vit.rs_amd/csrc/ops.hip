// ops.hip — the reference layer ops behind the C ABI (include/vit_ops.h), fp32 and bf16.
//
// Memory-bound ops (residual, GELU, LayerNorm, softmax/CE, SGD) are wave-per-row or
// grid-stride vectorised kernels; matmul_* go to the MFMA GEMMs of gemm.hip; attention to
// attention.hip.  Each op cites the reference function it replaces.
#include "ops_internal.h"
#include "ln_common.h"

namespace vit {

// ------------------------------------------------------------------ elementwise
__global__ void residual_fwd_k(float* __restrict__ out, const float* __restrict__ a,
                               const float* __restrict__ b, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        out[i] = a[i] + b[i];
}
__global__ void residual_bwd_k(float* __restrict__ d1, float* __restrict__ d2,
                               const float* __restrict__ dout, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const float g = dout[i];
        d1[i] += g;
        d2[i] += g;
    }
}
__global__ void gelu_fwd_k(float* __restrict__ out, const float* __restrict__ inp, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        out[i] = gelu_f(inp[i]);
}
__global__ void gelu_bwd_k(float* __restrict__ dinp, const float* __restrict__ inp,
                           const float* __restrict__ dout, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        dinp[i] += gelu_grad_f(inp[i]) * dout[i];
}
// bf16 GELU pair of the fused epilogues (gelu_fast_f / gelu_grad_fast_f, common.h), standalone
__global__ void gelu_fwd_bf16_k(bf16_t* __restrict__ out, const bf16_t* __restrict__ inp, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        out[i] = f2bf(gelu_fast_f(bf2f(inp[i])));
}
__global__ void gelu_bwd_bf16_k(float* __restrict__ dinp, const bf16_t* __restrict__ inp,
                                const bf16_t* __restrict__ dout, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        dinp[i] += gelu_grad_fast_f(bf2f(inp[i])) * bf2f(dout[i]);
}
__global__ void sgd_k(float* __restrict__ p, const float* __restrict__ g, long long n, float lr) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        p[i] = sgd_update(p[i], g[i], lr);
}
__global__ void f2bf_k(bf16_t* __restrict__ out, const float* __restrict__ inp, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        out[i] = f2bf(inp[i]);
}
__global__ void bf2f_k(float* __restrict__ out, const bf16_t* __restrict__ inp, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        out[i] = bf2f(inp[i]);
}

int grid_for(long long n, int threads) {
    long long b = (n + threads - 1) / threads;
    return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

// ------------------------------------------------------------------ LayerNorm
// one wave per row (train_vit.rs:453-480): two-pass mean/variance, biased var, eps 1e-5
template <typename TO>
__global__ __launch_bounds__(256) void ln_fwd_k(TO* __restrict__ out, float* __restrict__ mean,
                                                float* __restrict__ rstd,
                                                const float* __restrict__ inp,
                                                const float* __restrict__ w,
                                                const float* __restrict__ b, long long rows, int C) {
    const int lane = threadIdx.x & 63;
    const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float* x = inp + row * C;
    float s = 0.f;
    for (int i = lane; i < C; i += 64) s += x[i];
    const float m = warp_sum(s) / (float)C;
    float v = 0.f;
    for (int i = lane; i < C; i += 64) {
        const float d = x[i] - m;
        v += d * d;
    }
    v = warp_sum(v) / (float)C;
    const float r = 1.0f / sqrtf(v + 1e-5f);
    TO* o = out + row * C;
    for (int i = lane; i < C; i += 64) {
        const float y = (r * (x[i] - m)) * w[i] + b[i];
        if constexpr (sizeof(TO) == 2)
            o[i] = f2bf(y);
        else
            o[i] = y;
    }
    if (lane == 0) {
        mean[row] = m;
        rstd[row] = r;
    }
}

// train_vit.rs:603-637 (D5).  Two modes (compile time, so every load is unconditional):
//   ST = false: dinp (fp32) += LN_dinp(dout)                       (layernorm_backward, fp32 trainer)
//   ST = true : the trainer's residual-gradient stream in "bf16 + lo8" form (common.h lo8_*):
//               out = in + LN_dinp(dout), in/out as (bf16 plane, byte plane); dsum (nullable) gets the
//               column sums of out taken in fp32 (the next bias gradient)
// dweight / dbias (/ dsum) accumulate in per-wave LDS rows (each lane owns its columns: no atomics),
// are summed across the 4 waves in a fixed order and leave the block as its partial row
// part[blockIdx.x][2C or 3C] (dw | db | dsum), summed in a fixed order by rows_reduce_add — by the
// launcher, or by the trainer across micro-batches: deterministic.  TD: dout type (fp32 or bf16).
struct LnbIo {
    float* dinp;            // ST = false: accumulated in place
    bf16_t* hi_out;         // ST = true
    uint8_t* lo_out;
    const bf16_t* hi_in;
    const uint8_t* lo_in;
    float *dweight, *dbias, *dsum, *part;
};
__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16_t v) { return bf2f(v); }
__device__ __forceinline__ void lnb_flush(const LnbIo& io, const float* sm, int C) {
    __syncthreads();
    const int nsum = io.dsum ? 3 * C : 2 * C;
    for (int i = threadIdx.x; i < nsum; i += 256) {
        const float t = sm[i] + sm[3 * C + i] + sm[6 * C + i] + sm[9 * C + i];
        io.part[(long long)blockIdx.x * nsum + i] = t;
    }
}
// any C (the vectorised kernel below needs C % 256 == 0)
template <typename TD, bool ST>
__global__ __launch_bounds__(256) void ln_bwd_k(LnbIo io, const TD* __restrict__ dout,
                                                const float* __restrict__ inp,
                                                const float* __restrict__ weight,
                                                const float* __restrict__ mean,
                                                const float* __restrict__ rstd, long long rows, int C) {
    extern __shared__ float sm[];  // [4 waves][3][C]
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float* pw = sm + wave * 3 * C;
    float* pb = pw + C;
    float* ps = pw + 2 * C;
    for (int i = lane; i < C; i += 64) pw[i] = pb[i] = ps[i] = 0.f;
    const long long nwaves = (long long)gridDim.x * 4;
    for (long long row = blockIdx.x * 4LL + wave; row < rows; row += nwaves) {
        const TD* dy = dout + row * C;
        const float* x = inp + row * C;
        const float mu = mean[row], rs = rstd[row];
        float a = 0.f, bsum = 0.f;
        for (int i = lane; i < C; i += 64) {
            const float d = to_f32(dy[i]);
            const float nrm = (x[i] - mu) * rs;
            const float dn = weight[i] * d;
            a += dn;
            bsum += dn * nrm;
        }
        const float dnorm_mean = warp_sum(a) / (float)C;
        const float dnorm_norm_mean = warp_sum(bsum) / (float)C;
        for (int i = lane; i < C; i += 64) {
            const float d = to_f32(dy[i]);
            const float nrm = (x[i] - mu) * rs;
            const float dn = weight[i] * d;
            pb[i] += d;
            pw[i] += nrm * d;
            float dval = dn;
            dval -= dnorm_mean;
            dval -= nrm * dnorm_norm_mean;
            dval *= rs;
            const long long o = row * C + i;
            if constexpr (ST) {
                const float t = lo8_decode(bf2f(io.hi_in[o]), io.lo_in[o]) + dval;
                const bf16_t h = f2bf(t);
                io.hi_out[o] = h;
                io.lo_out[o] = (uint8_t)lo8_encode(t, bf2f(h));
                ps[i] += t;
            } else {
                io.dinp[o] += dval;
            }
        }
    }
    lnb_flush(io, sm, C);
}

// Vectorised LayerNorm for C % 256 == 0: one wave per row, NV float4 per lane held in registers
// (the row is read once).  Same formulas as ln_fwd_k / ln_bwd_k.
template <int NV, typename TO>
__global__ __launch_bounds__(256) void ln_fwd_vec_k(TO* __restrict__ out, float* __restrict__ mean,
                                                    float* __restrict__ rstd,
                                                    const float* __restrict__ inp,
                                                    const float* __restrict__ w,
                                                    const float* __restrict__ b, long long rows,
                                                    int C) {
    const int lane = threadIdx.x & 63;
    const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float4* x4 = reinterpret_cast<const float4*>(inp + row * C);
    float4 v[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) v[j] = x4[lane + 64 * j];
    float m, r;
    ln_vec_stats<NV>(v, C, m, r);  // ln_common.h (shared with ln_fwd_mx_k)
#pragma unroll
    for (int j = 0; j < NV; j++) {
        const int k = lane + 64 * j;
        const float4 y = ln_vec_y(v[j], reinterpret_cast<const float4*>(w)[k], reinterpret_cast<const float4*>(b)[k], m, r);
        if constexpr (sizeof(TO) == 2)
            reinterpret_cast<uint2*>(out + row * C)[k] = make_uint2(pack_bf16x2(y.x, y.y), pack_bf16x2(y.z, y.w));
        else
            reinterpret_cast<float4*>(out + row * C)[k] = y;
    }
    if (lane == 0) {
        mean[row] = m;
        rstd[row] = r;
    }
}

// 4 consecutive values k*4 .. k*4+3 of a row (fp32 or bf16 storage) as fp32
__device__ __forceinline__ float4 ld4(const float* p, int k) { return reinterpret_cast<const float4*>(p)[k]; }
__device__ __forceinline__ float4 ld4(const bf16_t* p, int k) {
    const uint2 u = reinterpret_cast<const uint2*>(p)[k];
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                       __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}

// C % 256 == 0: one wave per row, NV float4 per lane in registers, the next row's loads in flight
// while this row reduces and stores (every load unconditional — the last row re-fetches itself — so
// the compiler never drains the prefetch with a vmcnt(0))
template <int NV, typename TD, bool ST>
__global__ __launch_bounds__(256) void ln_bwd_vec_k(LnbIo io, const TD* __restrict__ dout,
                                                    const float* inp,  // not restrict: keeps its prefetch above the row's stores
                                                    const float* __restrict__ weight,
                                                    const float* __restrict__ mean,
                                                    const float* __restrict__ rstd, long long rows,
                                                    int C) {
    extern __shared__ float sm[];  // [4 waves][3][C]: this wave's dweight / dbias / dsum partials
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // the column partials live in the wave's LDS rows (each lane owns its 4*NV columns, so the
    // read-modify-writes need no synchronisation)
    float4* pw = reinterpret_cast<float4*>(sm + wave * 3 * C);
    float4* pb = reinterpret_cast<float4*>(sm + wave * 3 * C + C);
    float4* ps = reinterpret_cast<float4*>(sm + wave * 3 * C + 2 * C);
    float4 w4[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) {
        w4[j] = reinterpret_cast<const float4*>(weight)[lane + 64 * j];
        pw[lane + 64 * j] = pb[lane + 64 * j] = ps[lane + 64 * j] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const long long nwaves = (long long)gridDim.x * 4;
    float4 pdy[NV], px[NV], pri[NV];
    uint32_t plo[NV];
    float pmu = 0.f, prs = 0.f;
    auto fetch = [&](long long r) {
        const TD* dyr = dout + r * C;
        const float4* x4 = reinterpret_cast<const float4*>(inp + r * C);
#pragma unroll
        for (int j = 0; j < NV; j++) {
            pdy[j] = ld4(dyr, lane + 64 * j);
            px[j] = x4[lane + 64 * j];
            if constexpr (ST) {
                pri[j] = ld4(io.hi_in + r * C, lane + 64 * j);
                plo[j] = reinterpret_cast<const uint32_t*>(io.lo_in + r * C)[lane + 64 * j];
            } else {
                pri[j] = reinterpret_cast<const float4*>(io.dinp + r * C)[lane + 64 * j];
            }
        }
        pmu = mean[r];
        prs = rstd[r];
    };
    long long row = blockIdx.x * 4LL + wave;
    if (row < rows) fetch(row);
    for (; row < rows; row += nwaves) {
        float4 dy[NV], xr[NV], ri[NV], nr[NV];
#pragma unroll
        for (int j = 0; j < NV; j++) {
            dy[j] = pdy[j];
            xr[j] = px[j];
            ri[j] = pri[j];
            if constexpr (ST) {
                const uint32_t q = plo[j];
                ri[j] = make_float4(lo8_decode(ri[j].x, q), lo8_decode(ri[j].y, q >> 8), lo8_decode(ri[j].z, q >> 16),
                                    lo8_decode(ri[j].w, q >> 24));
            }
        }
        const float mu = pmu, rs = prs;
        fetch(row + nwaves < rows ? row + nwaves : row);
        // keep the prefetch at the top: the scheduler otherwise sinks it to the end of the row to
        // reuse this row's registers, and the next iteration waits a full HBM round trip
        __builtin_amdgcn_sched_barrier(0);
        float4 dvv[NV];
        ln_bwd_row<NV>(dy, xr, w4, mu, rs, C, nr, dvv);  // ln_common.h (shared with ln_bwd_mx_k)
#pragma unroll
        for (int j = 0; j < NV; j++) {
            const int k = lane + 64 * j;
            {
                float4 b = pb[k], w = pw[k];
                b.x += dy[j].x; b.y += dy[j].y; b.z += dy[j].z; b.w += dy[j].w;
                w.x += nr[j].x * dy[j].x; w.y += nr[j].y * dy[j].y;
                w.z += nr[j].z * dy[j].z; w.w += nr[j].w * dy[j].w;
                pb[k] = b;
                pw[k] = w;
            }
            const float4 dv = dvv[j];
            const float4 t = make_float4(ri[j].x + dv.x, ri[j].y + dv.y, ri[j].z + dv.z, ri[j].w + dv.w);
            if constexpr (ST) {
                float4 u = ps[k];
                u.x += t.x; u.y += t.y; u.z += t.z; u.w += t.w;
                ps[k] = u;
                const uint2 h = make_uint2(pack_bf16x2(t.x, t.y), pack_bf16x2(t.z, t.w));
                reinterpret_cast<uint2*>(io.hi_out + row * C)[k] = h;
                reinterpret_cast<uint32_t*>(io.lo_out + row * C)[k] =
                    lo8_encode(t.x, __uint_as_float(h.x << 16)) |
                    (lo8_encode(t.y, __uint_as_float(h.x & 0xffff0000u)) << 8) |
                    (lo8_encode(t.z, __uint_as_float(h.y << 16)) << 16) |
                    (lo8_encode(t.w, __uint_as_float(h.y & 0xffff0000u)) << 24);
            } else {
                reinterpret_cast<float4*>(io.dinp + row * C)[k] = t;
            }
        }
    }
    lnb_flush(io, sm, C);
}

// ------------------------------------------------------------------ softmax / cross-entropy
// train_vit.rs:493-517 — block per row, max init -10000 (:499)
__global__ __launch_bounds__(256) void softmax_k(float* __restrict__ probs,
                                                 const float* __restrict__ logits, int V) {
    __shared__ float red[4];
    const long long row = blockIdx.x;
    const float* l = logits + row * V;
    float* pr = probs + row * V;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float m = -10000.0f;
    for (int i = threadIdx.x; i < V; i += 256) m = fmaxf(m, l[i]);
    m = warp_max(m);
    if (lane == 0) red[w] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    float s = 0.f;
    for (int i = threadIdx.x; i < V; i += 256) {
        const float e = expf(l[i] - m);
        pr[i] = e;
        s += e;
    }
    s = warp_sum(s);
    if (lane == 0) red[w] = s;
    __syncthreads();
    s = red[0] + red[1] + red[2] + red[3];
    const float inv = 1.0f / s;
    for (int i = threadIdx.x; i < V; i += 256) pr[i] = pr[i] * inv;
}
__global__ void ce_fwd_k(float* __restrict__ losses, const float* __restrict__ probs,
                         const int* __restrict__ targets, long long rows, int V) {
    const long long r = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const int t = targets[r];  // out-of-range labels (the host checks host arrays) give NaN, never an OOB read
    losses[r] = (t >= 0 && t < V) ? -logf(probs[r * V + t]) : __builtin_nanf("");
}
__global__ void ce_bwd_k(float* __restrict__ dlogits, const float* __restrict__ dlosses,
                         const float* __restrict__ probs, const int* __restrict__ targets,
                         long long rows, int V) {
    const long long n = rows * V;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const long long r = i / V;
        const int v = (int)(i - r * V);
        const float ind = v == targets[r] ? 1.0f : 0.0f;
        dlogits[i] += (probs[i] - ind) * dlosses[r];
    }
}

// ------------------------------------------------------------------ patch embedding
// im2col of [B,3,IMG,IMG] -> rows (b,p) x cols (c*P+kh)*P+kw  (Conv2d weight flatten order)
template <typename TO>
__global__ void im2col_k(TO* __restrict__ out, const float* __restrict__ px, int B, int IMG, int P) {
    const int gw = IMG / P, NP = gw * gw, K = 3 * P * P;
    const long long n = (long long)B * NP * K;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < n;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long row = idx / K;
        const int k = (int)(idx - row * K);
        const int b = (int)(row / NP), p = (int)(row - (long long)b * NP);
        const int c = k / (P * P), r = k - c * P * P, kh = r / P, kw = r - kh * P;
        const int y = (p / gw) * P + kh, x = (p % gw) * P + kw;
        const float v = px[(((long long)b * 3 + c) * IMG + y) * IMG + x];
        if constexpr (sizeof(TO) == 2) out[idx] = f2bf(v); else out[idx] = v;
    }
}
// the same, 8 consecutive k (= 8 consecutive pixels of one image row: P % 8 == 0, IMG % 8 == 0) per
// thread: two 16-B loads, one 16-B (bf16) or two (fp32) stores, one index decode per 8 outputs
template <typename TO>
__global__ void im2col_vec_k(TO* __restrict__ out, const float* __restrict__ px, int B, int IMG, int P) {
    const int gw = IMG / P, NP = gw * gw, K8 = 3 * P * P / 8;
    const long long n = (long long)B * NP * K8;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < n;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long row = idx / K8;
        const int k = (int)(idx - row * K8) * 8;
        const int b = (int)(row / NP), p = (int)(row - (long long)b * NP);
        const int c = k / (P * P), r = k - c * P * P, kh = r / P, kw = r - kh * P;
        const int y = (p / gw) * P + kh, x = (p % gw) * P + kw;
        const float4* src = reinterpret_cast<const float4*>(px + (((long long)b * 3 + c) * IMG + y) * IMG + x);
        const float4 a = src[0], d = src[1];
        if constexpr (sizeof(TO) == 2) {
            reinterpret_cast<uint4*>(out)[idx] = make_uint4(pack_bf16x2(a.x, a.y), pack_bf16x2(a.z, a.w),
                                                            pack_bf16x2(d.x, d.y), pack_bf16x2(d.z, d.w));
        } else {
            reinterpret_cast<float4*>(out)[2 * idx] = a;
            reinterpret_cast<float4*>(out)[2 * idx + 1] = d;
        }
    }
}
// the same into rows of KPP columns (zeros past K = 3*P*P), 8 columns (one 16-B store) per thread
__global__ void im2col_pad_k(bf16_t* __restrict__ out, const float* __restrict__ px, int B, int IMG, int P, int KPP) {
    const int gw = IMG / P, NP = gw * gw, K = 3 * P * P, K8 = KPP / 8, PP = P * P;
    const long long n = (long long)B * NP * K8;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < n;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long row = idx / K8;
        const int k0 = (int)(idx - row * K8) * 8;
        const int b = (int)(row / NP), p = (int)(row - (long long)b * NP);
        const int y0 = (p / gw) * P, x0 = (p % gw) * P;
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int k = k0 + j;
            v[j] = 0.f;
            if (k < K) {
                const int c = k / PP, r = k - c * PP, kh = r / P, kw = r - kh * P;
                v[j] = px[(((long long)b * 3 + c) * IMG + y0 + kh) * IMG + x0 + kw];
            }
        }
        *reinterpret_cast<uint4*>(out + row * KPP + k0) =
            make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    }
}
// encoded[b,0] = cls + wpe[0]; encoded[b,1+p] = emb[b*NP+p] + wpe[1+p]
__global__ void patch_assemble_k(float* __restrict__ enc, const float* __restrict__ emb,
                                 const float* __restrict__ cls, const float* __restrict__ wpe,
                                 int B, int NP, int C) {
    const int T = NP + 1;
    const long long n = (long long)B * T * C;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < n;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long bt = idx / C;
        const int c = (int)(idx - bt * C);
        const int b = (int)(bt / T), t = (int)(bt - (long long)b * T);
        const float base = t == 0 ? cls[c] : emb[((long long)b * NP + t - 1) * C + c];
        enc[idx] = base + wpe[(long long)t * C + c];
    }
}
// the same for C % 4 == 0: 4 columns per thread (16-B loads and stores, one index decode per 4)
__global__ void patch_assemble_vec_k(float* __restrict__ enc, const float* __restrict__ emb,
                                     const float* __restrict__ cls, const float* __restrict__ wpe, int B, int NP,
                                     int C) {
    const int T = NP + 1, C4 = C / 4;
    const long long n = (long long)B * T * C4;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < n;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long bt = idx / C4;
        const int c4 = (int)(idx - bt * C4);
        const int b = (int)(bt / T), t = (int)(bt - (long long)b * T);
        const float4 base = t == 0 ? reinterpret_cast<const float4*>(cls)[c4]
                                   : reinterpret_cast<const float4*>(emb + ((long long)b * NP + t - 1) * C)[c4];
        const float4 w = reinterpret_cast<const float4*>(wpe + (long long)t * C)[c4];
        reinterpret_cast<float4*>(enc)[idx] = make_float4(base.x + w.x, base.y + w.y, base.z + w.z, base.w + w.w);
    }
}
// patch rows of a bf16 [B][T][C] gradient into [B*NP][C] bf16, 8 columns (16 B) per thread (C % 8 == 0)
__global__ void patch_gather_vec_k(bf16_t* __restrict__ out, const bf16_t* __restrict__ denc, int B, int NP, int C) {
    const int T = NP + 1, C8 = C / 8;
    const long long n = (long long)B * NP * C8;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < n;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long r = idx / C8;
        const int c8 = (int)(idx - r * C8);
        const int b = (int)(r / NP), p = (int)(r - (long long)b * NP);
        reinterpret_cast<uint4*>(out)[idx] = reinterpret_cast<const uint4*>(denc + ((long long)b * T + 1 + p) * C)[c8];
    }
}
// gather the patch rows of dencoded into [B*NP, C] (TO = float or bf16; TI likewise)
template <typename TO, typename TI>
__global__ void patch_gather_k(TO* __restrict__ out, const TI* __restrict__ denc, const uint8_t* __restrict__ lo,
                               int B, int NP, int C) {
    const int T = NP + 1;
    const long long n = (long long)B * NP * C;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < n;
         idx += (long long)gridDim.x * blockDim.x) {
        const long long r = idx / C;
        const int c = (int)(idx - r * C);
        const int b = (int)(r / NP), p = (int)(r - (long long)b * NP);
        const long long src = ((long long)b * T + 1 + p) * C + c;
        const TI v = denc[src];
        if constexpr (sizeof(TO) == sizeof(TI)) out[idx] = v;
        else if constexpr (sizeof(TO) == 2) out[idx] = f2bf(v);
        else out[idx] = lo ? lo8_decode(bf2f(v), lo[src]) : bf2f(v);
    }
}
// dwpe[t,c] += colsum_t[c] = sum_b denc[b,t,c] (a fixed order); colsum_t -> tsum[t][c]
template <typename TI>
__global__ void patch_small_grads_k(float* __restrict__ dwpe, float* __restrict__ tsum,
                                    const TI* __restrict__ denc, const uint8_t* __restrict__ lo, int B, int T,
                                    int C) {
    const long long n = (long long)T * C;
    for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < n;
         idx += (long long)gridDim.x * blockDim.x) {
        const int t = (int)(idx / C), c = (int)(idx - (long long)t * C);
        // 8 independent partial sums (images b = j mod 8), added in a fixed order: eight loads in
        // flight per thread instead of one dependent chain of B
        float ps[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const long long bs = (long long)T * C, e0 = (long long)t * C + c;
        int b = 0;
        for (; b + 8 <= B; b += 8) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const long long e = e0 + (b + j) * bs;
                ps[j] += lo ? lo8_decode(to_f32(denc[e]), lo[e]) : to_f32(denc[e]);
            }
        }
        for (int j = 0; b < B; b++, j++) {
            const long long e = e0 + b * bs;
            ps[j] += lo ? lo8_decode(to_f32(denc[e]), lo[e]) : to_f32(denc[e]);
        }
        const float s = ((ps[0] + ps[1]) + (ps[2] + ps[3])) + ((ps[4] + ps[5]) + (ps[6] + ps[7]));
        dwpe[idx] += s;
        tsum[idx] = s;
    }
}
// The trainer's form ("bf16 + lo8" input, C % 8 == 0): the images split into `nch` chunks; thread
// (chunk y, position t, 8 columns) sums its chunk's images in order with 16-B / 8-B loads into
// part[y][t][c..c+8]; psg_final_k adds the chunks in order (deterministic).  The one-thread-per-column
// loop over all B images above ran latency-bound at 0.6 TB/s.
__global__ void psg_part_k(float* __restrict__ part, const bf16_t* __restrict__ denc, const uint8_t* __restrict__ lo,
                           int B, int T, int C, int bc) {
    const int C8 = C / 8;
    const long long tc8 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (tc8 >= (long long)T * C8) return;
    const int y = blockIdx.y, b0 = y * bc, b1 = min(B, b0 + bc);
    const long long e0 = tc8 * 8, bs = (long long)T * C;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int b = b0; b < b1; b++) {
        const long long e = e0 + b * bs;
        const uint4 h = *reinterpret_cast<const uint4*>(denc + e);
        const uint2 q = *reinterpret_cast<const uint2*>(lo + e);
        const uint32_t hw[4] = {h.x, h.y, h.z, h.w}, qw[2] = {q.x, q.y};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t qq = qw[j >> 1] >> (16 * (j & 1));
            acc[2 * j] += lo8_decode(__uint_as_float(hw[j] << 16), qq & 0xffu);
            acc[2 * j + 1] += lo8_decode(__uint_as_float(hw[j] & 0xffff0000u), (qq >> 8) & 0xffu);
        }
    }
    float4* dst = reinterpret_cast<float4*>(part + (long long)y * bs + e0);
    dst[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    dst[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
}
__global__ void psg_final_k(float* __restrict__ dwpe, float* __restrict__ tsum, const float* __restrict__ part,
                            long long n, int nch) {
    const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = 0.f;
    for (int y = 0; y < nch; y++) s += part[y * n + i];
    dwpe[i] += s;
    tsum[i] = s;
}
// dcls[c] += tsum[0][c];  dpatch_b[c] += sum_{t>0} tsum[t][c] (a fixed order: no atomics)
__global__ void patch_small_grads_fin_k(float* __restrict__ dcls, float* __restrict__ dpb,
                                        const float* __restrict__ tsum, int T, int C) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float ps[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // t = 1 + j (mod 8): 8 loads in flight
    int t = 1;
    for (; t + 8 <= T; t += 8) {
#pragma unroll
        for (int j = 0; j < 8; j++) ps[j] += tsum[(long long)(t + j) * C + c];
    }
    for (int j = 0; t < T; t++, j++) ps[j] += tsum[(long long)t * C + c];
    const float s = ((ps[0] + ps[1]) + (ps[2] + ps[3])) + ((ps[4] + ps[5]) + (ps[6] + ps[7]));
    dcls[c] += tsum[c];
    dpb[c] += s;
}

// ------------------------------------------------------------------ launch helpers (internal)
template <typename TO>
static void ln_forward_any(TO* out, float* mean, float* rstd, const float* inp, const float* w,
                           const float* b, long long rows, int C, hipStream_t s) {
    if (rows <= 0) return;
    const int g = cdiv(rows, 4);
    const bool vec = C % 256 == 0 && C <= 2048 && (((uintptr_t)inp | (uintptr_t)out | (uintptr_t)w | (uintptr_t)b) & 15) == 0;
    switch (vec ? C / 256 : 0) {
        case 1: ln_fwd_vec_k<1, TO><<<g, 256, 0, s>>>(out, mean, rstd, inp, w, b, rows, C); break;
        case 2: ln_fwd_vec_k<2, TO><<<g, 256, 0, s>>>(out, mean, rstd, inp, w, b, rows, C); break;
        case 3: ln_fwd_vec_k<3, TO><<<g, 256, 0, s>>>(out, mean, rstd, inp, w, b, rows, C); break;
        case 4: ln_fwd_vec_k<4, TO><<<g, 256, 0, s>>>(out, mean, rstd, inp, w, b, rows, C); break;
        case 5: ln_fwd_vec_k<5, TO><<<g, 256, 0, s>>>(out, mean, rstd, inp, w, b, rows, C); break;
        case 6: ln_fwd_vec_k<6, TO><<<g, 256, 0, s>>>(out, mean, rstd, inp, w, b, rows, C); break;
        case 8: ln_fwd_vec_k<8, TO><<<g, 256, 0, s>>>(out, mean, rstd, inp, w, b, rows, C); break;
        default: ln_fwd_k<TO><<<g, 256, 0, s>>>(out, mean, rstd, inp, w, b, rows, C); break;
    }
    after_launch("layernorm_forward");
}
void ln_forward_f32(float* out, float* mean, float* rstd, const float* inp, const float* w,
                    const float* b, long long rows, int C, hipStream_t s) {
    ln_forward_any<float>(out, mean, rstd, inp, w, b, rows, C, s);
}
void ln_forward_bf16(bf16_t* out, float* mean, float* rstd, const float* inp, const float* w,
                     const float* b, long long rows, int C, hipStream_t s) {
    ln_forward_any<bf16_t>(out, mean, rstd, inp, w, b, rows, C, s);
}
int ln_bwd_blocks(long long rows);
template <typename TD, bool ST>
static void ln_backward_any(LnbIo io, const TD* dout, const float* inp, const float* w,
                            const float* mean, const float* rstd, long long rows, int C, hipStream_t s,
                            float* ws = nullptr) {
    if (rows <= 0) return;
    // io.part set: the caller reduces the partial rows; else they go to ws (nullptr = thread
    // workspace) and are added into dweight / dbias / dsum here
    const bool reduce = io.part == nullptr;
    const int nsum = io.dsum ? 3 * C : 2 * C;
    if (reduce) {
        io.part = ws ? ws : (float*)workspace((size_t)ln_bwd_blocks(rows) * nsum * sizeof(float));
        if (!io.part) return;
    }
    const bool vec = C % 256 == 0 && C <= 2048 &&
                     (((uintptr_t)io.dinp | (uintptr_t)dout | (uintptr_t)inp | (uintptr_t)w |
                       (uintptr_t)io.hi_in | (uintptr_t)io.hi_out | (uintptr_t)io.lo_in | (uintptr_t)io.lo_out) & 15) == 0;
    const int grid = ln_bwd_blocks(rows);
    const size_t lds = 12 * (size_t)C * sizeof(float);
    if (lds > 160 * 1024) { set_error("layernorm_backward: C=%d exceeds the LDS column partials", C); return; }
    if (!vec) {
        if (lds > 64 * 1024) VIT_HIP(hipFuncSetAttribute((const void*)ln_bwd_k<TD, ST>,
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        ln_bwd_k<TD, ST><<<grid, 256, lds, s>>>(io, dout, inp, w, mean, rstd, rows, C);
    } else {
#define VIT_LNB(NV)                                                                                        \
    if (lds > 64 * 1024) VIT_HIP(hipFuncSetAttribute((const void*)ln_bwd_vec_k<NV, TD, ST>,                 \
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    ln_bwd_vec_k<NV, TD, ST><<<grid, 256, lds, s>>>(io, dout, inp, w, mean, rstd, rows, C)
        switch (C / 256) {
            case 1: VIT_LNB(1); break;
            case 2: VIT_LNB(2); break;
            case 3: VIT_LNB(3); break;
            case 4: VIT_LNB(4); break;
            case 5: VIT_LNB(5); break;
            case 6: VIT_LNB(6); break;
            case 7: VIT_LNB(7); break;
            default: VIT_LNB(8); break;
        }
#undef VIT_LNB
    }
    after_launch("layernorm_backward");
    if (reduce) {
        const RowsJob jobs[3] = {{io.dweight, io.part, grid, nsum, C}, {io.dbias, io.part + C, grid, nsum, C},
                                 {io.dsum, io.part + 2 * C, grid, nsum, C}};
        rows_reduce_add(jobs, io.dsum ? 3 : 2, s);
    }
}
int ln_bwd_blocks(long long rows) {
    const long long g = (rows + 15) / 16;  // ~4 rows per wave
    // at most one round of resident blocks (3 per CU at 142-144 VGPRs; 256 CUs)
    return (int)(g < 1 ? 1 : (g > 768 ? 768 : g));
}
void ln_backward_f32(float* dinp, float* dw, float* db, const float* dout, const float* inp,
                     const float* w, const float* mean, const float* rstd, long long rows, int C,
                     hipStream_t s, float* ws) {
    LnbIo io{};
    io.dinp = dinp; io.dweight = dw; io.dbias = db;
    ln_backward_any<float, false>(io, dout, inp, w, mean, rstd, rows, C, s, ws);
}
void ln_backward_bf16_stream(bf16_t* dres_out, uint8_t* lo_out, const bf16_t* dres_in, const uint8_t* lo_in,
                             float* dw, float* db, float* dres_colsum, const bf16_t* dout, const float* inp,
                             const float* w, const float* mean, const float* rstd, long long rows, int C,
                             hipStream_t s, float* part) {
    if (!dres_out || !lo_out || !dres_in || !lo_in) { set_error("layernorm_backward: the bf16 stream needs its 4 planes"); return; }
    if (((uintptr_t)lo_in | (uintptr_t)lo_out) & 3) { set_error("layernorm_backward: lo8 planes need 4-B alignment"); return; }
    LnbIo io{};
    io.hi_out = dres_out; io.lo_out = lo_out; io.hi_in = dres_in; io.lo_in = lo_in;
    io.dweight = dw; io.dbias = db; io.dsum = dres_colsum; io.part = part;
    ln_backward_any<bf16_t, true>(io, dout, inp, w, mean, rstd, rows, C, s);
}
// out[c][r] = in[r][c] for `count` matrices of R x Cc bf16 spaced `stride` elements apart
// (in and out use the same stride); 64 x 64 tiles through LDS, 16-B global accesses.
__global__ __launch_bounds__(256) void transpose_bf16_k(bf16_t* __restrict__ out,
                                                        const bf16_t* __restrict__ in, int R, int Cc,
                                                        long long stride) {
    __shared__ uint16_t tile[64][64 + 2];
    const long long mo = (long long)blockIdx.z * stride;
    const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
    const int t = threadIdx.x, tr = t >> 2, tc = (t & 3) * 16;
#pragma unroll
    for (int h = 0; h < 2; h++) {  // 256 threads x 2 x 8 elements = the 64 x 64 tile
        const int r = r0 + tr, c = c0 + tc + h * 8;
        // clamped address, zeros selected after the load (no load behind a branch)
        const uint4 ld = *reinterpret_cast<const uint4*>(in + mo + (long long)min(r, R - 1) * Cc + min(c, Cc - 8));
        const uint4 v = (r < R && c < Cc) ? ld : make_uint4(0, 0, 0, 0);
        const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int j = 0; j < 8; j++) tile[tr][tc + h * 8 + j] = e[j];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int oc = c0 + tr, orr = r0 + tc + h * 8;  // output row = input column
        if (oc >= Cc || orr >= R) continue;
        uint16_t e[8];
#pragma unroll
        for (int j = 0; j < 8; j++) e[j] = tile[tc + h * 8 + j][tr];
        *reinterpret_cast<uint4*>(out + mo + (long long)oc * R + orr) = *reinterpret_cast<const uint4*>(e);
    }
}
void transpose_bf16(bf16_t* out, const bf16_t* in, int R, int Cc, int count, long long stride,
                    hipStream_t s) {
    if (R <= 0 || Cc <= 0 || count <= 0) return;
    if (R % 8 || Cc % 8) { set_error("transpose_bf16: dims must be multiples of 8 (%d x %d)", R, Cc); return; }
    dim3 grid(cdiv(Cc, 64), cdiv(R, 64), count);
    transpose_bf16_k<<<grid, 256, 0, s>>>(out, in, R, Cc, stride);
    after_launch("transpose_bf16");
}
void convert_f2bf(bf16_t* out, const float* inp, long long n, hipStream_t s) {
    if (n <= 0) return;
    f2bf_k<<<grid_for(n, 256), 256, 0, s>>>(out, inp, n);
    after_launch("convert_f32_to_bf16");
}
void sgd(float* p, const float* g, long long n, float lr, hipStream_t s) {
    if (n <= 0) return;
    sgd_k<<<grid_for(n, 256), 256, 0, s>>>(p, g, n, lr);
    after_launch("sgd_step");
}
void softmax_rows(float* probs, const float* logits, long long rows, int V, hipStream_t s) {
    if (rows <= 0) return;
    softmax_k<<<(unsigned)rows, 256, 0, s>>>(probs, logits, V);
    after_launch("softmax_forward");
}
void ce_forward(float* losses, const float* probs, const int* targets, long long rows, int V,
                hipStream_t s) {
    if (rows <= 0) return;
    ce_fwd_k<<<cdiv(rows, 256), 256, 0, s>>>(losses, probs, targets, rows, V);
    after_launch("crossentropy_forward");
}
void ce_backward(float* dlogits, const float* dlosses, const float* probs, const int* targets,
                 long long rows, int V, hipStream_t s) {
    if (rows <= 0) return;
    ce_bwd_k<<<grid_for(rows * V, 256), 256, 0, s>>>(dlogits, dlosses, probs, targets, rows, V);
    after_launch("crossentropy_softmax_backward");
}
static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
template <typename TO>
static void im2col_any(TO* out, const float* px, int B, int IMG, int P, hipStream_t s) {
    const long long n = (long long)B * (IMG / P) * (IMG / P) * 3 * P * P;
    if (P % 8 == 0 && IMG % 8 == 0 && al16(out) && al16(px))
        im2col_vec_k<TO><<<grid_for(n / 8, 256), 256, 0, s>>>(out, px, B, IMG, P);
    else
        im2col_k<TO><<<grid_for(n, 256), 256, 0, s>>>(out, px, B, IMG, P);
}
void im2col_f32(float* out, const float* px, int B, int IMG, int P, hipStream_t s) {
    im2col_any<float>(out, px, B, IMG, P, s);
    after_launch("im2col");
}
void im2col_bf16(bf16_t* out, const float* px, int B, int IMG, int P, hipStream_t s) {
    im2col_any<bf16_t>(out, px, B, IMG, P, s);
    after_launch("im2col_bf16");
}
void im2col_pad_bf16(bf16_t* out, const float* px, int B, int IMG, int P, int KPP, hipStream_t s) {
    const long long n = (long long)B * (IMG / P) * (IMG / P) * (KPP / 8);
    if (KPP % 8 || KPP < 3 * P * P || !al16(out)) {
        set_error("im2col_pad_bf16: KPP %% 8 == 0, KPP >= 3*P*P and a 16-B aligned output required (KPP=%d)", KPP);
        return;
    }
    im2col_pad_k<<<grid_for(n, 256), 256, 0, s>>>(out, px, B, IMG, P, KPP);
    after_launch("im2col_pad_bf16");
}
void patch_assemble(float* enc, const float* emb, const float* cls, const float* wpe, int B,
                    int NP, int C, hipStream_t s) {
    const long long n = (long long)B * (NP + 1) * C;
    if (C % 4 == 0 && al16(enc) && al16(emb) && al16(cls) && al16(wpe))
        patch_assemble_vec_k<<<grid_for(n / 4, 256), 256, 0, s>>>(enc, emb, cls, wpe, B, NP, C);
    else
        patch_assemble_k<<<grid_for(n, 256), 256, 0, s>>>(enc, emb, cls, wpe, B, NP, C);
    after_launch("patch_assemble");
}
void patch_gather_f32(float* out, const float* denc, int B, int NP, int C, hipStream_t s) {
    const long long n = (long long)B * NP * C;
    patch_gather_k<float, float><<<grid_for(n, 256), 256, 0, s>>>(out, denc, nullptr, B, NP, C);
    after_launch("patch_gather");
}
void patch_gather_bf16(bf16_t* out, const float* denc, int B, int NP, int C, hipStream_t s) {
    const long long n = (long long)B * NP * C;
    patch_gather_k<bf16_t, float><<<grid_for(n, 256), 256, 0, s>>>(out, denc, nullptr, B, NP, C);
    after_launch("patch_gather_bf16");
}
void patch_gather_f32(float* out, const bf16_t* denc, const uint8_t* lo, int B, int NP, int C, hipStream_t s) {
    const long long n = (long long)B * NP * C;
    patch_gather_k<float, bf16_t><<<grid_for(n, 256), 256, 0, s>>>(out, denc, lo, B, NP, C);
    after_launch("patch_gather");
}
void patch_gather_bf16(bf16_t* out, const bf16_t* denc, int B, int NP, int C, hipStream_t s) {
    const long long n = (long long)B * NP * C;
    if (C % 8 == 0 && al16(out) && al16(denc))
        patch_gather_vec_k<<<grid_for(n / 8, 256), 256, 0, s>>>(out, denc, B, NP, C);
    else
        patch_gather_k<bf16_t, bf16_t><<<grid_for(n, 256), 256, 0, s>>>(out, denc, nullptr, B, NP, C);
    after_launch("patch_gather_bf16");
}
template <typename TI>
static void patch_small_grads_any(float* dcls, float* dwpe, float* dpb, const TI* denc, const uint8_t* lo, int B,
                                  int T, int C, hipStream_t s, float* ws) {
    const long long n = (long long)T * C;
    if (!ws) ws = (float*)workspace(n * sizeof(float));
    if (!ws) return;
    patch_small_grads_k<TI><<<grid_for(n, 256), 256, 0, s>>>(dwpe, ws, denc, lo, B, T, C);
    patch_small_grads_fin_k<<<cdiv(C, 256), 256, 0, s>>>(dcls, dpb, ws, T, C);
}
void patch_small_grads(float* dcls, float* dwpe, float* dpb, const float* denc, int B, int T,
                       int C, hipStream_t s, float* ws) {
    patch_small_grads_any(dcls, dwpe, dpb, denc, nullptr, B, T, C, s, ws);
    after_launch("patch_small_grads");
}
void patch_small_grads(float* dcls, float* dwpe, float* dpb, const bf16_t* denc, const uint8_t* lo, int B, int T,
                       int C, hipStream_t s, float* ws, float* part) {
    if (part && lo && C % 8 == 0 && al16(denc) && ((uintptr_t)lo & 7) == 0 && ws) {
        const int bc = cdiv(B, PSG_CHUNKS), nch = cdiv(B, bc);
        const long long n = (long long)T * C;
        psg_part_k<<<dim3(cdiv(n / 8, 256), nch), 256, 0, s>>>(part, denc, lo, B, T, C, bc);
        psg_final_k<<<cdiv(n, 256), 256, 0, s>>>(dwpe, ws, part, n, nch);
        patch_small_grads_fin_k<<<cdiv(C, 256), 256, 0, s>>>(dcls, dpb, ws, T, C);
    } else {
        patch_small_grads_any(dcls, dwpe, dpb, denc, lo, B, T, C, s, ws);
    }
    after_launch("patch_small_grads");
}

}  // namespace vit

// ==================================================================== C ABI (fp32 reference ops)
using namespace vit;
extern "C" {

void residual_forward(float* out, const float* inp1, const float* inp2, int N) {
    if (N <= 0) return;
    residual_fwd_k<<<grid_for(N, 256), 256, 0, stream()>>>(out, inp1, inp2, N);
    after_launch("residual_forward");
}
void residual_backward(float* dinp1, float* dinp2, const float* dout, int N) {
    if (N <= 0) return;
    residual_bwd_k<<<grid_for(N, 256), 256, 0, stream()>>>(dinp1, dinp2, dout, N);
    after_launch("residual_backward");
}
void gelu_forward(float* out, const float* inp, int N) {
    if (N <= 0) return;
    gelu_fwd_k<<<grid_for(N, 256), 256, 0, stream()>>>(out, inp, N);
    after_launch("gelu_forward");
}
void gelu_backward(float* dinp, const float* inp, const float* dout, int N) {
    if (N <= 0) return;
    gelu_bwd_k<<<grid_for(N, 256), 256, 0, stream()>>>(dinp, inp, dout, N);
    after_launch("gelu_backward");
}
void matmul_forward(float* out, const float* inp, const float* weight, const float* bias, int B,
                    int T, int C, int OC) {
    GemmArgs a;
    a.A = inp; a.lda = C; a.a_kcontig = true;
    a.B = weight; a.ldb = C; a.b_kcontig = true;
    a.C = out; a.ldc = OC; a.bias = bias;
    a.M = B * T; a.N = OC; a.K = C; a.epi = EPI_F32_STORE;
    gemm_f32(a, stream());
}
void matmul_backward(float* dinp, float* dweight, float* dbias, const float* dout,
                     const float* inp, const float* weight, int B, int T, int C, int OC) {
    const int BT = B * T;
    if (dinp) {  // dinp[BT,C] += dout[BT,OC] . W[OC,C]
        GemmArgs a;
        a.A = dout; a.lda = OC; a.a_kcontig = true;
        a.B = weight; a.ldb = C; a.b_kcontig = false;
        a.C = dinp; a.ldc = C;
        a.M = BT; a.N = C; a.K = OC; a.epi = EPI_F32_ACC;
        gemm_f32(a, stream());
    }
    {  // dweight[OC,C] += dout^T . inp   (reduction over BT, split-K atomics when large)
        GemmArgs a;
        a.A = dout; a.lda = OC; a.a_kcontig = false;
        a.B = inp; a.ldb = C; a.b_kcontig = false;
        a.C = dweight; a.ldc = C;
        a.M = OC; a.N = C; a.K = BT;
        a.epi = (long long)BT > 4096 ? EPI_F32_ATOMIC : EPI_F32_ACC;
        gemm_f32(a, stream());
    }
    if (dbias) colsum_f32(dbias, dout, BT, OC, OC, stream());
}
void layernorm_forward(float* out, float* mean, float* rstd, const float* inp, const float* weight,
                       const float* bias, int B, int T, int C) {
    ln_forward_f32(out, mean, rstd, inp, weight, bias, (long long)B * T, C, stream());
}
void layernorm_backward(float* dinp, float* dweight, float* dbias, const float* dout,
                        const float* inp, const float* weight, const float* mean, const float* rstd,
                        int B, int T, int C) {
    ln_backward_f32(dinp, dweight, dbias, dout, inp, weight, mean, rstd, (long long)B * T, C,
                    stream());
}
void softmax_forward(float* probs, const float* logits, int B, int T, int V) {
    softmax_rows(probs, logits, (long long)B * T, V, stream());
}
void crossentropy_forward(float* losses, const float* probs, const int* targets, int B, int T,
                          int V) {
    ce_forward(losses, probs, targets, (long long)B * T, V, stream());
}
void crossentropy_softmax_backward(float* dlogits, const float* dlosses, const float* probs,
                                   const int* targets, int B, int T, int V) {
    ce_backward(dlogits, dlosses, probs, targets, (long long)B * T, V, stream());
}
void patch_embed_forward(float* encoded, const float* pixels, const float* patch_w,
                         const float* patch_b, const float* cls, const float* wpe, int B, int IMG,
                         int P, int C) {
    const int NP = (IMG / P) * (IMG / P), K = 3 * P * P;
    const size_t n_patch = (size_t)B * NP * K, n_emb = (size_t)B * NP * C;
    float* ws = (float*)workspace((n_patch + n_emb) * sizeof(float) + 256);
    if (!ws) return;
    float* patches = ws;
    float* emb = ws + ((n_patch + 63) & ~(size_t)63);
    hipStream_t s = stream();
    im2col_f32(patches, pixels, B, IMG, P, s);
    GemmArgs a;
    a.A = patches; a.lda = K; a.a_kcontig = true;
    a.B = patch_w; a.ldb = K; a.b_kcontig = true;
    a.C = emb; a.ldc = C; a.bias = patch_b;
    a.M = B * NP; a.N = C; a.K = K; a.epi = EPI_F32_STORE;
    gemm_f32(a, s);
    patch_assemble(encoded, emb, cls, wpe, B, NP, C, s);
}
void patch_embed_backward(float* dpatch_w, float* dpatch_b, float* dcls, float* dwpe,
                          const float* dencoded, const float* pixels, int B, int IMG, int P, int C) {
    const int NP = (IMG / P) * (IMG / P), K = 3 * P * P, T = NP + 1;
    const size_t n_patch = (size_t)B * NP * K, n_g = (size_t)B * NP * C;
    const size_t o_g = (n_patch + 63) & ~(size_t)63, o_t = (o_g + n_g + 63) & ~(size_t)63;
    float* ws = (float*)workspace((o_t + (size_t)T * C) * sizeof(float));
    if (!ws) return;
    float* patches = ws;
    float* g = ws + o_g;
    hipStream_t s = stream();
    im2col_f32(patches, pixels, B, IMG, P, s);
    patch_gather_f32(g, dencoded, B, NP, C, s);
    GemmArgs a;  // dpatch_w[C,K] += g^T . patches
    a.A = g; a.lda = C; a.a_kcontig = false;
    a.B = patches; a.ldb = K; a.b_kcontig = false;
    a.C = dpatch_w; a.ldc = K;
    a.M = C; a.N = K; a.K = B * NP;
    a.epi = (long long)B * NP > 4096 ? EPI_F32_ATOMIC : EPI_F32_ACC;
    gemm_f32(a, s);
    patch_small_grads(dcls, dwpe, dpatch_b, dencoded, B, T, C, s, ws + o_t);
}
void sgd_step(float* params, const float* grads, long long n, float lr) {
    sgd(params, grads, n, lr, stream());
}

// ---------------------------------------------------------------- bf16 extensions
void matmul_forward_bf16(uint16_t* out, const uint16_t* inp, const uint16_t* weight,
                         const float* bias, int B, int T, int C, int OC) {
    GemmArgs a;
    a.A = inp; a.lda = C; a.a_kcontig = true;
    a.B = weight; a.ldb = C; a.b_kcontig = true;
    a.C = out; a.ldc = OC; a.bias = bias;
    a.M = B * T; a.N = OC; a.K = C; a.epi = EPI_BF16_STORE;
    gemm_bf16(a, stream());
}
void matmul_backward_bf16(float* dinp, float* dweight, float* dbias, const uint16_t* dout,
                          const uint16_t* inp, const uint16_t* weight, int B, int T, int C, int OC) {
    const int BT = B * T;
    if (dinp) {
        GemmArgs a;
        a.A = dout; a.lda = OC; a.a_kcontig = true;
        a.B = weight; a.ldb = C; a.b_kcontig = false;
        a.C = dinp; a.ldc = C;
        a.M = BT; a.N = C; a.K = OC; a.epi = EPI_F32_ACC;
        gemm_bf16(a, stream());
    }
    {
        GemmArgs a;
        a.A = dout; a.lda = OC; a.a_kcontig = false;
        a.B = inp; a.ldb = C; a.b_kcontig = false;
        a.C = dweight; a.ldc = C;
        a.M = OC; a.N = C; a.K = BT; a.epi = EPI_F32_ATOMIC;
        a.dbias = dbias;  // fused column sum of dout
        gemm_bf16(a, stream());
    }
}
void layernorm_backward_bf16(float* dinp, float* dweight, float* dbias, const uint16_t* dout,
                             const float* inp, const float* weight, const float* mean,
                             const float* rstd, int B, int T, int C) {
    LnbIo io{};
    io.dinp = dinp; io.dweight = dweight; io.dbias = dbias;
    ln_backward_any<bf16_t, false>(io, (const bf16_t*)dout, inp, weight,
                    mean, rstd, (long long)B * T, C, stream());
}
void gelu_forward_bf16(uint16_t* out, const uint16_t* inp, int N) {
    if (N <= 0) return;
    gelu_fwd_bf16_k<<<grid_for(N, 256), 256, 0, stream()>>>(out, inp, N);
    after_launch("gelu_forward_bf16");
}
void gelu_backward_bf16(float* dinp, const uint16_t* inp, const uint16_t* dout, int N) {
    if (N <= 0) return;
    gelu_bwd_bf16_k<<<grid_for(N, 256), 256, 0, stream()>>>(dinp, inp, dout, N);
    after_launch("gelu_backward_bf16");
}
void layernorm_forward_bf16(uint16_t* out, float* mean, float* rstd, const float* inp,
                            const float* weight, const float* bias, int B, int T, int C) {
    ln_forward_bf16(out, mean, rstd, inp, weight, bias, (long long)B * T, C, stream());
}
void gemm_bf16_ex(void* C, long long ldc, const uint16_t* A, long long lda, int a_kcontig,
                  const uint16_t* B, long long ldb, int b_kcontig, const float* bias,
                  float* dbias, int M, int N, int K, int epi, int splitk) {
    VIT_REQUIRE(epi >= EPI_F32_STORE && epi <= EPI_BF16_STORE, "gemm_bf16_ex: epi %d", epi);
    GemmArgs a;
    a.A = A; a.lda = lda; a.a_kcontig = a_kcontig != 0;
    a.B = B; a.ldb = ldb; a.b_kcontig = b_kcontig != 0;
    a.C = C; a.ldc = ldc; a.bias = bias; a.dbias = dbias;
    a.M = M; a.N = N; a.K = K; a.epi = epi; a.splitk = splitk;
    gemm_bf16(a, stream());
}
void gemm_bf16_fused(void* C, void* C2, long long ldc, const void* aux, long long ldaux,
                     const uint16_t* A, long long lda, int a_kcontig, const uint16_t* B,
                     long long ldb, int b_kcontig, const float* bias, float* colsum_out, int M,
                     int N, int K, int epi) {
    VIT_REQUIRE(epi == EPI_BF16_GELU || epi == EPI_F32_RESID || epi == EPI_BF16_DGELU ||
                    epi == EPI_F32_STORE || epi == EPI_BF16_STORE || epi == EPI_BF16_GELU_D ||
                    epi == EPI_BF16_MUL,
                "gemm_bf16_fused: epi %d", epi);
    GemmArgs a;
    a.A = A; a.lda = lda; a.a_kcontig = a_kcontig != 0;
    a.B = B; a.ldb = ldb; a.b_kcontig = b_kcontig != 0;
    a.C = C; a.C2 = C2; a.ldc = ldc; a.aux = aux; a.ldaux = ldaux; a.bias = bias;
    a.colsum_out = colsum_out;
    a.M = M; a.N = N; a.K = K; a.epi = epi;
    gemm_bf16(a, stream());
}
void gemm_bf16_set_variant(int variant) { gemm_set_variant(variant); }
void gemm_bf16_set_debug(int flags) { gemm_set_debug(flags); }
void gemm_bf16_set_trace(unsigned long long* trace) { gemm_set_trace(trace); }
void convert_f32_to_bf16(uint16_t* out, const float* inp, long long n) {
    convert_f2bf(out, inp, n, stream());
}
void convert_bf16_to_f32(float* out, const uint16_t* inp, long long n) {
    if (n <= 0) return;
    bf2f_k<<<grid_for(n, 256), 256, 0, stream()>>>(out, inp, n);
    after_launch("convert_bf16_to_f32");
}

}  // extern "C"
