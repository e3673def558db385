// common.h — shared device helpers and the host-side error/stream context of libvit_hip.so.
// gfx950 (CDNA4) only: wave64, bf16 MFMA, ds_read_b64_tr_b16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>

#include "../../include/vit_ops.h"

typedef uint16_t bf16_t;  // raw bf16 bits in HBM
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// ds_read_b64_tr_b16 at LDS byte address a + OFF, issued as inline asm.  With the builtin
// (__builtin_amdgcn_ds_read_tr16_b64_v4bf16) hipcc (ROCm 7.2) puts `s_waitcnt vmcnt(0)` in front
// of the read whenever an LDS-DMA (global_load_lds) may be in flight, which drains the whole
// prefetch ring of a pipelined GEMM at every phase (plain ds_read_b128 loads do not get that
// wait).  The compiler does not count an asm read on lgkmcnt: callers must wait lgkmcnt(0) and
// fence with sched_barrier(0) before the first use of the result.
template <int OFF>
__device__ __forceinline__ bf16x4_t ds_read_tr16_asm(const void* lds) {
    bf16x4_t r;
    const uint32_t a = (uint32_t)(uintptr_t)LDS_PTR(const char, lds);
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
    return r;
}

// ---------------------------------------------------------------- host context
namespace vit {
// Sticky, thread-local error (the reference ops return () — train_vit.rs:376-670 — so errors
// are reported through vit_last_error()).
void set_error(const char* fmt, ...);
bool has_error();
hipStream_t stream();
bool sync_each_op();
void* workspace(size_t bytes);  // per-thread device scratch, grown on demand
void after_launch(const char* what);
void count_hit(int kind);  // VIT_HIT_* (include/vit_ops.h)
}  // namespace vit

#define VIT_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) vit::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call, \
                                             hipGetErrorString(e_));                   \
    } while (0)

#define VIT_REQUIRE(cond, ...)          \
    do {                                \
        if (!(cond)) {                  \
            vit::set_error(__VA_ARGS__); \
            return;                     \
        }                               \
    } while (0)

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
// one float2 -> bf16x2 conversion (v_cvt_pk_bf16_f32 a, b; RNE like f2bf).  The scalar form
// "f2bf(a) | f2bf(b) << 16" let hipcc pair the conversions of neighbouring calls its own way and
// then spend an and, a shift and an or_sdwa per pack putting the halves back
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    typedef float f2_t __attribute__((ext_vector_type(2)));
    typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2_t{a, b}, b2_t));
}

// "bf16 + lo8": a value t kept as hi = bf16(t) plus one signed byte q = rint((t - hi) / (ulp(hi) / 256)),
// t ~ hi + q * ulp(hi) / 256: a 16-bit significand in 3 bytes, with hi directly usable as a bf16
// GEMM operand.  ulp(hi)/256 = 2^(E - 142) for hi's biased exponent E (hi of magnitude < 2^-111
// keeps q = 0).
__device__ __forceinline__ float lo8_step(float hf) {
    const uint32_t e = (__float_as_uint(hf) >> 23) & 0xffu;
    return e > 15u ? __uint_as_float((e - 15u) << 23) : 0.f;
}
__device__ __forceinline__ float lo8_decode(float hf, uint32_t q8) {
    return hf + (float)(int)(int8_t)(uint8_t)q8 * lo8_step(hf);
}
__device__ __forceinline__ uint32_t lo8_encode(float t, float hf) {
    const uint32_t e = (__float_as_uint(hf) >> 23) & 0xffu;
    const float inv = (e > 15u && e < 255u) ? __uint_as_float((269u - e) << 23) : 0.f;
    const float q = fminf(fmaxf(rintf((t - hf) * inv), -127.f), 127.f);
    return (uint32_t)(uint8_t)(int8_t)(int)q;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// tanh-GELU (train_vit.rs:482-491) and its derivative with the D4 fix (sech^2 of the argument)
__device__ __forceinline__ float gelu_f(float x) {
    const float s = 0.7978845608028654f;
    float cube = 0.044715f * x * x * x;
    return 0.5f * x * (1.0f + tanhf(s * (x + cube)));
}
__device__ __forceinline__ float gelu_grad_f(float x) {
    const float s = 0.7978845608028654f;
    float cube = 0.044715f * x * x * x;
    float a = s * (x + cube);
    float th = tanhf(a);
    float sech2 = 1.0f - th * th;  // == 1/cosh^2(a)
    return 0.5f * (1.0f + th) + x * 0.5f * sech2 * s * (1.0f + 3.0f * 0.044715f * x * x);
}

// The same two functions in the logistic form used by the bf16 GEMM epilogues, where they run
// on every element of a 256x256 output tile per CU and tanhf (a long libm sequence) made the
// fc / fcproj-dgrad epilogues VALU-bound:  0.5(1 + tanh a) = sigmoid(2a), 1 - tanh^2 a =
// 4 sigmoid(2a)(1 - sigmoid(2a)).  One v_exp + one v_rcp per element; |error| <~ 1e-7
// absolute against the tanh form, far below the bf16 rounding of the stored value.
// bf16-epilogue forms: x * sigmoid(2a) with a = sqrt(2/pi)(x + 0.044715 x^3) (= 0.5 x (1 + tanh a)),
// on the raw v_exp_f32 (2^x) and v_rcp_f32 (1 ulp) instructions.  __expf / __frcp_rn wrapped them
// in range-reduction and correctly-rounded refinement sequences (~12 VALU per element, the bulk of
// the GELU / GELU' epilogues); the results are rounded to bf16, so 1-ulp fp32 terms do not show.
// x -> -inf: exp2 -> inf, rcp -> 0, product -> -0; x -> +inf: sigmoid -> 1.
// (r04) The tanh argument in Horner form: z = k (x + c x^3) = x * fma(k c, x^2, k), and the
// derivative as sg + [x sg (1 - sg)] * [2 s (1 + 3 c x^2)] = fma(fma(-g, sg, g), w, sg) with
// g = x sg: 8 VALU + 2 transcendentals per element for the pair (was 11 + 2).  The fc forward's
// GELU-pair epilogue is vector-issue bound, so the count is its cost.
constexpr float GELU_K = -2.0f * 0.7978845608028654f * 1.4426950408889634f;  // -2 sqrt(2/pi) log2(e)
constexpr float GELU_KC = GELU_K * 0.044715f;
constexpr float GELU_W0 = 2.0f * 0.7978845608028654f;                       // 2 s
constexpr float GELU_W2 = 2.0f * 0.7978845608028654f * 3.0f * 0.044715f;    // 2 s 3 c
__device__ __forceinline__ float gelu_sigmoid_f(float x, float x2) {       // 0.5 (1 + tanh a)
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * fmaf(GELU_KC, x2, GELU_K)));
}
__device__ __forceinline__ float gelu_fast_f(float x) {
    return x * gelu_sigmoid_f(x, x * x);
}
// derivative with sech^2 of the tanh argument (D4): sg + 2 s x sg (1 - sg) (1 + 3 * 0.044715 x^2)
__device__ __forceinline__ float gelu_grad_fast_f(float x) {
    const float x2 = x * x;
    const float sg = gelu_sigmoid_f(x, x2);
    const float g = x * sg;
    return fmaf(fmaf(-g, sg, g), fmaf(GELU_W2, x2, GELU_W0), sg);
}

// gelu_fast_f(x) and gelu_grad_fast_f(x) from one sigmoid (bit-identical to the two calls)
__device__ __forceinline__ void gelu_pair_fast_f(float x, float& g, float& d) {
    const float x2 = x * x;
    const float sg = gelu_sigmoid_f(x, x2);
    g = x * sg;
    d = fmaf(fmaf(-g, sg, g), fmaf(GELU_W2, x2, GELU_W0), sg);
}

// optimizer_step (train_vit.rs:740): p -= lr*g with two roundings like the Rust reference
// (no FMA contraction), so the fp32 update is bit-exact.
__device__ __forceinline__ float sgd_update(float p, float g, float lr) {
#pragma clang fp contract(off)
    return p - lr * g;
}

// AdamW (oracle ref_adamw_step): one element, every operation rounded like the
// oracle's line-by-line C (no contraction, correctly rounded sqrt / divide).  omb1 = 1-beta1, omb2 = 1-beta2,
// bc1/bc2 = the bias corrections 1 - beta^t, computed on the host exactly as the oracle does.
__device__ __forceinline__ float adamw_update(float p, float g, float& m, float& v, float lr,
                                              float b1, float b2, float omb1, float omb2,
                                              float bc1, float bc2, float eps, float wd) {
#pragma clang fp contract(off)
    const float mi = b1 * m + omb1 * g;
    const float vi = b2 * v + omb2 * g * g;
    m = mi;
    v = vi;
    // '/' and __builtin_sqrtf are IEEE-rounded under hipcc's default
    // -fhip-fp32-correctly-rounded-divide-sqrt; __fsqrt_rn is NOT (it maps to the native,
    // approximate v_sqrt unless OCML_BASIC_ROUNDED_OPERATIONS is defined)
    const float mh = mi / bc1, vh = vi / bc2;
    return p - lr * (mh / (__builtin_sqrtf(vh) + eps) + wd * p);
}

// XCD-aware bijective remap of a linear workgroup id (cdna_hip_programming.md §5, "XCD swizzle
// must be bijective"): blocks dealt round-robin over 8 XCDs get contiguous tile ranges per XCD.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

__host__ __device__ static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
