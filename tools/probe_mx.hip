// probe_mx.hip — pins, on the GPU, the operand / scale lane layout of
// v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3 operands, E8M0 block scales) and the rounding of
// v_cvt_pk_fp8_f32, against host references.  Build: hipcc --offload-arch=gfx950 -O2 probe_mx.hip
// Measured on MI355X (ROCm 7.2): data layout c=16 with scale map 0 matches exactly (max abs err 0):
//   lane l (i = l&15, g = l>>4) holds A[i][16g + j] in bytes j = 0..15 and A[i][64 + 16g + j - 16]
//   in bytes j = 16..31 (B likewise with the column on i); lane l's scale byte (opsel 0) scales
//   row/column i, k-block (32 deep) g; C/D: col = l&15, row = 4*(l>>4) + r.
// v_mfma_scale_f32_32x32x64_f8f6f4 (measured): lane l (r = l&31, h = l>>5) carries k-block 0 in
//   bytes 0..15 and k-block 1 in bytes 16..31 (layouts c=8 and c=16 both match: the hardware pairs
//   A and B bytes slot for slot, so only block membership is observable); the gemm uses c=16:
//   bytes 0..15 = k [16h, 16h+16), bytes 16..31 = k [32+16h, 32+16h+16); lane l's scale byte
//   scales row/column r, k-block h; C/D: col = l&31, row = (reg&3) + 8*(reg>>2) + 4*(l>>5).
// v_cvt_pk_fp8_f32 is OCP e4m3fn with round-to-nearest-even and NO saturation (500 -> NaN), so
// the quantizers must bound |x| <= 448 before converting.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

// OCP e4m3fn decode (bias 7, no inf, 0x7f/0xff NaN)
static float e4m3_to_f(unsigned char b) {
    const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
    float v;
    if (e == 15 && m == 7) return NAN;
    if (e == 0) v = ldexpf((float)m, -9);
    else v = ldexpf(1.0f + m / 8.0f, e - 7);
    return s ? -v : v;
}

// operands gathered through host-computed maps: lane l, byte j <- A[amap[l*32+j]] (index m*128+k),
// B[bmap[l*32+j]] (index k*16+n); lane l's scale bytes sa[samap[l]], sb[sbmap[l]]
__global__ void mma_k(float* out, const unsigned char* A, const unsigned char* B, const unsigned char* sa,
                      const unsigned char* sb, const int* amap, const int* bmap, const int* samap,
                      const int* sbmap) {
    const int l = threadIdx.x;
    v8i a, b;
    unsigned char* pa = (unsigned char*)&a;
    unsigned char* pb = (unsigned char*)&b;
    for (int j = 0; j < 32; j++) {
        pa[j] = A[amap[l * 32 + j]];
        pb[j] = B[bmap[l * 32 + j]];
    }
    const int scale_a = sa[samap[l]];
    const int scale_b = sb[sbmap[l]];
    v4f c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, scale_a, 0, scale_b);
    for (int r = 0; r < 4; r++) out[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

typedef float v16f __attribute__((ext_vector_type(16)));
// v_mfma_scale_f32_32x32x64_f8f6f4: A [32][64], B [64][32], maps as mma_k
__global__ void mma32_k(float* out, const unsigned char* A, const unsigned char* B, const unsigned char* sa,
                        const unsigned char* sb, const int* amap, const int* bmap, const int* samap,
                        const int* sbmap) {
    const int l = threadIdx.x;
    v8i a, b;
    unsigned char* pa = (unsigned char*)&a;
    unsigned char* pb = (unsigned char*)&b;
    for (int j = 0; j < 32; j++) {
        pa[j] = A[amap[l * 32 + j]];
        pb[j] = B[bmap[l * 32 + j]];
    }
    v16f c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa[samap[l]], 0, sb[sbmap[l]]);
    for (int r = 0; r < 16; r++) out[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}

static double run32(const unsigned char* hA, const unsigned char* hB, const unsigned char* hsa,
                    const unsigned char* hsb, int c) {
    // k = c*h + (j % c) + 2c*(j / c), h = l>>5; scale lane l -> (row l&31, block l>>5)
    int amap[2048], bmap[2048], samap[64], sbmap[64];
    for (int l = 0; l < 64; l++) {
        for (int j = 0; j < 32; j++) {
            const int k = c * (l >> 5) + (j % c) + 2 * c * (j / c);
            amap[l * 32 + j] = (l & 31) * 64 + k;
            bmap[l * 32 + j] = k * 32 + (l & 31);
        }
        samap[l] = (l & 31) * 2 + (l >> 5);
        sbmap[l] = samap[l];
    }
    unsigned char *dA, *dB, *dsa, *dsb;
    int *dam, *dbm, *dsam, *dsbm;
    float* dC;
    (void)hipMalloc(&dA, 2048); (void)hipMalloc(&dB, 2048); (void)hipMalloc(&dsa, 64); (void)hipMalloc(&dsb, 64);
    (void)hipMalloc(&dam, 8192); (void)hipMalloc(&dbm, 8192); (void)hipMalloc(&dsam, 256); (void)hipMalloc(&dsbm, 256);
    (void)hipMalloc(&dC, 4096);
    (void)hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsa, hsa, 64, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsb, hsb, 64, hipMemcpyHostToDevice);
    (void)hipMemcpy(dam, amap, 8192, hipMemcpyHostToDevice);
    (void)hipMemcpy(dbm, bmap, 8192, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsam, samap, 256, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsbm, sbmap, 256, hipMemcpyHostToDevice);
    mma32_k<<<1, 64>>>(dC, dA, dB, dsa, dsb, dam, dbm, dsam, dsbm);
    float hC[1024];
    (void)hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    double maxerr = 0;
    for (int m = 0; m < 32; m++)
        for (int n = 0; n < 32; n++) {
            double ref = 0;
            for (int k = 0; k < 64; k++)
                ref += (double)e4m3_to_f(hA[m * 64 + k]) * ldexp(1.0, hsa[m * 2 + k / 32] - 127) *
                       (double)e4m3_to_f(hB[k * 32 + n]) * ldexp(1.0, hsb[n * 2 + k / 32] - 127);
            maxerr = fmax(maxerr, fabs(ref - hC[m * 32 + n]));
        }
    return maxerr;
}

__global__ void cvt_k(unsigned int* out, const float* in, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * i + 1 >= n) return;
    out[i] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(in[2 * i], in[2 * i + 1], 0, false) & 0xffffu;
}

static double run(const unsigned char* hA, const unsigned char* hB, const unsigned char* hsa,
                  const unsigned char* hsb, int c, int shyp) {
    // data hypothesis c: k = c*(l>>4) + (j % c) + 4c*(j / c); scale hypothesis 0: lane l -> (row l&15,
    // block l>>4); 1: lane l -> (row l&15, block (l>>4)) with blocks of the data's own k (c=32 only)
    int amap[2048], bmap[2048], samap[64], sbmap[64];
    for (int l = 0; l < 64; l++) {
        for (int j = 0; j < 32; j++) {
            const int k = c * (l >> 4) + (j % c) + 4 * c * (j / c);
            amap[l * 32 + j] = (l & 15) * 128 + k;
            bmap[l * 32 + j] = k * 16 + (l & 15);
        }
        samap[l] = shyp == 0 ? (l & 15) * 4 + (l >> 4) : (l >> 2) * 4 + (l & 3);
        sbmap[l] = samap[l];
    }
    static unsigned char *dA, *dB, *dsa, *dsb;
    static int *dam, *dbm, *dsam, *dsbm;
    static float* dC;
    if (!dA) {
        (void)hipMalloc(&dA, 2048); (void)hipMalloc(&dB, 2048); (void)hipMalloc(&dsa, 64); (void)hipMalloc(&dsb, 64);
        (void)hipMalloc(&dam, 8192); (void)hipMalloc(&dbm, 8192); (void)hipMalloc(&dsam, 256); (void)hipMalloc(&dsbm, 256);
        (void)hipMalloc(&dC, 1024);
    }
    (void)hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsa, hsa, 64, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsb, hsb, 64, hipMemcpyHostToDevice);
    (void)hipMemcpy(dam, amap, 8192, hipMemcpyHostToDevice);
    (void)hipMemcpy(dbm, bmap, 8192, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsam, samap, 256, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsbm, sbmap, 256, hipMemcpyHostToDevice);
    mma_k<<<1, 64>>>(dC, dA, dB, dsa, dsb, dam, dbm, dsam, dsbm);
    float hC[256];
    (void)hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    double maxerr = 0;
    for (int m = 0; m < 16; m++)
        for (int n = 0; n < 16; n++) {
            double ref = 0;
            for (int k = 0; k < 128; k++)
                ref += (double)e4m3_to_f(hA[m * 128 + k]) * ldexp(1.0, hsa[m * 4 + k / 32] - 127) *
                       (double)e4m3_to_f(hB[k * 16 + n]) * ldexp(1.0, hsb[n * 4 + k / 32] - 127);
            maxerr = fmax(maxerr, fabs(ref - hC[m * 16 + n]));
        }
    return maxerr;
}

int main() {
    srand(7);
    unsigned char hA[16 * 128], hB[128 * 16], hsa[64], hsb[64], one[64];
    const unsigned char vals[7] = {0x00, 0x38, 0xb8, 0x40, 0xc0, 0x44, 0x30};  // 0, 1, -1, 2, -2, 3, 0.5
    for (auto& x : hA) x = vals[rand() % 7];
    for (auto& x : hB) x = vals[rand() % 7];
    for (auto& x : hsa) x = 125 + rand() % 5;  // 2^-2 .. 2^2
    for (auto& x : hsb) x = 125 + rand() % 5;
    for (auto& x : one) x = 127;
    for (int c : {8, 16, 32})
        printf("unit scales, data layout c=%d: max abs err %.4g\n", c, run(hA, hB, one, one, c, 0));
    for (int c : {8, 16, 32})
        for (int sh : {0, 1})
            printf("random scales, c=%d, scale map %d: max abs err %.4g\n", c, sh, run(hA, hB, hsa, hsb, c, sh));

    for (int c : {8, 16, 32})
        printf("32x32x64: random scales, data layout c=%d: max abs err %.4g\n", c, run32(hA, hB, hsa, hsb, c));

    // conversion: every representable value, midpoints (ties), and overflow
    const int N = 4096;
    float hin[N];
    int n = 0;
    for (int b = 0; b < 256 && n < N; b++) {
        const float v = e4m3_to_f((unsigned char)b);
        if (std::isnan(v)) continue;
        hin[n++] = v;
        const float w = e4m3_to_f((unsigned char)(b + 1));
        if ((b & 0x7f) < 0x7e && !std::isnan(w)) hin[n++] = 0.5f * (v + w);  // tie
    }
    hin[n++] = 448.f; hin[n++] = 464.f; hin[n++] = 500.f; hin[n++] = 1e6f; hin[n++] = -1e6f;
    hin[n++] = 1e-4f; hin[n++] = 1e-3f;
    if (n & 1) hin[n++] = 0.f;
    float* din;
    unsigned* dout;
    hipMalloc(&din, n * 4); hipMalloc(&dout, n * 2);
    hipMemcpy(din, hin, n * 4, hipMemcpyHostToDevice);
    cvt_k<<<(n / 2 + 255) / 256, 256>>>(dout, din, n);
    unsigned hout[N / 2];
    hipMemcpy(hout, dout, n * 2, hipMemcpyDeviceToHost);
    int exact = 0, rne_ok = 0, ties = 0;
    for (int i = 0; i < n; i++) {
        const unsigned char q = (hout[i / 2] >> (8 * (i & 1))) & 0xff;
        const float back = e4m3_to_f(q);
        if (back == hin[i]) exact++;
        // ties: RNE picks the even mantissa
        if (i < n - 8 && !(back == hin[i])) {
            ties++;
            if ((q & 1) == 0 && fabsf(back - hin[i]) <= fabsf(hin[i]) * 0.07f) rne_ok++;
        }
    }
    printf("cvt_pk_fp8_f32: %d values, %d exact, %d ties (%d rounded to even mantissa)\n", n, exact, ties, rne_ok);
    for (int i = n - 8; i < n; i++) {
        const unsigned char q = (hout[i / 2] >> (8 * (i & 1))) & 0xff;
        printf("  %g -> 0x%02x (%g)\n", hin[i], q, e4m3_to_f(q));
    }
    return 0;
}
