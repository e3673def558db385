// probe_store.hip — epilogue store throughput: G workgroups (512 threads, one per CU) each write
// R rounds of a 256x256 bf16 tile (128 KiB) in the GEMM epilogue's pattern (16-B stores, 8 rows x
// 128 B per wave instruction) into disjoint regions.  Time vs G separates a per-CU store-issue
// limit (time flat in G) from a chip-wide HBM-write limit (time grows with G).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512) void store_k(uint4* out, int rounds, long long ld16, int contig) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint4 v = make_uint4(tid, blockIdx.x, 7, 9);
    for (int r = 0; r < rounds; r++) {
        // tile (blockIdx, r): rows [256*(b*rounds + r), +256), 256 bf16 = 32 x 16-B per row
        const long long row0 = 256LL * ((long long)blockIdx.x * rounds + r);
        if (contig) {  // each wave instruction: 1 KiB contiguous (2 rows of the 512-B row... 64 lanes)
            for (int it = 0; it < 16; it++) {
                const long long idx = (row0 * 32) + ((long long)(it * 8 + w) * 64 + lane);
                out[idx] = v;
            }
        } else {  // GEMM staged-epilogue pattern: wave w owns rows 128*(w>>2)..+127, cols 64*(w&3)..+63
            const int rr = lane >> 3, cc = lane & 7;  // 8 rows x 8 lanes (128 B) per instruction
            for (int pass = 0; pass < 2; pass++)
                for (int it = 0; it < 8; it++) {
                    const long long row = row0 + 128 * (w >> 2) + 64 * pass + it * 8 + rr;
                    out[row * ld16 + (w & 3) * 8 + cc] = v;
                }
        }
    }
}

int main() {
    const int rounds = 8;
    const long long ld16 = 32;  // 256 bf16 per row = 32 x 16 B
    const long long maxg = 256;
    const size_t bytes = maxg * rounds * 256 * 512ULL;
    uint4* d;
    if (hipMalloc(&d, bytes) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int contig = 0; contig < 2; contig++)
        for (int g : {16, 32, 64, 128, 256}) {
            store_k<<<g, 512>>>(d, rounds, ld16, contig);
            hipDeviceSynchronize();
            hipEventRecord(e0);
            for (int k = 0; k < 5; k++) store_k<<<g, 512>>>(d, rounds, ld16, contig);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= 5;
            const double mb = (double)g * rounds * 128 * 1024 / 1e6;
            printf("%s G=%3d: %8.1f us  %7.1f MB  %6.2f TB/s  per-CU %5.1f GB/s\n", contig ? "contig " : "epilogue",
                   g, ms * 1e3, mb, mb / ms / 1e6 * 1e3 / 1e3, mb / ms / g);
        }
    return 0;
}
