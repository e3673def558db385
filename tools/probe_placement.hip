// probe_placement.hip — which CU each workgroup of a 2-workgroups-per-CU launch lands on (the
// LDS size of the g4 GEMM engine, 72 KiB, caps residency at 2 per CU), from HW_ID / XCC_ID.
// Prints, for the first 1024 workgroups, how many distinct CUs the first 256 / 512 fill and
// whether workgroup pairs (b, b+256), (b, b+1), (b, b+8) share a CU.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <vector>

__global__ __launch_bounds__(256) void where_k(int* out, int spin) {
    __shared__ char big[72 * 1024];
    if (threadIdx.x == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
        const int cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        out[blockIdx.x] = (((int)(xcc & 15) * 8 + se) * 2 + sh) * 16 + cu;
        big[0] = (char)cu;
    }
    // hold the CU so later workgroups cannot reuse the slot
    for (int k = 0; k < spin; k++) __builtin_amdgcn_s_sleep(127);
    if (big[0] == 99) out[0] = -1;
}

int main() {
    const int n = 1024;
    int* d;
    (void)hipMalloc(&d, n * 4);
    where_k<<<n, 256>>>(d, 200);
    std::vector<int> h(n);
    (void)hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    std::map<int, std::vector<int>> by;
    for (int b = 0; b < n; b++) by[h[b]].push_back(b);
    auto distinct = [&](int lo, int hi) {
        std::map<int, int> c;
        for (int b = lo; b < hi; b++) c[h[b]]++;
        return (int)c.size();
    };
    printf("distinct CUs: first 256 wgs %d, first 512 %d, all %d\n", distinct(0, 256), distinct(0, 512),
           distinct(0, n));
    int s256 = 0, s1 = 0, s8 = 0;
    for (int b = 0; b < 256; b++) {
        s256 += h[b] == h[b + 256];
        s1 += h[b] == h[b ^ 1];
        s8 += h[b] == h[b + 8];
    }
    printf("pairs sharing a CU (of 256): (b, b+256) %d, (b, b^1) %d, (b, b+8) %d\n", s256, s1, s8);
    printf("first 16 CUs of workgroups 0..31:");
    for (int b = 0; b < 32; b++) printf(" %d", h[b]);
    printf("\nworkgroups on the CU of wg 0:");
    for (int b : by[h[0]]) printf(" %d", b);
    printf("\n");
    return 0;
}
