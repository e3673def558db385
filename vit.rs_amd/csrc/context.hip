// context.hip — per-thread stream / sticky error / workspace for the C ABI (include/vit_ops.h).
#include <cstdarg>
#include <cstdlib>
#include <atomic>
#include <cstring>

#include "common.h"
#include "../../include/vit_ops.h"

namespace vit {
namespace {
struct Ctx {
    hipStream_t stream = nullptr;
    int err = 0;
    char msg[512] = {0};
    void* ws = nullptr;
    size_t ws_bytes = 0;
};
thread_local Ctx g_ctx;
int g_sync_each = -1;
}  // namespace

void set_error(const char* fmt, ...) {
    if (g_ctx.err) return;  // keep the first error (sticky)
    g_ctx.err = 1;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_ctx.msg, sizeof(g_ctx.msg), fmt, ap);
    va_end(ap);
    if (getenv("VIT_VERBOSE")) fprintf(stderr, "[vit] error: %s\n", g_ctx.msg);
}
bool has_error() { return g_ctx.err != 0; }
hipStream_t stream() { return g_ctx.stream; }
bool sync_each_op() {
    if (g_sync_each < 0) {
        const char* e = getenv("VIT_SYNC");
        g_sync_each = (e && atoi(e) != 0) ? 1 : 0;
    }
    return g_sync_each == 1;
}
void* workspace(size_t bytes) {
    if (bytes > g_ctx.ws_bytes) {
        if (g_ctx.ws) {
            VIT_HIP(hipStreamSynchronize(g_ctx.stream));
            VIT_HIP(hipFree(g_ctx.ws));
        }
        g_ctx.ws = nullptr;
        g_ctx.ws_bytes = 0;
        size_t want = bytes + (bytes >> 2);
        if (hipMalloc(&g_ctx.ws, want) != hipSuccess) {
            set_error("workspace: hipMalloc(%zu) failed", want);
            return nullptr;
        }
        g_ctx.ws_bytes = want;
    }
    return g_ctx.ws;
}
// launch counters (vit_kernel_hits): which engine / kernel each call ran
static std::atomic<long long> g_hits[VIT_HIT_COUNT];
void count_hit(int k) {
    if (k >= 0 && k < VIT_HIT_COUNT) g_hits[k].fetch_add(1, std::memory_order_relaxed);
}
void after_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    if (sync_each_op()) {
        e = hipStreamSynchronize(g_ctx.stream);
        if (e != hipSuccess) set_error("%s: %s", what, hipGetErrorString(e));
    }
}
}  // namespace vit

extern "C" {
int vit_init(int device) {
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        vit::set_error("hipSetDevice(%d): %s", device, hipGetErrorString(e));
        return 1;
    }
    return 0;
}
void vit_set_stream(void* s) { vit::g_ctx.stream = (hipStream_t)s; }
void* vit_get_stream(void) { return (void*)vit::g_ctx.stream; }
int vit_sync(void) {
    hipError_t e = hipStreamSynchronize(vit::g_ctx.stream);
    if (e != hipSuccess) {
        vit::set_error("vit_sync: %s", hipGetErrorString(e));
        return 1;
    }
    return vit::g_ctx.err;
}
int vit_last_error(const char** msg) {
    if (msg) *msg = vit::g_ctx.msg;
    return vit::g_ctx.err;
}
void vit_clear_error(void) {
    vit::g_ctx.err = 0;
    vit::g_ctx.msg[0] = 0;
}
void* vit_malloc(size_t bytes) {
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e != hipSuccess) {
        vit::set_error("vit_malloc(%zu): %s", bytes, hipGetErrorString(e));
        return nullptr;
    }
    return p;
}
int vit_kernel_hits(long long* out, int n) {
    const int m = n < VIT_HIT_COUNT ? n : VIT_HIT_COUNT;
    for (int k = 0; k < m; k++) out[k] = vit::g_hits[k].load(std::memory_order_relaxed);
    return VIT_HIT_COUNT;
}
void vit_kernel_hits_reset(void) {
    for (auto& h : vit::g_hits) h.store(0, std::memory_order_relaxed);
}
void vit_free(void* p) {
    if (p) VIT_HIP(hipFree(p));
}
int vit_memcpy_h2d(void* dst, const void* src, size_t n) {
    hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, vit::g_ctx.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(vit::g_ctx.stream);
    if (e != hipSuccess) vit::set_error("vit_memcpy_h2d: %s", hipGetErrorString(e));
    return e != hipSuccess;
}
int vit_memcpy_d2h(void* dst, const void* src, size_t n) {
    hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, vit::g_ctx.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(vit::g_ctx.stream);
    if (e != hipSuccess) vit::set_error("vit_memcpy_d2h: %s", hipGetErrorString(e));
    return e != hipSuccess;
}
int vit_memcpy_d2d(void* dst, const void* src, size_t n) {
    hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, vit::g_ctx.stream);
    if (e != hipSuccess) vit::set_error("vit_memcpy_d2d: %s", hipGetErrorString(e));
    return e != hipSuccess;
}
int vit_memset(void* dst, int v, size_t n) {
    hipError_t e = hipMemsetAsync(dst, v, n, vit::g_ctx.stream);
    if (e != hipSuccess) vit::set_error("vit_memset: %s", hipGetErrorString(e));
    return e != hipSuccess;
}
void* vit_event_create(void) {
    hipEvent_t ev = nullptr;
    VIT_HIP(hipEventCreate(&ev));
    return (void*)ev;
}
void vit_event_destroy(void* ev) {
    if (ev) VIT_HIP(hipEventDestroy((hipEvent_t)ev));
}
int vit_event_record(void* ev) {
    hipError_t e = hipEventRecord((hipEvent_t)ev, vit::g_ctx.stream);
    if (e != hipSuccess) vit::set_error("vit_event_record: %s", hipGetErrorString(e));
    return e != hipSuccess;
}
float vit_event_elapsed_ms(void* a, void* b) {
    float ms = -1.f;
    hipError_t e = hipEventSynchronize((hipEvent_t)b);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, (hipEvent_t)a, (hipEvent_t)b);
    if (e != hipSuccess) vit::set_error("vit_event_elapsed_ms: %s", hipGetErrorString(e));
    return ms;
}
}  // extern "C"
