// attn_h64.hip — fused MFMA attention instances for head size 64 (attn_fused.h), one
// translation unit per head size so the instances compile in parallel.
#include "attn_fused.h"

namespace vit {
VIT_FA_DEFINE(64)
}  // namespace vit

#if VIT_ATTN_DIAG & 4
extern "C" int vit_attn_trace_read_h64(void* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(vit::fa::attn_trace), sizeof(vit::fa::attn_trace));
}
#endif
