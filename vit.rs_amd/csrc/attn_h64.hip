// attn_h64.hip — fused MFMA attention instances for head size 64 (attn_fused.h), one
// translation unit per head size so the instances compile in parallel.
#include "attn_fused.h"

namespace vit {
VIT_FA_DEFINE(64)
}  // namespace vit
