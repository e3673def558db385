// attn_h32.hip — fused MFMA attention instances for head size 32 (attn_fused.h), one
// translation unit per head size so the instances compile in parallel.
#include "attn_fused.h"

namespace vit {
VIT_FA_DEFINE(32)
}  // namespace vit
