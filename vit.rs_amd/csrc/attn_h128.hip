// attn_h128.hip — fused MFMA attention instances for head size 128 (attn_fused.h), one
// translation unit per head size so the instances compile in parallel.
#include "attn_fused.h"

namespace vit {
VIT_FA_DEFINE(128)
}  // namespace vit
