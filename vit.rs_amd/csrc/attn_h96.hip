// attn_h96.hip — fused MFMA attention instances for head size 96 (attn_fused.h), one
// translation unit per head size so the instances compile in parallel.
#include "attn_fused.h"

namespace vit {
VIT_FA_DEFINE(96)
}  // namespace vit
