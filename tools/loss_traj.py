"""Print the loss trajectory of test_training_reduces_loss's setup for both precisions."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vitpkg import vit
assert vit.lib().vit_init(0) == 0
cfg = vit.data.CONFIGS["test_h64"]
params = vit.data.init_params(cfg, "parity", seed=1)
px, lab = vit.data.synthetic_batch(cfg, 8, seed=2)
lr = float(sys.argv[1]) if len(sys.argv) > 1 else 0.5
for prec in (vit.VIT_FP32, vit.VIT_BF16):
    m = vit.ViT.build(cfg, 8, prec, params=params)
    m.set_batch(px, lab)
    losses = []
    for _ in range(40):
        m.train_step(lr)
        losses.append(round(float(vit.lib().vit_trainer_mean_loss(m.h)), 3))
    print(os.environ.get("VIT_LIB", "new"), "lr", lr, "prec", prec, losses, flush=True)
    m.close()
