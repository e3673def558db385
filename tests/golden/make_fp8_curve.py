"""Records the fp8-mode loss curve fixture tests/golden/fp8_curve_test_h64.json (run on a GPU box;
the fp8 path has no reference counterpart, so this pins it against drift of its own numerics:
block-scale layout, rounding, operand routing).  Usage, from the repo root on the GPU box:
    python3 tests/golden/make_fp8_curve.py gpurun_out/fp8_curve_test_h64.json
then copy the file into tests/golden/.  The same recipe runs inside test_fp8_loss_curve_fixture."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def curve(v, steps=14):
    cfg = v.data.CONFIGS["test_h64"]
    params = v.data.init_params(cfg, "parity", seed=21)
    px, lab = v.data.synthetic_batch(cfg, 128, seed=22)
    m = v.ViT.build(cfg, 128, v.VIT_FP8, params=params)
    m.set_batch(px, lab)
    out = []
    for _ in range(steps):
        m.train_step(0.01)
        out.append(float(v.lib().vit_trainer_mean_loss(m.h)))
    m.close()
    return out


if __name__ == "__main__":
    from vitpkg import vit
    assert vit.lib().vit_init(0) == 0
    losses = curve(vit)
    json.dump({"config": "test_h64", "batch": 128, "precision": "fp8", "lr": 0.01, "seeds": [21, 22],
               "losses": losses}, open(sys.argv[1], "w"), indent=1)
    print(losses)
