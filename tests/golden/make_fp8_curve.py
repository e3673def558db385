"""Records the fp8-mode loss curve fixture tests/golden/fp8_curve_test_h64.json (run on a GPU box;
the fp8 path has no reference counterpart, so this pins it against drift of its own numerics:
block-scale layout, rounding, operand routing).  Usage, from the repo root on the GPU box:
    python3 tests/golden/make_fp8_curve.py gpurun_out/fp8_curve_test_h64.json
then copy the file into tests/golden/.  The same recipe runs inside test_fp8_loss_curve_fixture.

Re-record rule.  The fixture is a DRIFT ALARM, not a numerics gate: 14 chaotic SGD
steps amplify any rounding change anywhere in the step, so a change that is numerically sound (e.g. a
different summation order inside attention) can move the curve past its 2e-3 margin.  When
test_fp8_loss_curve_fixture fails, the fixture may be re-recorded only if, on the same build:
  1. every oracle-anchored gate passes: the fp8 error-model gates against the fp32 oracle
     (tests/parity.py fp8_limit in test_fp8_trainer_vs_oracle, test_production_fp8_step_vs_oracle,
     test_config5_fp8_shard_vs_oracle_two_images, test_h14_fp8_bench_shapes_all_gradients_vs_oracle) and
     the per-tensor rms baseline (parity.fp8_rms_gate, tests/golden/fp8_err_baseline.json);
  2. the bit-exact fp8 component tests pass (quantizers and fused MX epilogues against tests/mx.py,
     the fp8 GEMM against float64 numpy on the dequantized operands);
  3. the change that moved the curve is outside the fp8 path or is itself justified by a measurement,
     and the new file's "recorded" field names it.
A failure with any of 1-2 red is a regression to fix, not a fixture to re-record."""
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
               "recorded": sys.argv[2] if len(sys.argv) > 2 else "", "losses": losses},
              open(sys.argv[1], "w"), indent=1)
    print(losses)
