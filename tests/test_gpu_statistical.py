"""End-to-end statistical parity of the HIP engine with the fp32 torch engine on generator organisms
(SURVEY §7.4): 16 organisms drawn from the synthetic generator (genome/generator.py, the reference's
synthetic_serann_generator), the same initial weights, one epoch on synthetic MNIST at the production
batch (750).  bf16 operands make the two trajectories diverge step by step, so the test compares what
the evolution loop consumes -- the per-organism validation accuracy and replication MSE
(reference experiment_worker.py:66-128) -- not the weights."""
import numpy as np
import pytest

from serann.genome.generator import generate
from serann.genome.interpreter import interpret
from serann.models.organism import init_params

pytestmark = pytest.mark.gpu


def test_generator_population_matches_fp32_torch_engine():
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import HipPopulationEngine
    from serann.engine.torch_engine import TorchPopulationEngine
    # (no class blending / label noise: the converged organisms below must reach 0.95 in one epoch)
    data = get_serann_data(synthetic_encodings(), synthetic_mnist(n_train=15000, n_test=1000, seed=17, label_noise=0.0,
                                                                  mix=0.0),
                           n_train=15000, n_test=1000)
    df = generate(16, seed=2024, validation_genotype_size=100)
    irs = [interpret(code) for code in df["code"]]
    seeds = list(range(100, 116))
    cfg = TrainConfig(epochs=1, batch_size=750)
    # fp32 oracle on the CPU (~45 s): independent of the GPU library paths
    ref = TorchPopulationEngine(irs, seeds, device="cpu", cfg=cfg)
    rr = ref.fit(data, cfg)
    hip = HipPopulationEngine(irs, seeds, device="cuda", cfg=cfg,
                              params=[init_params(ir, s) for ir, s in zip(irs, seeds)])
    rh = hip.fit(data, cfg)
    hip.close()
    assert rh.steps == rr.steps == 19
    d_acc = np.abs(rh.val_acc - rr.val_acc)
    r_mse = np.abs(rh.val_mse - rr.val_mse) / np.maximum(rr.val_mse, 1e-6)
    table = "\n".join(f"{i:2d} acc {a:.4f} vs {b:.4f}  mse {c:.5f} vs {d:.5f}"
                      for i, (a, b, c, d) in enumerate(zip(rh.val_acc, rr.val_acc, rh.val_mse, rr.val_mse)))
    print(table)
    assert np.all(np.isfinite(rh.val_acc)) and np.all(np.isfinite(rh.val_mse)), table
    # organisms still in the middle of their learning curve after one epoch (fp32 val_acc < 0.95)
    # follow chaotic trajectories under any change of rounding; the converged ones must agree per
    # organism, the population on average
    done = rr.val_acc >= 0.95
    assert done.sum() >= 8, table
    assert np.all(d_acc[done] <= 0.02), table
    assert abs(rh.val_acc.mean() - rr.val_acc.mean()) <= 0.05, table
    assert np.all(r_mse <= 0.10), table
