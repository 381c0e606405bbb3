"""Planner side of the fp32 bias gradient of a Dense(units=1) subtracted from a BatchNormalization input
(x = a - Dense(..), the mutant form of tests/archs.py mutant_bn_axis_bsub): the BN backward (phase 5) takes
-sum(dx) into that Dense's bias (BnDesc pdb, flags 128) and the Dense's WGRAD skips its bias.  Built on the CPU
without launching anything; tests/test_gpu_engine.py checks the numbers against the fp32 oracle."""
import numpy as np

from .archs import ARCHS
from serann.genome.interpreter import interpret


def test_sub_dense_bias_from_bn_backward():
    from serann.engine.hip_engine import HipPopulationEngine
    from serann.ops import hip_ops as H
    ir = interpret(ARCHS["mutant_bn_axis_bsub"])
    eng = HipPopulationEngine([ir], [0], device="cpu")
    mem = eng._alloc_buffers(96, with_grads=True)
    pl = eng._build_plan("train", 96, mem, [{"X": 0, "g": 0}], 0, [0], None, adam_ctx=1)
    lay = eng.layouts[0]
    dense1 = next(n.id for n in ir.nodes if n.op == "gemm" and n.attrs["kind"] == "dense" and n.attrs["f"] == 1)
    bias_ptr = eng.g.data_ptr() + 8 * lay.b[dense1]
    bn5 = [r for la in pl.launches if la.kind == "bn" and la.arg == 5
           for r in np.frombuffer(la.descs.numpy().tobytes(), dtype=H.BN_DTYPE)]
    hits = [r for r in bn5 if int(r["pdb"]) == bias_ptr]
    assert len(hits) == 1 and int(hits[0]["flags"]) & 128, bn5
    wg = [r for la in pl.launches if la.kind == "gemm3" and la.arg[0] == H.MODE_WGRAD
          for r in np.frombuffer(la.descs.numpy().tobytes(), dtype=H.GEMM_DTYPE)]
    w_dense1 = [r for r in wg if int(r["out"]) == eng.g.data_ptr() + 8 * lay.w[dense1]]
    assert len(w_dense1) == 1 and int(w_dense1[0]["bias"]) == 0
