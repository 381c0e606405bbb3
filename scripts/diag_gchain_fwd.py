"""Diagnostic: BatchNorm output of a fused genotype chain (gchain.hip) vs the unfused HIP path vs the
fp32 CPU oracle, plus the BN batch statistics, for one architecture and (param seed, batch seed, B)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from serann.engine import hip_engine as he  # noqa: E402
from serann.genome.interpreter import interpret  # noqa: E402
from serann.models import organism as om  # noqa: E402
from tests.archs import ARCHS  # noqa: E402
from tests.test_gpu_engine import _batch, _oracle, _rel  # noqa: E402


def node_out(eng, nid):
    mem = eng._debug_mem
    rec = mem["orgs"][0]
    kind, off = rec["act"][rec["owner"][nid]]
    n = eng.layouts[0].ir.node(nid)
    cnt = mem["B"] * int(np.prod(n.shape))
    return mem["act"].view(off, cnt).float().cpu().numpy().reshape(mem["B"], -1)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "gchain_f64_bn_dense"
    ir = interpret(ARCHS[name])
    last, (cid, did, bid) = next(iter(he.gchain_triples(ir).items()))
    for seed, bseed, B in ((5, 4, 80), (7, 0, 96)):
        params = om.init_params(ir, seed)
        x, g, y = _batch(B, seed=bseed)
        store = {}
        orig = om.Organism._bn

        def rec_bn(self, n, xin, training):
            out = orig(self, n, xin, training)
            store[n.id] = (xin.detach().reshape(xin.shape[0], -1).numpy(), out.detach().reshape(out.shape[0], -1).numpy())
            return out

        om.Organism._bn = rec_bn
        _oracle(ir, params, x, g, y)
        om.Organism._bn = orig
        xo, yo = store[bid]
        he.FUSE_GCHAIN = True
        fused = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
        fused.debug_train_step(x, g, y)
        he.FUSE_GCHAIN = False
        plain = he.HipPopulationEngine([ir], [0], device="cuda", params=[params])
        plain.debug_train_step(x, g, y)
        he.FUSE_GCHAIN = True
        yf, yp = node_out(fused, bid), node_out(plain, bid)
        xp = node_out(plain, did)
        C = ir.node(bid).attrs["channels"]
        xo_c = xo.reshape(-1, C)
        mu_o, var_o = xo_c.mean(0), xo_c.var(0)
        for tag, eng in (("fused", fused), ("plain", plain)):
            rec = eng._debug_mem["orgs"][0]["bn"][bid]
            f32 = eng._debug_mem["f32"]
            mu = f32.view(rec["mean"], C).cpu().numpy()
            istd = f32.view(rec["invstd"], C).cpu().numpy()
            var = 1.0 / istd ** 2 - 1e-3
            print(f"{name} s{seed} {tag}: mean rel {_rel(mu, mu_o):.2e} var rel {_rel(var, var_o):.2e}", flush=True)
        print(f"{name} s{seed}: BN out fused-oracle {_rel(yf, yo):.4f} plain-oracle {_rel(yp, yo):.4f} "
              f"fused-plain {_rel(yf, yp):.4f}; dense out plain-oracle {_rel(xp, xo):.4f}", flush=True)
        err = np.abs(yf - yo).reshape(-1, C)
        print("  worst channels (fused):", np.argsort(-err.max(0))[:5], err.max(0)[np.argsort(-err.max(0))[:5]])
        rows = np.abs(yf - yo).reshape(-1, C).max(1)
        print("  worst rows (fused):", np.argsort(-rows)[:8], rows[np.argsort(-rows)[:8]])


if __name__ == "__main__":
    main()
