"""Debug: BatchNormalization on the raw image (bn_first_and_pool3, node 2) -- its output gradient dy
(written by the conv DGRAD) and the beta / gamma gradients, HIP engine vs fp32 torch, at B=750."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from serann.engine.hip_engine import HipPopulationEngine  # noqa: E402
from serann.genome.interpreter import interpret  # noqa: E402
from serann.models.organism import Organism, init_params  # noqa: E402
from tests.archs import ARCHS  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "bn_first_and_pool3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 750
ir = interpret(ARCHS[name])
params = init_params(ir, 7)
rng = np.random.default_rng(2)
x = rng.random((B, 28, 28, 1)).astype(np.float32)
g = rng.integers(0, 2, (B, 100)).astype(np.float32)
y = rng.integers(0, 10, B).astype(np.int64)
eng = HipPopulationEngine([ir], [0], device="cuda", params=[params])
grads, _ = eng.debug_train_step(x, g, y)
mem = eng._debug_mem
rec = mem["orgs"][0]
bn = [n for n in ir.nodes if n.op == "bn"][0]
n = B * int(np.prod(bn.shape))
off = (mem["grad"].ptr(rec["grad"][bn.id]) - mem["grad"].t.data_ptr()) // 2
dy_h = mem["grad"].t.narrow(0, off, n).float().cpu().numpy()

org = Organism(ir, params, device="cpu")
vals = {}
orig_bn = org._bn


def hook(nn_, xin, training):
    out = orig_bn(nn_, xin, training)
    if nn_.id == bn.id:
        out.retain_grad()
        vals["y"] = out
    return out


org._bn = hook
cl, rl = org(torch.as_tensor(x), torch.as_tensor(g)[..., None], training=True)
lb = ir.loss_balance
loss = lb * F.cross_entropy(cl, torch.as_tensor(y)) + (1 - lb) * ((torch.sigmoid(rl) - torch.as_tensor(g)) ** 2).mean()
loss.backward()
dy_t = vals["y"].grad.detach().numpy().reshape(-1)
print("dy rel err", np.linalg.norm(dy_h - dy_t) / np.linalg.norm(dy_t))
print("sum dy: hip", dy_h.astype(np.float64).sum(), "torch", dy_t.astype(np.float64).sum(),
      "sum |dy|", np.abs(dy_t).sum())
hg = eng.export_arena(0, grads)
tg = {k: v.grad.numpy() for k, v in org.params.items()}
print("beta hip", hg[bn.id].get("beta"), "torch", tg.get(f"n{bn.id}_beta"))
print("gamma hip", hg[bn.id].get("gamma"), "torch", tg.get(f"n{bn.id}_gamma"))
xs = torch.as_tensor(x).reshape(-1).double()
xh = ((xs - xs.mean()) / torch.sqrt(xs.var(unbiased=False) + 1e-3)).numpy()
print("sum dy*xhat: hip-dy", (dy_h * xh).sum(), "torch-dy", (dy_t * xh).sum())
