"""Gradient of every parameter of one test architecture: HIP engine vs fp32 CPU oracle vs torch bf16 (norms,
relative errors, first values) -- to localise a gradient that misses the bf16-relative criterion."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from serann.engine.hip_engine import HipPopulationEngine  # noqa: E402
from serann.genome.interpreter import interpret  # noqa: E402
from serann.models.organism import init_params  # noqa: E402
from tests.archs import ARCHS  # noqa: E402
from tests.test_gpu_engine import _batch, _oracle, _oracle_dev  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "mutant_bn_axis_bsub"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 750
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 0
ir = interpret(ARCHS[name])
params = init_params(ir, 7)
x, g, y = _batch(B, seed=seed)
eng = HipPopulationEngine([ir], [0], device="cuda", params=[params])
grads, _ = eng.debug_train_step(x, g, y)
_, ref = _oracle(ir, params, x, g, y)
bf = _oracle_dev(ir, params, x, g, y, "cuda", torch.bfloat16)
hip = eng.export_arena(0, grads)
for nid, d in sorted(ref.items()):
    for k, v in d.items():
        h, b_ = np.asarray(hip[nid][k], np.float64), np.asarray(bf[nid][k], np.float64)
        print(f"node {nid:2d} {k:8s} |v| {np.linalg.norm(v):.4g}  |hip-v| {np.linalg.norm(h - v):.4g}  "
              f"|bf-v| {np.linalg.norm(b_ - v):.4g}  v[:3] {np.ravel(v)[:3]}  hip[:3] {np.ravel(h)[:3]}  bf[:3] {np.ravel(b_)[:3]}",
              flush=True)
if len(sys.argv) > 4:     # print one gradient fully: node, key
    nid, key = int(sys.argv[4]), sys.argv[5]
    v = np.ravel(ref[nid][key]); h = np.ravel(hip[nid][key]); b_ = np.ravel(bf[nid][key])
    for i in range(len(v)):
        print(f"  {i:3d} fp32 {v[i]: .6f}  hip {h[i]: .6f} ({h[i] - v[i]: .2e})  bf16 {b_[i]: .6f} ({b_[i] - v[i]: .2e})")
if os.environ.get("DIAG_BN"):     # moving statistics after the step: engine vs an fp32 CPU forward
    from serann.models.organism import Organism
    org = Organism(ir, params, device="cpu")
    org(torch.as_tensor(x), torch.as_tensor(g)[..., None], training=True)
    sp = eng.export_params(0)
    for n in ir.nodes:
        if n.op != "bn":
            continue
        for k in ("moving_mean", "moving_variance"):
            r = org.p(n.id, k).detach().numpy()
            h = sp[n.id][k]
            print(f"node {n.id:2d} {k:16s} rel {np.linalg.norm(h - r) / np.linalg.norm(r):.3g}")
            for c in range(min(8, len(r))):
                print(f"    c{c:2d} ref {r[c]: .6e}  hip {h[c]: .6e}")
if os.environ.get("DIAG_ACT"):    # gchain_f64_bn_dense: the BN output (node 4) against a numpy fp32 forward
    mem = eng._debug_mem
    kind, off = mem["orgs"][0]["act"][4]
    R = B * 100
    hy = (mem["act"] if kind == "act" else mem["f32"]).view(off, R * 64).float().cpu().numpy().reshape(R, 64)
    gg = g.reshape(R, 1).astype(np.float32)
    z1 = gg * params[2]["kernel"].reshape(1, 64) + params[2]["bias"]
    xx = np.maximum(z1 @ params[3]["kernel"].reshape(64, 64) + params[3]["bias"], 0)
    mu, var = xx.mean(0), xx.var(0)
    ry = (xx - mu) / np.sqrt(var + 1e-3)
    print("BN out rel", np.linalg.norm(hy - ry) / np.linalg.norm(ry))
    err = np.abs(hy - ry).max(1)
    bad = np.argsort(-err)[:10]
    print("worst rows", [(int(r), float(err[r])) for r in bad])
    rows_bad = np.where(err > 0.05 * np.abs(ry).max())[0]
    print("n rows with large error", len(rows_bad), rows_bad[:40])
    ch = np.argsort(-np.abs(hy - ry).max(0))[:5]
    print("worst channels", ch, [(float(hy[bad[0], c]), float(ry[bad[0], c])) for c in ch])
if os.environ.get("DIAG_DUMP"):   # every activation buffer of organism 0 -> npz (compare two runs offline)
    mem = eng._debug_mem
    out = {}
    for nid, ko in mem["orgs"][0]["act"].items():
        if ko is None:
            continue
        kind, off = ko
        n = int(np.prod(ir.node(nid).shape)) * B
        out[f"a{nid}"] = (mem["act"] if kind == "act" else mem["f32"]).view(off, n).float().cpu().numpy()
    for nid, off in mem["orgs"][0]["grad"].items():
        try:
            n = int(np.prod(ir.node(nid).shape)) * B
            out[f"g{nid}"] = mem["grad"].view(off, n).float().cpu().numpy()
        except Exception as e:  # noqa: BLE001
            print("grad", nid, e)
    np.savez(os.environ["DIAG_DUMP"], **out)
