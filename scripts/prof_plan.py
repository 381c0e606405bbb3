#!/usr/bin/env python
"""cProfile of the training-plan build (HipPopulationEngine._build_plan, all stream groups) on a fixed
population: where the per-generation host planning time goes.  --device cpu runs it without a GPU (the
CPU pays torch.zeros of the workspaces, which the GPU does not)."""
import argparse
import cProfile
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--population-file", default="populations/bench_gen3_pop125.json")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    from serann.engine.base import TrainConfig
    from serann.engine.hip_engine import HipPopulationEngine
    from serann.genome.interpreter import try_interpret
    irs = [try_interpret(s).ir for s in json.load(open(a.population_file))]
    cfg = TrainConfig(epochs=1, batch_size=750)
    dev = torch.device(a.device)
    xb = torch.zeros(750 * 784 + 256, dtype=torch.bfloat16, device=dev)
    gb = torch.zeros(750 * 100 + 256, dtype=torch.bfloat16, device=dev)
    yb = torch.zeros(750, dtype=torch.int32, device=dev)
    for rep in range(a.repeat):
        eng = HipPopulationEngine(irs, list(range(len(irs))), device=a.device, cfg=cfg)
        mem = eng._alloc_buffers(750, with_grads=True)
        metrics = torch.zeros(len(irs), 4, dtype=torch.int64, device=dev)
        inputs = [{"X": xb.data_ptr(), "g": gb.data_ptr()} for _ in irs]
        groups = eng._stream_groups(a.streams)
        pr = cProfile.Profile()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t = time.perf_counter()
        pr.enable()
        plans = [eng._build_plan("train", 750, mem, inputs, yb.data_ptr(), [gb.data_ptr()] * len(irs), metrics,
                                 orgs=g) for g in groups]
        pr.disable()
        dt = time.perf_counter() - t
        print(f"rep {rep}: plan_s={dt:.4f} launches={sum(len(p.launches) for p in plans)} organisms={len(irs)}",
              flush=True)
        if rep == a.repeat - 1:
            pstats.Stats(pr).sort_stats("cumulative").print_stats(a.top)
            pstats.Stats(pr).sort_stats("tottime").print_stats(25)
        eng.close()


if __name__ == "__main__":
    main()
