"""Shard capacity (waves, out-of-memory fallback, admission), the per-generation watchdog and the
supervised relaunch with auto-resume (reference experiment_worker.py:121-126,
run_experiment.py:100-104, evolutionary_experiment/config.py:7)."""
import os
import subprocess
import sys
import textwrap
import time

import numpy as np
import pytest

from serann.config import default_parameters
from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
from serann.engine.base import TrainConfig
from serann.experiment import capacity
from serann.experiment import worker as W
from serann.genome.interpreter import interpret

from .archs import ARCHS

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def data():
    enc = synthetic_encodings()
    return get_serann_data(enc, synthetic_mnist(n_train=800, n_test=200, seed=2), n_train=800, n_test=200)


def _shard(names=("conv_pool_dense", "odd_channels_bn", "empty_x_branch", "narrow_bn_x")):
    irs = [interpret(ARCHS[n]) for n in names]
    ids = [f"org{i}" for i in range(len(irs))]
    genos = np.random.default_rng(0).integers(0, 2, (len(irs), 100)).astype(np.float64)
    return irs, ids, genos


def _run(data, max_per_wave=None, **kw):
    p = default_parameters("example")
    w = W.ShardWorker(p, data, "torch", "cpu", TrainConfig(epochs=1, batch_size=200), max_per_wave=max_per_wave,
                      log=lambda m: None)
    irs, ids, genos = _shard(**kw)
    res = w.run(list(range(len(irs))), ids, genos, irs, 3, generation=1, random_seed=7)
    return w, res


def test_plan_waves():
    assert capacity.plan_waves([5, 5, 5], None) == [[0, 1, 2]]
    assert capacity.plan_waves([5, 5, 5], 10) == [[0, 1], [2]]
    assert capacity.plan_waves([50, 5], 10) == [[0], [1]]          # an oversized organism gets its own wave
    assert capacity.plan_waves([1] * 5, None, max_per_wave=2) == [[0, 1], [2, 3], [4]]
    assert capacity.plan_waves([], 10) == []


def test_device_bytes_estimate_scales_with_batch():
    ir = interpret(ARCHS["conv_pool_dense"])
    a, b = capacity.organism_device_bytes(ir, 375), capacity.organism_device_bytes(ir, 750)
    assert 1.5 < b / a < 2.1
    assert capacity.organism_device_bytes(ir, 750, 50) > b


def test_waves_are_numerically_transparent(data):
    """Training a shard in waves gives every organism exactly the metrics and offspring of one engine."""
    w1, one = _run(data)
    w2, waves = _run(data, max_per_wave=2)
    assert w1.last_waves == [[0, 1, 2, 3]] and w2.last_waves == [[0, 1], [2, 3]]
    assert np.array_equal(one.metrics, waves.metrics)
    assert np.array_equal(one.offspring, waves.offspring)


def test_budget_env_forces_waves(data, monkeypatch):
    monkeypatch.setenv(capacity.ENV_BUDGET, "1e-9")               # every organism exceeds it: one per wave
    w, res = _run(data)
    assert w.last_waves == [[0], [1], [2], [3]]
    assert np.all(np.isfinite(res.metrics[:, 0]))


def test_oom_splits_the_wave_then_half_batch_then_fails_soft(data, monkeypatch):
    """An allocation failure splits the failing wave; a single organism that still fails is retried at
    half the batch (the reference's behaviour), and after that reported with NaN metrics."""
    import torch
    real = W.make_engine
    calls = []

    def fake(name, irs, seeds, device, cfg):
        calls.append((len(irs), cfg.batch_size))
        if len(irs) > 1:
            raise torch.cuda.OutOfMemoryError("HIP out of memory (simulated)")
        if len(irs) == 1 and irs[0].arch_hash() == interpret(ARCHS["narrow_bn_x"]).arch_hash():
            raise RuntimeError("HIP error: out of memory")       # never fits: fails soft
        return real(name, irs, seeds, device, cfg)

    monkeypatch.setattr(W, "make_engine", fake)
    w, res = _run(data)
    assert (4, 200) in calls and (1, 100) in calls             # split, then a half-batch retry
    assert [m for m in w.last_waves] == [[0], [1], [2], [3]]
    assert np.all(np.isfinite(res.metrics[:3, 0])) and np.all(np.isnan(res.metrics[3]))
    assert res.offspring[3].sum() == 0
    monkeypatch.setattr(W, "make_engine", real)
    _, ref = _run(data)
    assert np.array_equal(ref.metrics[:3], res.metrics[:3])      # the split waves train identically


def test_non_oom_errors_propagate(data, monkeypatch):
    def boom(*a, **k):
        raise ValueError("not an allocation failure")
    monkeypatch.setattr(W, "make_engine", boom)
    with pytest.raises(ValueError):
        _run(data)


def test_watchdog_fires_on_a_stalled_generation(tmp_path):
    """A rank whose generation stalls (SERANN_FAULT_INJECT mode=hang) is ended by the watchdog with
    status EXIT_TIMEOUT well before any collective timeout."""
    script = tmp_path / "stall.py"
    script.write_text(textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {REPO!r})
        from serann.utils.faults import GenerationWatchdog, maybe_inject
        wd = GenerationWatchdog(1.0)
        wd.arm("generation 0")
        maybe_inject(0, 0, spec="generation=0,mode=hang")
    """))
    t0 = time.time()
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=60)
    from serann.utils.faults import EXIT_TIMEOUT
    assert r.returncode == EXIT_TIMEOUT, (r.returncode, r.stderr)
    assert "exceeded its timeout" in r.stderr
    assert time.time() - t0 < 30


def test_watchdog_disarmed_does_not_fire():
    from serann.utils.faults import GenerationWatchdog
    wd = GenerationWatchdog(0.2)
    with wd.arm("g"):
        pass
    time.sleep(0.4)                                            # still alive


def test_supervised_relaunch_resumes_with_recorded_id(tmp_path):
    """``--max-restarts``: a child that dies after recording its experiment id is relaunched with
    ``--resume-experiment-id <id>``; restarts stop at the first success."""
    from serann.cli.launch import RUN_ID_ENV, _with_resume, supervise
    log = tmp_path / "calls.txt"
    child = tmp_path / "child.py"
    child.write_text(textwrap.dedent(f"""
        import os, sys
        with open({str(log)!r}, "a") as f:
            f.write(" ".join(sys.argv[1:]) + "\\n")
        if "--resume-experiment-id" not in sys.argv:
            with open(os.environ[{RUN_ID_ENV!r}], "w") as f:
                f.write("exp-123")
            sys.exit(76)
        sys.exit(0)
    """))
    rc = supervise(lambda a: [sys.executable, str(child), *a], ["-p", "x.json"], max_restarts=2)
    assert rc == 0
    calls = log.read_text().splitlines()
    assert calls == ["-p x.json", "-p x.json --resume-experiment-id exp-123"]
    assert _with_resume(["-r", "old", "-p", "y"], "new") == ["-p", "y", "--resume-experiment-id", "new"]
    # a run that fails before recording an id is not restarted
    bad = tmp_path / "bad.py"
    bad.write_text("import sys; sys.exit(3)\n")
    assert supervise(lambda a: [sys.executable, str(bad), *a], [], max_restarts=3) == 3


def test_supervisor_stops_when_watchdog_repeats_at_same_generation(tmp_path):
    """A watchdog timeout (EXIT_TIMEOUT) at the same committed generation twice ends supervision: the
    relaunch would redo the identical work.  Relaunches carry SERANN_SUPERVISED_RESUME=1."""
    from serann.cli.launch import RESUME_ENV, RUN_ID_ENV, read_run_id, record_run_id, supervise
    from serann.utils.faults import EXIT_TIMEOUT
    log = tmp_path / "calls.txt"
    child = tmp_path / "child.py"
    child.write_text(textwrap.dedent(f"""
        import os, sys
        with open({str(log)!r}, "a") as f:
            f.write(os.environ.get({RESUME_ENV!r}, "-") + "\\n")
        with open(os.environ[{RUN_ID_ENV!r}], "w") as f:
            f.write("exp-9\\n4")
        sys.exit({EXIT_TIMEOUT})
    """))
    rc = supervise(lambda a: [sys.executable, str(child), *a], [], max_restarts=5)
    assert rc == EXIT_TIMEOUT
    assert log.read_text().split() == ["-", "1"]          # first run + one relaunch, then it gives up
    f = tmp_path / "id"
    import os
    os.environ[RUN_ID_ENV] = str(f)
    try:
        record_run_id("abc", 7)
    finally:
        del os.environ[RUN_ID_ENV]
    assert read_run_id(str(f)) == ("abc", 7)


def test_watchdog_scales_with_shard_and_is_off_for_cpu_runs(monkeypatch):
    from serann.utils.faults import JOB_ORGANISMS, GenerationWatchdog, job_scale
    assert job_scale(0) == 1 and job_scale(JOB_ORGANISMS) == 1 and job_scale(JOB_ORGANISMS + 1) == 2
    assert job_scale(10, waves=3) == 3
    wd = GenerationWatchdog(10.0)
    wd.arm("g", job_scale(300))
    assert wd._armed_s == 30.0
    wd.disarm()
    from serann.cli.launch import CHILD_ENV
    from serann.experiment.experiment import Experiment
    monkeypatch.delenv(CHILD_ENV, raising=False)

    class W:
        engine_name = "torch"
    e = Experiment("x", None, W(), None, {"genotype_size": 8, "num_classification_classes": 10}, None)
    assert e._watchdog.timeout_s == 0           # CPU engine, unsupervised: never armed
    W.engine_name = "hip"
    e = Experiment("x", None, W(), None, {"genotype_size": 8, "num_classification_classes": 10}, None)
    assert e._watchdog.timeout_s > 0
    # a CPU run under the supervising launcher (--max-restarts / --nproc) arms the reference's job timeout
    W.engine_name = "torch"
    monkeypatch.setenv(CHILD_ENV, "1")
    e = Experiment("x", None, W(), None, {"genotype_size": 8, "num_classification_classes": 10}, None)
    from serann.config import experiment_config
    assert e._watchdog.timeout_s == float(experiment_config["worker_pool_job_timeout"])


def test_supervisor_gives_up_on_repeated_timeout_before_any_commit(tmp_path):
    """Two watchdog timeouts with nothing committed (committed generation None both times): the same work
    would time out again, so the supervisor stops after one relaunch instead of using every restart."""
    import sys
    import textwrap
    from serann.cli.launch import supervise
    from serann.utils.faults import EXIT_TIMEOUT
    log = tmp_path / "runs.log"
    child = tmp_path / "child.py"
    child.write_text(textwrap.dedent(f"""
        import os, sys
        sys.path.insert(0, {repr(str(__import__('pathlib').Path(__file__).resolve().parents[1]))})
        from serann.cli.launch import record_run_id
        with open({repr(str(log))}, "a") as f:
            f.write("run ")
        record_run_id("exp-1", None)
        sys.exit({EXIT_TIMEOUT})
    """))
    rc = supervise(lambda a: [sys.executable, str(child), *a], [], max_restarts=5)
    assert rc == EXIT_TIMEOUT
    assert log.read_text().split() == ["run", "run"]


def test_collective_timeout_follows_job_timeout(monkeypatch):
    from serann.config import experiment_config
    from serann.parallel.comm import collective_timeout_s
    monkeypatch.setitem(experiment_config, "worker_pool_job_timeout", 100)
    assert collective_timeout_s() == 400.0


def test_device_bytes_cover_conv_wgrad_slabs():
    """Split conv WGRADs allocate fp32 slabs (ops/hip_ops.py conv_wgrad_splits, ``_wgfin``): the estimate counts
    at least the slab bytes the planner gives an organism's KxK convolutions at the production batch."""
    from serann.ops import hip_ops as H
    ir = interpret("X_layer = Conv2D(filters=32, kernel_size=3, strides=1)(X_layer)\n"
                   "X_layer = Conv2D(filters=32, kernel_size=3, strides=1)(X_layer)\n\n"
                   "con = concatenate([Reshape((1, -1))(X_layer), Reshape((1, -1))(g_layer)])\n\n"
                   "con = Dense(units=64, activation='relu')(con)\n\nloss_balance = 0.5")
    B = 750
    slab = 0
    for n in ir.nodes:
        if n.op != "gemm" or n.attrs["kh"] * n.attrs["kw"] <= 1:
            continue
        a = n.attrs
        (Hh, Ww, C), (OH, OW, F) = ir.node(n.inputs[0]).shape, n.shape
        row = dict(a=0, b=0, out=1, H=Hh, W=Ww, C=C, OH=OH, OW=OW, F=F, KH=a["kh"], KW=a["kw"], SH=1, SW=1, M=F,
                   N=a["kh"] * a["kw"] * C, K=B * OH * OW, flags=0)
        for _, rws, _ in H.gemm3_plan(H.MODE_WGRAD, [row], [(F, row["N"], row["K"])]):
            if rws[0].get("_wgfin"):
                slab += 4 * H.wgrad_slab_elems(rws[0])
    assert slab > 0
    with_slabs = capacity.organism_device_bytes(ir, B)
    # the same organism's estimate without the convolutions' slabs (the old formula) would miss them
    assert with_slabs >= slab + 24 * sum(n.attrs["f"] * n.attrs["kh"] * n.attrs["kw"] * n.attrs["cin"]
                                         for n in ir.nodes if n.op == "gemm" and n.attrs["kind"] not in
                                         ("head_cls", "head_rep"))
