"""The SPMD path with the HIP engine: two ranks (gloo communicator, both on cuda:0, one process each)
through two generations write the same experiment DB, row for row and bit for bit, as one rank
(reference split being replaced: evolutionary_experiment/logic/experiment.py:170-178).

This holds only because every organism trains bit-identically whatever shard it lands in: reduction
splits are per problem (ops/hip_ops.py) and partial sums meet in order-free fixed point
(csrc/hip/common.h), so the LPT partition changes the schedule, never the numbers."""
import os
import socket
import sqlite3
import subprocess
import sys

import pandas as pd
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launch(db, world, pop, gens, backend="gloo"):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SERANN_COMM_BACKEND=backend, HSA_ENABLE_IPC_MODE_LEGACY="0")
        if backend == "nccl":
            env["SERANN_FORCE_DIST"] = "1"
        elif world == 1:
            for k in ("RANK", "WORLD_SIZE", "MASTER_PORT"):
                env.pop(k)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_experiment.py"), str(db), str(pop),
                                       str(gens)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for pr in procs:
        try:
            out, _ = pr.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
        assert pr.returncode == 0, out.decode(errors="replace")[-3000:]
    return outs


def test_two_ranks_write_the_single_rank_db(tmp_path):
    one, two = tmp_path / "one.sqlite", tmp_path / "two.sqlite"
    _launch(one, 1, 8, 2)
    _launch(two, 2, 8, 2)
    q = "select * from serann order by generation, id"
    a = pd.read_sql(q, sqlite3.connect(one))
    b = pd.read_sql(q, sqlite3.connect(two))
    assert len(a) == 16 and a["is_valid"].sum() > 0
    pd.testing.assert_frame_equal(a, b)
    cols = ("generation, survival_rate, mean_classification_validation_accuracy, mean_replication_mse, "
            "genotype_nucleotide_diversity, source_code_species_richness")
    pd.testing.assert_frame_equal(pd.read_sql(f"select {cols} from generations", sqlite3.connect(one)),
                                  pd.read_sql(f"select {cols} from generations", sqlite3.connect(two)))


def test_rccl_communicator_with_hip_engine(tmp_path):
    """The RCCL (``nccl``) communicator in the same process as the HIP engine's captured graphs and
    side streams: one rank through torch.distributed over RCCL -- length all-gather, packed
    ``all_gather_into_tensor`` of the device payload, broadcasts, barrier -- writes the same DB as the
    plain local communicator.  (Two RCCL ranks cannot share one GPU; the 2-rank schedule is covered by
    the gloo test above and the multi-GPU bench.)"""
    local, rccl = tmp_path / "local.sqlite", tmp_path / "rccl.sqlite"
    _launch(local, 1, 8, 2)
    out = _launch(rccl, 1, 8, 2, backend="nccl")
    assert "comm backend=nccl world=1" in out[0], out[0][-2000:]
    q = "select * from serann order by generation, id"
    pd.testing.assert_frame_equal(pd.read_sql(q, sqlite3.connect(local)), pd.read_sql(q, sqlite3.connect(rccl)))
