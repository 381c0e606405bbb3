"""Helper script for tests/test_gpu_distributed.py (run as a subprocess, one per rank): a short seeded
experiment on the HIP engine; rank 0 writes the DB to argv[1].  The communicator comes from the
environment (RANK / WORLD_SIZE / MASTER_*; SERANN_COMM_BACKEND=gloo lets two ranks share one GPU;
SERANN_FORCE_DIST=1 with SERANN_COMM_BACKEND=nccl runs one rank through RCCL)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(db_path: str, pop: int, gens: int):
    from serann.config import default_parameters
    from serann.data.datasets import get_serann_data, synthetic_encodings, synthetic_mnist
    from serann.engine.base import TrainConfig
    from serann.experiment.experiment import Experiment
    from serann.experiment.runner import default_device
    from serann.experiment.worker import ShardWorker
    from serann.genome.codec import TableCodec
    from serann.parallel.comm import make_comm
    from serann.utils.db import ExperimentDB

    # SERANN_FORCE_DIST=1: a torch.distributed communicator even for world_size 1 (RCCL on one GPU)
    comm = make_comm(distributed=True if os.environ.get("SERANN_FORCE_DIST") == "1" else None)
    print(f"comm backend={getattr(comm, 'backend', 'local')} world={comm.world_size}", flush=True)
    device = default_device(comm)
    enc = synthetic_encodings()
    data = get_serann_data(enc, synthetic_mnist(n_train=2400, n_test=400, seed=3), n_train=2400, n_test=400)
    p = default_parameters("example")
    p.update(num_seranns=pop, num_generations=gens, training_epochs=1)
    codec = TableCodec.from_generator(256, seed=2, ancestor=p["ancestor_genotype"], sensitive_bits=8)
    w = ShardWorker(p, data, "hip", device, TrainConfig(epochs=1, batch_size=300))
    db = ExperimentDB(db_path) if comm.is_root else None
    e = Experiment("exp", enc, w, db, p, codec, comm=comm, random_seed=11, verbose=False)
    e.execute()
    comm.shutdown()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]))
