"""world_size-2 gloo tests of the multi-GPU path: sequences are sharded across ranks with no
per-frame exchange, and per-sequence records are gathered once at the end (boxmot_amd/shard.py,
the same code bench.py runs over RCCL).  The per-rank compute here is the CPU oracle."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from boxmot_amd.shard import gather_records, output_checksum, shard_sequences

N_SEQ, N_FRAMES = 5, 15


def run_sequence(g):
    from boxmot_amd.synth import SyntheticScene
    from oracle import pyoracle as po

    sc = SyntheticScene(n_obj=20 + 3 * g, seed=50 + g, layout="crowded" if g % 2 else "grid")
    tr = po.OracleTracker("bytetrack", track_thresh=0.6, match_thresh=0.9)
    outs = [tr.update(sc.frame(t)[0]) for t in range(1, N_FRAMES + 1)]
    return np.concatenate(outs, 0) if outs else np.zeros((0, 8))


def _worker(rank, world, port, path):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = shard_sequences([N_FRAMES + g for g in range(N_SEQ)], world, rank)
    recs = np.array([[g, N_FRAMES, output_checksum(run_sequence(g))] for g in mine]).reshape(-1, 3)
    allrec = gather_records(recs, dist, "cpu")
    if rank == 0:
        with open(path, "w") as f:
            json.dump(allrec.tolist(), f)
    dist.barrier()
    dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
def test_sharded_run_equals_single_process(world):
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "rec.json")
        mp.spawn(_worker, args=(world, free_port(), path), nprocs=world, join=True)
        got = np.array(json.load(open(path)))
    got = got[np.argsort(got[:, 0])]
    assert list(got[:, 0]) == list(range(N_SEQ))  # every sequence exactly once
    ref = np.array([output_checksum(run_sequence(g)) for g in range(N_SEQ)])
    np.testing.assert_array_equal(got[:, 2], ref)


def test_shard_sequences_partition():
    for world in (1, 2, 3, 8):
        fc = [300, 525, 260, 410, 600, 340, 470, 500, 290]
        parts = [shard_sequences(fc, world, r) for r in range(world)]
        flat = sorted(i for p in parts for i in p)
        assert flat == list(range(len(fc)))
        loads = [sum(fc[i] for i in p) for p in parts]
        assert max(loads) - min(loads) <= max(fc)  # LPT balance bound
        parts = [shard_sequences(1024 * world, world, r) for r in range(world)]
        assert [p[0] for p in parts] == [1024 * r for r in range(world)]
