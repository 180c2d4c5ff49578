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


# ---------------------------------------------------------------------------------------------
# The same sharded run with the HIP engine on every rank (GPU box: both ranks share cuda:0 and
# gather over gloo; on a multi-GPU node bench.py runs this code path one rank per GPU over RCCL).
# Each rank steps its shard of sequences through ONE batched engine launch per frame and the
# gathered per-sequence checksums must equal the single-process oracle's.
GPU_KINDS = ("bytetrack", "botsort")


def gpu_sequences(kind, g):
    from boxmot_amd.synth import SyntheticScene

    emb = 64 if kind == "botsort" else 0
    return SyntheticScene(n_obj=20 + 3 * g, seed=70 + g, emb_dim=emb,
                          layout="crowded" if g % 2 else "grid")


def gpu_args(kind):
    return (dict(min_conf=0.1, track_thresh=0.6, match_thresh=0.9, track_buffer=30)
            if kind == "bytetrack" else dict(track_high_thresh=0.6, new_track_thresh=0.7,
                                             match_thresh=0.8))


def _gpu_worker(rank, world, port, path, kind):
    import torch
    import torch.distributed as dist

    from boxmot_amd.engine import Engine, EngineParams

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    mine = shard_sequences([N_FRAMES + g for g in range(N_SEQ)], world, rank)
    scenes = [gpu_sequences(kind, g) for g in mine]
    emb = 64 if kind == "botsort" else 0
    eng = Engine(kind, n_seq=len(mine), track_cap=256, det_cap=128, emb_dim=emb,
                 params=EngineParams(**gpu_args(kind)))
    outs = [[] for _ in mine]
    for t in range(1, N_FRAMES + 1):
        fr = [sc.frame(t) for sc in scenes]
        off = np.zeros(len(mine) + 1, np.int32)
        off[1:] = np.cumsum([f[0].shape[0] for f in fr])
        d = torch.from_numpy(np.concatenate([f[0] for f in fr]).astype(np.float32)).cuda()
        e = torch.from_numpy(np.concatenate([f[1] for f in fr])).cuda() if emb else None
        o = torch.empty((max(int(off[-1]), 1), 8), dtype=torch.float64, device="cuda")
        c = torch.empty(len(mine), dtype=torch.int32, device="cuda")
        eng.step(d, torch.from_numpy(off).cuda(), e, None, o, c)
        o, c = o.cpu().numpy(), c.cpu().numpy()
        for k in range(len(mine)):
            outs[k].append(o[off[k]: off[k] + c[k]])
    assert eng.status() == 0
    recs = np.array([[g, N_FRAMES, output_checksum(np.concatenate(outs[k], 0))]
                     for k, g in enumerate(mine)]).reshape(-1, 3)
    allrec = gather_records(recs, dist, "cpu")
    if rank == 0:
        with open(path, "w") as f:
            json.dump(allrec.tolist(), f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", GPU_KINDS)
def test_sharded_engine_run_equals_oracle(kind):
    from oracle import pyoracle as po

    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "rec.json")
        mp.spawn(_gpu_worker, args=(2, free_port(), path, kind), nprocs=2, join=True)
        got = np.array(json.load(open(path)))
    got = got[np.argsort(got[:, 0])]
    assert list(got[:, 0]) == list(range(N_SEQ))
    ref = []
    for g in range(N_SEQ):
        sc, tr = gpu_sequences(kind, g), po.OracleTracker(kind, **gpu_args(kind))
        ref.append(output_checksum(np.concatenate(
            [tr.update(*sc.frame(t)[:2]) for t in range(1, N_FRAMES + 1)], 0)))
    np.testing.assert_array_equal(got[:, 2], np.array(ref))
