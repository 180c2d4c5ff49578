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
# The same sharded run with the HIP engines on every rank (GPU box: both ranks share cuda:0 and
# gather over gloo; on a multi-GPU node bench.py runs this code path one rank per GPU over RCCL).
# Each rank steps its shard of sequences through ONE batched engine launch per frame; every
# output row is gathered ([sequence, frame, row...]) and must equal the single-process oracle's.
GPU_KINDS = ("bytetrack", "botsort", "ocsort", "boosttrack", "strongsort")
NCOL = {"strongsort": 10}
BOOST_ARGS = dict(max_age=60, min_hits=3, det_thresh=0.6, iou_threshold=0.3, use_ecc=True,
                  min_box_area=10, aspect_ratio_thresh=1.6, lambda_iou=0.5, lambda_mhd=0.25,
                  lambda_shape=0.25, use_dlo_boost=True, use_duo_boost=True, dlo_boost_coef=0.65,
                  s_sim_corr=False, use_rich_s=True, use_sb=True, use_vt=True, with_reid=True)
SS_ARGS = dict(min_conf=0.1, max_cos_dist=0.15, max_iou_dist=0.7, max_age=50, n_init=2,
               nn_budget=150, mc_lambda=0.995, ema_alpha=0.9, conf_thresh_high=0.7,
               conf_thresh_low=0.3, id_preservation_weight=0.1, crowd_detection=True,
               born_confirmed=True)
OCS_ARGS = dict(min_conf=0.1, det_thresh=0.6, max_age=30, min_hits=3, asso_threshold=0.3,
                delta_t=3, inertia=0.1, use_byte=False, Q_xy_scaling=0.01, Q_s_scaling=0.0001)
EMB = {"botsort": 64, "boosttrack": 32, "strongsort": 32}


def gpu_sequences(kind, g):
    from boxmot_amd.synth import SyntheticScene

    kw = {}
    if kind in ("boosttrack", "strongsort"):
        kw = dict(emb_dtype=np.float64, conf_lo=0.3)
    if kind == "ocsort":
        kw = dict(conf_lo=0.3)
    return SyntheticScene(n_obj=20 + 3 * g, seed=70 + g, emb_dim=EMB.get(kind, 0),
                          layout="crowded" if g % 2 else "grid", **kw)


def gpu_args(kind):
    return {"bytetrack": dict(min_conf=0.1, track_thresh=0.6, match_thresh=0.9, track_buffer=30),
            "botsort": dict(track_high_thresh=0.6, new_track_thresh=0.7, match_thresh=0.8),
            "ocsort": OCS_ARGS, "boosttrack": BOOST_ARGS, "strongsort": SS_ARGS}[kind]


def make_engine(kind, n):
    from boxmot_amd import engine as E

    a = gpu_args(kind)
    if kind == "ocsort":
        return E.OcsortEngine(n_seq=n, track_cap=128, det_cap=128, params=E.OcsortParams(**a))
    if kind == "boosttrack":
        return E.BoostEngine(n_seq=n, track_cap=128, det_cap=128, emb_dim=EMB[kind],
                             params=E.BoostParams(**a))
    if kind == "strongsort":
        return E.SsEngine(n_seq=n, track_cap=256, det_cap=128, emb_dim=EMB[kind], vec_cap=32,
                          params=E.SsParams(**a))
    return E.Engine(kind, n_seq=n, track_cap=256, det_cap=128, emb_dim=EMB.get(kind, 0),
                    params=E.EngineParams(**a))


def _gpu_worker(rank, world, port, path, kind):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    mine = shard_sequences([N_FRAMES + g for g in range(N_SEQ)], world, rank)
    scenes = [gpu_sequences(kind, g) for g in mine]
    eng = make_engine(kind, len(mine))
    ncol = NCOL.get(kind, 8)
    f64 = kind == "strongsort"  # StrongSort takes float64 detections (no setup_decorator)
    rows = []
    for t in range(1, N_FRAMES + 1):
        fr = [sc.frame(t) for sc in scenes]
        off = np.zeros(len(mine) + 1, np.int32)
        off[1:] = np.cumsum([f[0].shape[0] for f in fr])
        d = torch.from_numpy(np.concatenate([f[0] for f in fr]).astype(
            np.float64 if f64 else np.float32)).cuda()
        e = (torch.from_numpy(np.concatenate([f[1] for f in fr])).cuda()
             if EMB.get(kind) else None)
        o = torch.empty((max(int(off[-1]), 1), ncol), dtype=torch.float64, device="cuda")
        c = torch.empty(len(mine), dtype=torch.int32, device="cuda")
        do = torch.from_numpy(off).cuda()
        if kind == "ocsort":
            eng.step(d, do, o, c)
        else:
            eng.step(d, do, e, None, o, c)
        o, c = o.cpu().numpy(), c.cpu().numpy()
        for k, g in enumerate(mine):
            r = o[off[k]: off[k] + c[k]]
            rows.append(np.concatenate([np.full((r.shape[0], 1), g), np.full((r.shape[0], 1), t),
                                        r], 1))
    assert eng.status() == 0
    recs = np.concatenate(rows, 0) if rows else np.zeros((0, ncol + 2))
    allrec = gather_records(recs.reshape(-1, ncol + 2), dist, "cpu")
    if rank == 0:
        np.save(path, allrec)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", GPU_KINDS)
def test_sharded_engine_run_equals_oracle(kind):
    """All five trackers: world-size-2 sequence sharding with the HIP engine per rank; the
    gathered output rows of every sequence equal the oracle's, bit for bit."""
    from oracle import pyoracle as po

    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "rows.npy")
        mp.spawn(_gpu_worker, args=(2, free_port(), path, kind), nprocs=2, join=True)
        got = np.load(path)
    assert sorted(set(got[:, 0].astype(int))) == list(range(N_SEQ))
    for g in range(N_SEQ):
        sc, tr = gpu_sequences(kind, g), po.OracleTracker(kind, **gpu_args(kind))
        ref = []
        for t in range(1, N_FRAMES + 1):
            dets, embs, _ = sc.frame(t)
            o = tr.update(dets, embs) if EMB.get(kind) else tr.update(dets)
            ref.append(np.concatenate([np.full((o.shape[0], 1), t), o], 1))
        mine = got[got[:, 0] == g][:, 1:]
        np.testing.assert_array_equal(mine, np.concatenate(ref, 0), err_msg=f"{kind} seq {g}")


@pytest.mark.gpu
def test_gather_records_over_rccl_single_gpu():
    """The RCCL ("nccl" backend) branch of gather_records, on the one GPU a box has: a world of
    one rank still runs both all_gathers (sizes, then the padded payload) on the device."""
    import torch
    import torch.distributed as dist

    if not torch.cuda.is_available():
        pytest.fail("GPU test collected without a HIP device")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0,
                            world_size=1)
    try:
        rng = np.random.default_rng(7)
        for n in (0, 1, 37):
            recs = rng.standard_normal((n, 3))
            got = gather_records(recs, dist, torch.device("cuda", 0), collective=True)
            np.testing.assert_array_equal(got, recs)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


def _bench(args, backend, timeout=900):
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["BX_DIST_BACKEND"] = backend
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_gpus_n_refuses_more_ranks_than_gpus_over_rccl():
    """`bench.py --gpus 2` without a launcher starts two ranks itself; over RCCL each rank refuses
    a world larger than the visible device count (none here), and the launcher exits non-zero
    instead of timing one GPU and reporting it as two."""
    r = _bench(["--gpus", "2", "--config", "boosttrack_mot8", "--steps", "1", "--warmup", "1",
                "--no-cpu-baseline"], "nccl", timeout=300)
    assert r.returncode != 0
    assert "need 2 GPUs" in r.stderr, r.stderr[-2000:]
    assert "rank(s) failed" in r.stderr


@pytest.mark.gpu
def test_bench_gpus_2_launches_two_ranks():
    """`python bench.py --gpus 2` (no torch.distributed launcher) on the one-GPU box with gloo:
    two ranks share the card (modulo rehearsal), C5's eight sequences are LPT-sharded over them,
    the line reports n_gpus 2 with all eight gathered, and every sequence's last-frame checksum
    equals the one-rank run's (sharding never changes a sequence's outputs)."""
    args = ["--config", "boosttrack_mot8", "--steps", "3", "--warmup", "2", "--no-cpu-baseline"]
    two = _bench(["--gpus", "2"] + args, "gloo")
    assert two.returncode == 0, two.stderr[-3000:]
    l2 = json.loads(two.stdout.strip().splitlines()[-1])
    assert l2["n_gpus"] == 2
    assert l2["config"]["sequences_gathered"] == 8
    assert sorted(map(int, l2["config"]["last_frame_checksums"])) == list(range(8))
    one = _bench(["--gpus", "1"] + args, "gloo")
    assert one.returncode == 0, one.stderr[-3000:]
    l1 = json.loads(one.stdout.strip().splitlines()[-1])
    assert l1["n_gpus"] == 1
    assert l1["config"]["last_frame_checksums"] == l2["config"]["last_frame_checksums"]
