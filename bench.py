#!/usr/bin/env python
"""Association-FPS benchmark (BASELINE.json metric) for the MI355X engine.

A step = one frame of every sequence this rank holds, advanced by one `Engine.step` (the frame
pipeline of kernels).  Workload (BASELINE.json configs[2], the north_star's
256-track x 128-det x 512-d target): BoT-SORT on synthetic grid scenes of 256 objects detected
w.p. 0.5 (~128 dets/frame, all above track_high_thresh) with 512-d float32 embeddings;
`--config bytetrack` runs configs[1] (ByteTrack, IoU only); `--config boosttrack` the C5 tracker
(BoostTrack++ with 512-d float64 ReID on MOT17-sized scenes: 60 objects, ~30 dets/frame).  Each rank holds `--seqs` independent
sequences (weak scaling: the sequence count per GPU is fixed as N grows; no per-frame
collective).  Inputs for every timed frame are generated on the GPU and resident in HBM before
the timed region.

Roofline: the last `len(STAGES)` warm-up steps time each pipeline stage once (HIP events around
that stage's launch, `Engine.probe`); the slowest stage is the dominant kernel and is probed on
every timed step.  Its algorithmic bytes per launch (DESIGN.md §4 per-stage model, priced with
the engine's own per-frame unit counts) over its measured average launch time is `achieved`.

Single process: `python bench.py`.  Multi-GPU: `python bench.py --gpus N` starts N child ranks
itself (one per GPU, `launch_ranks`), or `torch.distributed.run --nproc-per-node N bench.py
--gpus N` sets RANK/WORLD_SIZE for it; either way RCCL only gathers the per-sequence records
once, at the end.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "association FPS (frames/sec) at N_tracks×N_dets×feat_dim, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# dense fp64 matrix rate: MI355X spec 78.6 TFLOP/s (the guide's MFMA table has no f64 row); the
# v_mfma_f64_16x16x4 rate measured on the box is 73.1 (tools/probes/mfma_f64_peak.hip) and rides
# along in the line as peak_measured
F64_MFMA_PEAK_TFS = 78.6
F64_MFMA_MEASURED_TFS = 73.1

from boxmot_amd.workloads import (  # noqa: E402  (the workloads: shared with the tests)
    C5_TOTAL, CONFIGS, DEFAULT_SEQS, MOT_DETS, OCS_CONF_LO, SS_C4_CAPS, ss_caps)

# OCSort per-launch algorithmic bytes: per live track the XYSR state (x[7], P[49] f64) read and
# written plus its observation record (last_obs, velocity, k-previous box: 12 f64) read; per
# detection one f32 row in; per output one f64 row out.
OCS_TRACK_BYTES = 2 * 56 * 8 + 12 * 8

KF_STATE = 576  # fp64 mean[8] + covariance[64] per track


def stage_bytes(stage, u, F, es=4):
    """Algorithmic HBM bytes of one launch of `stage`, from the unit counts `u`
    of a frame summed over sequences: dets, high, active, lost, records, pairs."""
    listed = u["active"] + u["lost"]
    return {
        # the embedding row of every high detection + 3 norms out
        "det_features": u["high"] * (F * es + 24),
        # mean read + predicted mean and pre-predict (h, a|w) written, per pooled track
        "predict": listed * (64 + 64 + 16),
        # track box per listed track, det row per det, one pair word per gated pair
        "gate": listed * 32 + u["dets"] * 24 + u["pairs"] * 4,
        # smooth_feat row + embedding row per gated pair, distance out
        "cosine": u["pairs"] * (2 * F * es + 8),
        # det rows, track boxes/flags/lists, records out
        "assoc": u["dets"] * 24 + listed * (32 + 16) + u["records"] * 8,
        # state read + written per update record, det row in
        "update": u["records"] * (2 * KF_STATE + 24),
        # covariance read + written for pooled tracks without an update
        "cov_predict": max(listed - u["records"], 0) * 2 * 512,
        # embedding row + smooth_feat read, smooth_feat written, per record with a feature
        "features": u["records"] * 3 * F * es,
        # box per listed track, output row per activated track
        "finish": listed * 48 + u["dets"] * 64,
    }[stage]


def boost_stage_bytes(stage, u, F):
    """Algorithmic HBM bytes of one BoostTrack launch from the frame's unit counts
    summed over sequences: dets, kept, tracks (entering the frame), outputs, records, pairs."""
    return {
        # every detection's and live track's f64 embedding read once, one f64 entry per pair out
        "embcost": (u["dets"] + u["tracks"]) * F * 8 + u["pairs"] * 8,
        # Kalman state (x[8], P[64] + scalars, 616 B) read + written per track, f32 det rows in,
        # the pair's ReID entry read, output rows + update records out
        "frame": u["tracks"] * 2 * 616 + u["dets"] * 24 + u["pairs"] * 8 + u["outputs"] * 64 +
                 u["records"] * 16,
        # detection row + track embedding read, track embedding written, per record
        "feature": u["records"] * 3 * F * 8,
    }[stage]


def ss_stage_bytes(stage, u, F):
    """Algorithmic HBM bytes of one StrongSort launch from the frame's unit
    counts summed over sequences: dets (kept), tracks, queried (confirmed tracks with a gallery),
    rows (distinct gallery samples compared), outputs."""
    return {
        # embedding row in, NN-normalised and track-normalised rows out
        "prep": u["dets"] * 3 * F * 8,
        # every compared sample row and every detection row read once, one distance per
        # (queried track, detection) out
        "nn": (u["rows"] + u["dets"]) * F * 8 + u["queried"] * (u["dets"] // max(u["seqs"], 1)) * 8,
        # the feature row of each lost track and the detection rows
        "recovery": u["dets"] * F * 8,
        # track records (mean, cov, histories: ~1.2 kB) read + written, detection rows
        "pre": u["tracks"] * 2 * 1200 + u["dets"] * 64,
        # per confirmed track: its record read, one cost per detection written
        "cost": u["queried"] * 1200 + u["queried"] * (u["dets"] // max(u["seqs"], 1)) * 8,
        # the cost entries gathered by the cascade levels, the IoU stage's detection rows
        "match": u["queried"] * (u["dets"] // max(u["seqs"], 1)) * 8 + u["dets"] * 64,
        # per match: the detection's normalised row and the last feature read, the new vector
        # written (then read back twice for its norms), the track record read + written
        "update": u["matches"] * (5 * F * 8 + 2 * 1200),
        "post": u["tracks"] * 1200 + u["outputs"] * 80,
        # per listed track: its gallery entries (<= budget + 10 of 16 B) read + written
        "fit": u["tracks"] * 2 * 160 * 16,
    }[stage]


# The reference's own CPU path (Python/numpy/scipy), measured during the survey on one core of an
# Intel Xeon (8 vCPU) container — carried beside the port's numbers, with its
# hardware; the Python reference itself never runs on the GPU box.
REFERENCE_CPU_FPS = {
    "botsort": (26.4, "C3 BoT-SORT 256 x 129 x 512-d"),
    "bytetrack": (29.6, "C2 ByteTrack 256 x 129"),
    "strongsort_c4": (0.16, "C4 StrongSort 1024 x ~512 x 2048-d"),
    "boosttrack": (36.3, "BoostTrack 256 x 129 x 512-d (one sequence)"),
    "ocsort": (430.0, "C1 OCSort MOT17-02 (~17 tracks)"),
}


def cpu_quota():
    """CPUs' worth of time the cgroup grants this process (cgroup v2 cpu.max / v1 cfs quota), or
    None when unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return float(q) / float(per)
        return None
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return q / per if q > 0 else None
    except (OSError, ValueError):
        return None


def host_cpu():
    """CPU model, logical CPUs of the machine, CPUs this process may run on, and the cgroup's
    CPU quota (the cores the baseline can actually use at once)."""
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    quota = cpu_quota()
    cores = usable if quota is None else max(1, min(usable, int(quota)))
    # the GPU pool grants each 1-GPU job a CPU share and exports it as OMP_NUM_THREADS (16);
    # its rules ask worker pools to stay within that share, so the baseline does too
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        cores = min(cores, int(share))
    return {"model": model, "logical_cpus": os.cpu_count(), "usable_cpus": usable,
            "cgroup_cpu_quota": quota, "job_cpu_share": int(share) if share.isdigit() else None,
            "cores": cores}


def cpu_worker(spec):
    """One CPU-baseline worker (run in a child process: no torch, no GPU): the C oracle on one
    sequence of the workload, `warm` untimed frames, then frames until `seconds` of busy time."""
    from boxmot_amd.synth import SyntheticScene
    from oracle import pyoracle as po

    kind, n_obj, emb_dim, params = spec["kind"], spec["n_obj"], spec["emb_dim"], spec["params"]
    po.set_threads(spec.get("threads", 1))
    if "c5" in spec:  # one of C5's eight sequences, played to its end at most
        from boxmot_amd.synth import c5_sequences

        _, sc, nf = c5_sequences(MOT_DETS, emb_dim)[spec["c5"]]
        spec["max_frames"] = min(spec.get("max_frames", 1 << 30), nf - spec["warm"])
    else:
        extra = dict(conf_lo=OCS_CONF_LO) if kind in ("ocsort", "boosttrack", "strongsort") else {}
        if kind in ("boosttrack", "strongsort"):
            extra["emb_dtype"] = np.float64
        sc = SyntheticScene(n_obj=n_obj, seed=spec["seed"], emb_dim=emb_dim,
                            layout=spec.get("layout", "grid"), **extra)
    tr = po.OracleTracker(kind, **params)
    t = 0
    for _ in range(spec["warm"]):
        t += 1
        d, e, _ = sc.frame(t)
        tr.update(d, e)
    frames, busy = 0, 0.0
    while busy < spec["seconds"] and frames < spec.get("max_frames", 1 << 30):
        t += 1
        d, e, _ = sc.frame(t)  # generation excluded from the timed work
        t0 = time.perf_counter()
        tr.update(d, e)
        busy += time.perf_counter() - t0
        frames += 1
    return {"frames": frames, "busy": busy, "first": spec["warm"] + 1, "last": t}


def run_cpu_workers(specs):
    """Run each spec in its own child process (subprocess: a fresh interpreter per worker, like
    val.py:389's process pool; the parent's GPU context is never forked or exec'd over)."""
    import subprocess

    procs = [subprocess.Popen([sys.executable, str(Path(__file__).resolve()), "--cpu-worker",
                               json.dumps(sp)], stdout=subprocess.PIPE, text=True,
                              env=dict(os.environ, OMP_NUM_THREADS=str(sp.get("threads", 1))))
             for sp in specs]
    res = []
    for p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"cpu worker failed (rc {p.returncode})")
        res.append(json.loads(out.strip().splitlines()[-1]))
    return res


def cpu_baseline(config, kind, n_obj, emb_dim, params, seconds=15.0):
    """The C oracle (port of the reference semantics) on the GPU box's host cores: one sequence on
    one thread, and one process per sequence on all usable cores (val.py:389's model; C4 is one
    sequence, so its all-cores variant is one process whose NN rows run on all cores)."""
    host = host_cpu()
    P = host["cores"]  # every core the process may use at once (affinity, capped by the cgroup)
    c4 = config == "strongsort_c4"
    warm = 8 if c4 else 40
    base = dict(kind=kind, n_obj=n_obj, emb_dim=emb_dim, params=params, warm=warm,
                layout="crowded" if config.endswith("_crowded") else "grid",
                seconds=seconds, max_frames=6 if c4 else 1 << 30)
    c5 = config == "boosttrack_mot8"
    if c5:  # the workload's own eight sequences, one process each (MOT17-04 for one thread)
        one = run_cpu_workers([dict(base, seed=0, c5=1, threads=1)])[0]
        many = run_cpu_workers([dict(base, seed=0, c5=k, threads=1) for k in range(C5_TOTAL)])
    elif c4:
        one = run_cpu_workers([dict(base, seed=12345, threads=1)])[0]
        many = run_cpu_workers([dict(base, seed=12345, threads=P)])
    else:
        one = run_cpu_workers([dict(base, seed=12345, threads=1)])[0]
        many = run_cpu_workers([dict(base, seed=12345 + k, threads=1) for k in range(P)])
    fps1 = one["frames"] / one["busy"]
    fpsP = sum(r["frames"] / r["busy"] for r in many)
    # sequences are independent and the oracle is single-threaded per sequence, so the whole
    # machine's rate is the per-core rate times its usable CPUs (a projection, not a measurement)
    proj = None if (c4 or c5) else round(fpsP / P * host["usable_cpus"], 1)
    what = (f"{n_obj} objects (~{n_obj // 2} dets/frame)" + (f" x {emb_dim}-d" if emb_dim else ""))
    if c5:
        P = min(P, C5_TOTAL)
        what = "C5's 8 sequences (MOT17-02/04 public dets + 6 synthetic) x 512-d"
    ref = REFERENCE_CPU_FPS.get(config)
    return {
        "value": round(fpsP, 2), "unit": "frames/s", "cores": P, "kind": "port",
        "sample": (f"{'1 sequence, NN rows on' if c4 else f'{P} sequences, one process each on'}"
                   f" {P} cores; {what}; frames {warm + 1}..{many[0]['last']} per sequence, "
                   f"~{seconds:.0f}s busy each; oracle/ C fp64 port"),
        "host": host,
        "projected_all_usable_cpus": None if proj is None else {
            "value": proj, "cores": host["usable_cpus"],
            "note": "measured per-core rate x usable CPUs (linear: one process per sequence)"},
        "single_thread": {"value": round(fps1, 2), "cores": 1,
                          "sample": f"1 sequence, frames {one['first']}..{one['last']} "
                                    f"({one['frames']} timed, {one['busy']:.1f}s)"},
        "reference_python": None if ref is None else {
            "value": ref[0], "unit": "frames/s", "cores": 1, "workload": ref[1],
            "hardware": "survey container, Intel Xeon 8 vCPU, 1 core (BASELINE.md §2)"},
    }


def load_traffic(config, stage):
    """HBM bytes per launch of `stage` from the committed PMC summary (FETCH_SIZE x2 on gfx950
    + WRITE_SIZE, MI355X_MICROARCH.md §HBM), or None."""
    p = ROOT / "profiles" / f"pmc_{config}.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        return d.get("stages", {}).get(stage, {}).get("hbm_bytes_per_launch_corrected")
    except Exception:
        return None


def run_dropin(args):
    """The drop-in single-stream path: `create_tracker(kind).update(dets, img, embs)` per frame on
    one sequence, numpy inputs in host memory (how val.py and Ultralytics call the trackers), the
    wall time of the update calls only (input generation excluded).  One JSON line."""
    from boxmot_amd.synth import SyntheticScene
    from boxmot_amd.tracker_zoo import create_tracker

    kind, n_obj, F, params = CONFIGS[args.config]
    os.environ.setdefault("GITHUB_ACTIONS", "true")  # StrongSort born Confirmed, as its fixtures
    extra = dict(conf_lo=OCS_CONF_LO) if kind in ("ocsort", "boosttrack", "strongsort") else {}
    if kind in ("boosttrack", "strongsort"):
        extra["emb_dtype"] = np.float64
    sc = SyntheticScene(n_obj=n_obj, seed=777, emb_dim=F,
                        layout="crowded" if args.config.endswith("_crowded") else "grid", **extra)
    kw = {k: v for k, v in params.items() if k != "born_confirmed"}
    if kind == "strongsort":
        kw.update(handle_occlusions=False, **ss_caps(args.config, n_obj))
    tr = create_tracker(kind, evolve_param_dict=kw)
    img = np.zeros((1080, 1920, 3), np.uint8)
    frames = [sc.frame(t) for t in range(1, args.warmup + args.steps + 1)]
    for d, e, _ in frames[: args.warmup]:
        tr.update(d, img, e) if F else tr.update(d, img)
    t0 = time.perf_counter()
    for d, e, _ in frames[args.warmup:]:
        tr.update(d, img, e) if F else tr.update(d, img)
    wall = time.perf_counter() - t0
    mean_d = float(np.mean([f[0].shape[0] for f in frames[args.warmup:]]))
    ref = REFERENCE_CPU_FPS.get(args.config)
    line = {
        "metric": METRIC, "value": round(args.steps / wall, 1), "unit": "frames/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "none", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (numpy scenes in host memory, as the drop-in contract takes them)",
        "config": {"workload": f"{args.config} drop-in: one sequence x {n_obj} tracks x "
                               f"~{mean_d:.0f} dets" + (f" x {F}-d ReID" if F else "") +
                               ", tracker.update() per frame",
                   "tracker": kind, "n_seq_per_gpu": 1, "n_tracks": n_obj,
                   "n_dets_mean": round(mean_d, 1), "feat_dim": F, "parallelism": "single stream"},
        "roofline": {"bound": "latency", "note": "one sequence per call: launch and host<->device "
                                                 "latency bound, not an HBM/MFMA roofline"},
        "cpu_baseline": None if ref is None else {
            "value": ref[0], "unit": "frames/s", "cores": 1, "kind": "reference",
            "sample": f"the reference's Python tracker, {ref[1]}, survey container Intel Xeon "
                      f"(BASELINE.md §2)"},
    }
    print(json.dumps(line), flush=True)


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`python bench.py --gpus N` without a torch.distributed launcher: start N child processes of
    this script, one per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT
    in their environment; the reference's one-process-per-sequence-pool model, val.py:389-392),
    wait for all of them and print rank 0's JSON line.  This parent never imports torch.cuda or
    touches a GPU, and never execs: the children are ordinary subprocesses.  A failing rank ends
    the run: the others are killed (by their own Popen handles) and the exit code is non-zero."""
    import subprocess

    port = os.environ.get("MASTER_PORT") or str(free_port())
    argv = [sys.executable, "-u", str(Path(__file__).resolve())] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen(argv, env=env, stdout=subprocess.PIPE if r == 0 else None))
    out0 = procs[0].communicate()[0].decode()
    rc0 = procs[0].returncode
    rcs = [rc0]
    for p in procs[1:]:
        if rc0 != 0 and p.poll() is None:
            p.kill()
        rcs.append(p.wait())
    bad = [(r, c) for r, c in enumerate(rcs) if c != 0]
    sys.stdout.write(out0)
    sys.stdout.flush()
    if bad:
        sys.stderr.write(f"bench.py --gpus {n}: rank(s) failed {bad}\n")
        raise SystemExit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", choices=list(CONFIGS), default="botsort")
    ap.add_argument("--seqs", type=int, default=None,
                    help="sequences per GPU (default 1024; strongsort 256, strongsort_c4 1)")
    ap.add_argument("--chunk", type=int, default=0,
                    help="sequences per pipeline launch (0 = all; BoT-SORT/ByteTrack)")
    ap.add_argument("--track-cap", type=int, default=512,
                    help="BoT-SORT/ByteTrack engine track slots per sequence")
    ap.add_argument("--det-cap", type=int, default=256,
                    help="BoT-SORT/ByteTrack engine detection slots per sequence")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--with-d2h", action="store_true",
                    help="deliver every frame's output rows to pinned host memory inside the "
                         "timed region (a side-stream copy per frame, overlapped with the next "
                         "frame), as motio.run_sequences users receive them")
    ap.add_argument("--early-features", action="store_true",
                    help="BoT-SORT: each frame's detection-feature kernel starts on its own "
                         "stream beside the previous frame's tail (bx_engine_set_early_features; "
                         "the frames are resident before timing)")
    ap.add_argument("--lsap-exact", action="store_true",
                    help="StrongSort: solve every LSAP in scipy's row order (bx_ss_set_lsap_mode "
                         "0) instead of solve + certify")
    ap.add_argument("--no-overlap", action="store_true",
                    help="join each step's feature EMA before it returns (bx_engine_set_overlap off)")
    ap.add_argument("--start-frame", type=int, default=0,
                    help="first timed frame (raises the warm-up so the timed frames start there: "
                         "StrongSort C4 at gallery steady state)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-worker", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--dropin", action="store_true",
                    help="time the drop-in tracker.update() on one sequence instead")
    args = ap.parse_args()
    if args.cpu_worker:
        print(json.dumps(cpu_worker(json.loads(args.cpu_worker))), flush=True)
        return
    if args.dropin:
        return run_dropin(args)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus)  # this process stays off the GPU

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting {world} ranks",
              file=sys.stderr)
    dist = None
    backend = os.environ.get("BX_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI on ROCm
    if world > 1:
        import torch.distributed as dist

        ndev = torch.cuda.device_count()  # counts devices without initialising one
        if backend == "nccl" and world > ndev:
            # RCCL: one rank per GPU, no oversubscription (gloo keeps the 1-GPU modulo rehearsal)
            print(f"bench.py: {world} ranks over RCCL need {world} GPUs, {ndev} visible",
                  file=sys.stderr)
            raise SystemExit(3)
        if ndev == 0:
            raise SystemExit("bench.py: no HIP device visible")
        # one process per GPU; modulo only so a 1-GPU rehearsal (gloo) can run 2 ranks
        torch.cuda.set_device(local % ndev)
        dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from boxmot_amd.shard import gather_records, output_checksum, shard_sequences
    from boxmot_amd.workloads import BenchFrames, bench_engine

    kind, n_obj, F, params = CONFIGS[args.config]
    S = args.seqs if args.seqs is not None else DEFAULT_SEQS.get(args.config, 1024)
    c5 = args.config == "boosttrack_mot8"
    # the input stream and the engine (shared with tests/test_bench_workload.py, which checks
    # this exact workload against the oracle); C5: this rank's LPT shard of its 8 sequences
    src = BenchFrames(args.config, S, dev, rank, world)
    S = src.n_seq
    c5_mine = src.mine
    ocs = kind == "ocsort"
    bst = kind == "boosttrack"
    sss = kind == "strongsort"
    eng, stages = bench_engine(args.config, S, args.track_cap, args.det_cap,
                               overlap=not args.no_overlap, early=args.early_features)
    layout = src.layout
    if sss and args.lsap_exact:
        eng.set_lsap_mode(False)
    # W warm-up steps (at least start_frame - 1 - probes: the first timed frame), then one
    # untimed probe step per pipeline stage, then the K timed steps.  The stages are probed on
    # the last 2 x stages untimed steps (warm-up ones included), each twice, the larger kept: one
    # event pair beside a concurrent side stream can read short
    n_probe = len(stages)
    warmup = max(args.warmup, args.start_frame - 1 - n_probe)
    t_first = warmup + n_probe
    n_pr = min(2 * n_probe, t_first)
    total = t_first + args.steps
    # after the timed steps, one more probe step per stage: the stages at the timed frames' state
    # (StrongSort's galleries, for one, are still filling during the early probes)
    n_frames = total + n_probe
    if c5 and n_frames > src.n_frames_max:
        raise SystemExit("boosttrack_mot8: warmup + probes + steps exceed the shortest "
                         "sequence (600 frames)")
    frames = [src.frame(t) for t in range(1, n_frames + 1)]  # resident in HBM before timing
    n_rows = [int(f[1][-1].item()) for f in frames]  # detections per frame (host, pre-timing)
    max_n = max(n_rows)
    width = 10 if kind == "strongsort" else 8
    out = torch.empty((max_n, width), dtype=torch.float64, device=dev)
    cnt = torch.empty(S, dtype=torch.int32, device=dev)
    # --with-d2h: a ring of output buffers, each frame's rows (and per-sequence counts) copied to
    # pinned host memory on a side stream while the next frame computes; a buffer is rewritten
    # only after its copy completed (event), so no frame's rows are lost or torn
    RING = 3
    d2h = None
    if args.with_d2h:
        d2h = dict(
            outs=[torch.empty((max_n, width), dtype=torch.float64, device=dev)
                  for _ in range(RING)],
            cnts=[torch.empty(S, dtype=torch.int32, device=dev) for _ in range(RING)],
            host=[torch.empty((max_n, width), dtype=torch.float64, pin_memory=True)
                  for _ in range(RING)],
            hcnt=[torch.empty(S, dtype=torch.int32, pin_memory=True) for _ in range(RING)],
            side=torch.cuda.Stream(device=dev),
            done=[None] * RING, bytes=0)
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()

    # sequences per launch: the frame pipeline runs over sequence chunks one after the other, so
    # that a chunk's feature rows and Kalman state are re-read from the 256 MiB Infinity Cache
    # by its later kernels instead of from HBM (BoT-SORT / ByteTrack engines)
    chunk = args.chunk if (args.chunk and not (ocs or bst or sss)) else S
    bounds = [(c0, min(c0 + chunk, S)) for c0 in range(0, S, chunk)]

    def step(k):
        if d2h is not None:
            return step_d2h(k)
        d, off, e = frames[k]
        if ocs:
            eng.step(d, off, out, cnt, stream=stream.cuda_stream)
        elif bst or sss:
            eng.step(d, off, e, None, out, cnt, stream=stream.cuda_stream)
        else:
            for c0, c1 in bounds:
                eng.step(d, off[c0:c1 + 1], e, None, out, cnt[c0:c1], seq0=c0, nseq=c1 - c0,
                         stream=stream.cuda_stream)

    def step_d2h(k):
        nonlocal out, cnt
        slot = k % RING
        if d2h["done"][slot] is not None:
            stream.wait_event(d2h["done"][slot])  # this buffer's previous copy has landed
        out, cnt = d2h["outs"][slot], d2h["cnts"][slot]
        d, off, e = frames[k]
        if ocs:
            eng.step(d, off, out, cnt, stream=stream.cuda_stream)
        elif bst or sss:
            eng.step(d, off, e, None, out, cnt, stream=stream.cuda_stream)
        else:
            for c0, c1 in bounds:
                eng.step(d, off[c0:c1 + 1], e, None, out, cnt[c0:c1], seq0=c0, nseq=c1 - c0,
                         stream=stream.cuda_stream)
        ev = torch.cuda.Event()
        ev.record(stream)
        side = d2h["side"]
        side.wait_event(ev)
        n = n_rows[k]
        with torch.cuda.stream(side):
            d2h["host"][slot][:n].copy_(out[:n], non_blocking=True)
            d2h["hcnt"][slot].copy_(cnt, non_blocking=True)
            done = torch.cuda.Event()
            done.record(side)
        d2h["done"][slot] = done
        d2h["bytes"] += n * width * 8 + S * 4

    # warm-up, then the probe steps: each times one stage to find the dominant kernel
    stage_ms = {}
    for k in range(t_first):
        j = k - (t_first - n_pr)
        if j >= 0:
            eng.probe(stages[j % n_probe])
        step(k)
        if j >= 0:
            ms, n = eng.probe_read()
            # the stage's launches of one step (one per chunk), the larger of its two probes
            stage_ms[stages[j % n_probe]] = max(ms, stage_ms.get(stages[j % n_probe], 0.0))
            eng.probe(None)
    # (StrongSort's "pre" probe spans its side-stream branch — crowd test, pre kernel, detection
    # sort — from events that also wait for the gallery distance's waves beside it: 0.15-0.18 ms
    # probed against ~45 us of kernels in the trace at 256 sequences, so it is not a candidate)
    cand = {k: v for k, v in stage_ms.items() if not (sss and k == "pre")}
    dominant = max(cand, key=cand.get) if cand else (
        "ocsort_frame" if ocs else ("features" if F else "assoc"))
    # StrongSort: the roofline kernel is the gallery distance, its one matrix-core kernel and the
    # largest at the timed frames (stage_ms_after_timed); the probes run on the first frames,
    # while the galleries are still filling (C4 at frames 11-19: nn 0.36 ms against the match's
    # 0.38; at frames 20-69 0.56-0.58 ms)
    if sss and "nn" in stage_ms:
        dominant = "nn"
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # two event records per step around the dominant stage's launch (OCSort: its one kernel)
    eng.probe(True if ocs else dominant)
    if d2h is not None:
        d2h["bytes"] = 0
    t0 = time.perf_counter()
    for k in range(t_first, total):
        step(k)
    torch.cuda.synchronize()  # (every stream of the device: the side-stream copies included)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    d2h_bytes = d2h["bytes"] if d2h is not None else 0
    dom_ms, dom_n = eng.probe_read()
    eng.probe(False if ocs else None)
    dom_ms /= args.steps  # per step: the dominant stage's launches over all chunks
    if eng.status() != 0:
        raise RuntimeError(f"engine status {eng.status()} (capacity overflow)")
    units = eng.frame_stats()  # last timed frame, all sequences of this rank
    if ocs:
        units["dets"] = int(frames[total - 1][1][-1].item())
    emb_bytes = 8 if bst or sss else 4
    if sss:
        units["seqs"] = S
        # distinct gallery samples compared per queried track at the last timed frame
        units["rows_per_queried_track"] = round(units["rows"] / max(units["queried"], 1), 2)
        # LSAPs solved (all frames of this rank): certified unique / unique up to rejected pairs
        # / ties re-solved in scipy's order / cascade stages restarted
        units["lsap_all_frames"] = eng.lsap_stats()
    if kind in ("bytetrack", "botsort"):
        # associations whose optimum was tied, re-solved in lapx's JV order, summed
        # over all frames of this rank
        units["lap_ties_all_frames"] = eng.lap_ties()

    # per-sequence records of this rank's shard: [global seq id, frames timed, dets timed,
    # rows of the last frame, checksum of the last frame, rank wall s, dominant-stage ms]
    off_h = [frames[k][1].cpu().numpy() for k in range(t_first, total)]
    dets_seq = np.sum([np.diff(o) for o in off_h], 0)
    last_off, cnt_h, out_h = off_h[-1], cnt.cpu().numpy(), out.cpu().numpy()
    # untimed, after the timed region and its outputs: one probe step per stage at the timed
    # frames' state (StrongSort's galleries, for one, are still filling during the early probes)
    stage_ms_late = {}
    for j in range(n_probe):
        eng.probe(stages[j])
        step(total + j)
        stage_ms_late[stages[j]] = eng.probe_read()[0]
        eng.probe(None)
    torch.cuda.synchronize()
    recs = np.zeros((S, 7))
    for i, g in enumerate(c5_mine if c5 else shard_sequences(S * world, world, rank)):
        rows_i = out_h[last_off[i]: last_off[i] + cnt_h[i]]
        recs[i] = [g, args.steps, dets_seq[i], cnt_h[i], output_checksum(rows_i), wall, dom_ms]
    # RCCL over xGMI only to gather these KB-scale records once, never per frame
    allrec = gather_records(recs, dist, dev if backend == "nccl" else "cpu")
    t_max = float(allrec[:, 5].max())
    total_frames = float(allrec[:, 1].sum())
    value = total_frames / t_max
    if rank == 0:
        n_all = C5_TOTAL if c5 else S * world
        assert np.array_equal(np.sort(allrec[:, 0]), np.arange(n_all)), "shard gather"
        mean_d = float(allrec[:, 2].sum() / allrec[:, 1].sum())
        if ocs:
            per_launch = (units["tracks"] * OCS_TRACK_BYTES + units["dets"] * 24 +
                          units["outputs"] * 64)
        elif bst:
            per_launch = boost_stage_bytes(dominant, units, F)
        elif sss:
            per_launch = ss_stage_bytes(dominant, units, F)
        else:
            per_launch = stage_bytes(dominant, units, F)
        achieved = per_launch / (dom_ms * 1e-3) / 1e9
        traffic = load_traffic(args.config, dominant)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic}
        if sss and dominant == "nn":
            # the gallery distance is fp64 matrix-core work: 2 x sample rows x detections x F
            # per launch against the measured dense fp64 MFMA rate
            flops = 2.0 * units["rows"] * (units["dets"] / max(units["seqs"], 1)) * F
            tf = flops / (dom_ms * 1e-3) / 1e12
            roof = {"bound": "mfma", "achieved": round(tf, 2), "peak": F64_MFMA_PEAK_TFS,
                    "unit": "TFLOP/s", "frac": round(tf / F64_MFMA_PEAK_TFS, 4),
                    "peak_measured": F64_MFMA_MEASURED_TFS,
                    "frac_of_measured": round(tf / F64_MFMA_MEASURED_TFS, 4),
                    "traffic": traffic, "algorithmic_flops_per_launch": int(flops)}
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong" if c5 else "weak", "vs_baseline": None, "dtype": "f64",
            "data": ("MOT17-02/04 public detections (tests/golden/mot17_public_dets.npz) with "
                     "identity-linked synthetic ReID + 6 synthetic sequences, resident in HBM "
                     "before timing" if c5 else
                     f"synthetic (GPU-generated {layout} scenes, resident in HBM before timing)"),
            "config": {"workload": (f"{args.config}: 8 sequences (MOT17-02, MOT17-04, 6 synthetic"
                                    f" 60-object) sharded over {world} GPU(s), {S} on rank 0, "
                                    f"~{mean_d:.0f} dets x {F}-d ReID" if c5 else
                                    f"{args.config}: {S} sequences/GPU x {n_obj} tracks x "
                                    f"~{mean_d:.0f} dets" + (f" x {F}-d ReID" if F else "")),
                       "tracker": kind, "n_seq_per_gpu": S, "n_tracks": n_obj,
                       "n_dets_mean": round(mean_d, 1), "feat_dim": F,
                       "emb_dtype": "f64" if emb_bytes == 8 else "f32",
                       "parallelism": f"seq-sharded x{world}",
                       "sequences_gathered": int(allrec.shape[0]),
                       **({"last_frame_checksums": {str(int(g)): c for g, c in
                                                    sorted(zip(allrec[:, 0], allrec[:, 4]))}}
                          if c5 else {}),
                       "dist_backend": backend if world > 1 else None,
                       "timed_frames": [t_first + 1, total],
                       **({"feature_overlap": not args.no_overlap,
                           "early_features": bool(args.early_features)}
                          if kind == "botsort" and F else {}),
                       **({"outputs_to_host": {
                           "what": "every frame's output rows + per-sequence counts copied to "
                                   "pinned host memory on a side stream inside the timed region",
                           "bytes_per_step": round(d2h_bytes / args.steps),
                           "GB_s": round(d2h_bytes / t_max / 1e9, 2)}} if d2h is not None else
                          {})},
            "roofline": {**roof, "kernel": dominant,
                         "kernel_ms": round(dom_ms, 4), "probe_steps": n_pr,
                         "launches_per_step": len(bounds),
                         "algorithmic_bytes_per_launch": int(per_launch),
                         "units_last_frame": units,
                         "stage_ms_probe": {k: round(v, 4) for k, v in stage_ms.items()},
                         "stage_ms_after_timed": {k: round(v, 4)
                                                  for k, v in stage_ms_late.items()}},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.config, kind, n_obj, F, params,
                                                args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
