"""The workloads bench.py times, at their bench shape, checked against the oracle.

Every other parity test drives the engines with `SyntheticScene` streams of a few sequences at
test capacities.  These drive exactly what `bench.py` times — `workloads.BenchFrames` (the GPU
`TorchSceneBatch` generator, or C5's eight MOT17 / synthetic sequences) into
`workloads.bench_engine` (bench capacities, BoT-SORT overlap mode), with the bench's probe
schedule (W warm-up steps, one probe step per stage, the dominant stage probed on every later
step) and no host synchronisation between steps — and compare sampled sequences, spread over
the batch, every frame bitwise with the C oracle fed the same device-generated inputs, then
their Kalman state at the end.

* C3 `botsort` (the driver-timed line): 1024 sequences, track_cap 512 / det_cap 256, overlap
  mode, 60 frames (`trackers/botsort/botsort.py:94-166`).
* C4 `strongsort_c4`: 1 sequence x 1024 objects x 2048-d at `SS_C4_CAPS`, 64 frames — past the
  frame where the galleries' distinct samples per track stop growing
  (`sort/linear_assignment.py:555-600`, `sort/tracker.py:166-178`).
* C5 `boosttrack_mot8`: the 8 sequences on one GPU, 100 frames (`boosttrack.py:221-336`).
"""
import numpy as np
import pytest

from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected without a HIP device")
    from boxmot_amd import _native

    _native.load()  # the in-tree HIP library, never a fallback
    return torch


def drive_bench(torch, config, n_seq, n_frames, warmup=10, track_cap=512, det_cap=256,
                lap_stats=False, assoc_build=-1, early=False):
    """Run `n_frames` steps of bench.py's workload for `config` the way bench.py runs them (probe
    schedule included, one launch per frame over every sequence, no host sync in between).
    Returns (engine, frames on device, per-frame (out, cnt) on device)."""
    from boxmot_amd.workloads import CONFIGS, BenchFrames, bench_engine

    kind = CONFIGS[config][0]
    dev = torch.device("cuda", 0)
    src = BenchFrames(config, n_seq, dev)
    eng, stages = bench_engine(config, src.n_seq, track_cap, det_cap, overlap=True, early=early)
    if lap_stats:
        eng.set_lap_stats(True)
    if assoc_build != -1:
        eng.force_assoc_build(assoc_build)
    S = src.n_seq
    stream = torch.cuda.current_stream()
    width = 10 if kind == "strongsort" else 8
    frames, outs = [], []
    dominant = stages[-1] if stages else None
    if early:  # the early-features contract: inputs complete when each step is called
        pre = [src.frame(t) for t in range(1, n_frames + 1)]
        torch.cuda.synchronize()
    for t in range(1, n_frames + 1):
        d, off, e = pre[t - 1] if early else src.frame(t)
        frames.append((d, off, e))
        j = t - 1 - warmup
        probed = None
        if stages and 0 <= j < len(stages):
            probed = stages[j]
        elif stages and j == len(stages):
            probed = dominant
        if probed is not None:
            eng.probe(probed)
        out = torch.empty((max(int(d.shape[0]), 1), width), dtype=torch.float64, device=dev)
        cnt = torch.empty(S, dtype=torch.int32, device=dev)
        if kind == "ocsort":
            eng.step(d, off, out, cnt, stream=stream.cuda_stream)
        elif kind in ("boosttrack", "strongsort"):
            eng.step(d, off, e, None, out, cnt, stream=stream.cuda_stream)
        else:
            eng.step(d, off, e, None, out, cnt, seq0=0, nseq=S, stream=stream.cuda_stream)
        outs.append((out, cnt))
        if probed is not None and j < len(stages):
            eng.probe_read()
            eng.probe(None)
    torch.cuda.synchronize()
    assert eng.status() == 0
    return eng, frames, outs


def host_rows(frames, outs, s, t):
    """(dets, embs, engine rows) of sequence s at frame t (1-based), on the host."""
    d, off, e = frames[t - 1]
    out, cnt = outs[t - 1]
    o = off.cpu().numpy()
    a, b = int(o[s]), int(o[s + 1])
    dets = d[a:b].cpu().numpy().astype(np.float64)
    embs = None if e is None else e[a:b].cpu().numpy()
    rows = out[a: a + int(cnt[s].item())].cpu().numpy()
    return dets, embs, rows


@pytest.mark.parametrize("early", [False, True])
def test_botsort_c3_bench_workload_vs_oracle(torch_cuda, early):
    """The driver-timed line (BASELINE configs[2]): 1024 sequences in one launch per frame at
    bench capacities in overlap mode (and in early-features mode: each frame's K1 on its own
    stream beside the previous frame's tail, the norms double-buffered); 8 sequences spread over
    the batch (first, last, both halves' edges) bitwise against the oracle every frame, and their
    Kalman state at the end."""
    from boxmot_amd.workloads import CONFIGS

    _, _, F, params = CONFIGS["botsort"]
    n_frames = 60
    eng, frames, outs = drive_bench(torch_cuda, "botsort", 1024, n_frames, early=early)
    st = eng.frame_stats()
    assert st["dets"] > 1024 * 100 and st["active"] > 1024 * 100, st  # the C3 shape, really
    for s in (0, 1, 255, 511, 512, 700, 1022, 1023):
        orc = po.OracleTracker("botsort", **params)
        for t in range(1, n_frames + 1):
            dets, embs, rows = host_rows(frames, outs, s, t)
            assert embs.dtype == np.float32 and embs.shape[1] == F
            np.testing.assert_array_equal(rows, orc.update(dets, embs),
                                          err_msg=f"seq {s} frame {t}")
        g, r = eng.tracks(s), orc.tracks()
        for k in ("id", "state", "mean", "covariance"):
            np.testing.assert_array_equal(g[k], r[k], err_msg=f"seq {s} {k}")


@pytest.mark.timeout(600)
def test_strongsort_c4_bench_workload_vs_oracle(torch_cuda):
    """BASELINE configs[3] as bench.py times it (TorchSceneBatch seed 1000, 1024 objects, 2048-d,
    SS_C4_CAPS) for 64 frames — past the frame where the distinct gallery samples per track
    level off — every frame's rows and the final Kalman state bitwise against the oracle."""
    from boxmot_amd.workloads import CONFIGS

    _, _, F, params = CONFIGS["strongsort_c4"]
    n_frames = 64
    eng, frames, outs = drive_bench(torch_cuda, "strongsort_c4", 1, n_frames)
    st = eng.frame_stats()
    assert st["dets"] > 450 and st["tracks"] > 900, st
    ls = eng.lsap_stats()
    print(f"C4 LSAPs over {n_frames} frames: {ls}")
    assert ls["unique"] + ls["unique_up_to_rejected"] > 0, ls  # solve + certify really ran
    orc = po.OracleTracker("strongsort", **params)
    for t in range(1, n_frames + 1):
        dets, embs, rows = host_rows(frames, outs, 0, t)
        assert dets.shape[1] == 6 and embs.shape[1] == F
        np.testing.assert_array_equal(rows, orc.update(dets, embs), err_msg=f"frame {t}")
    L = po.lib()
    g = eng.tracks(0)
    n = L.bxo_ss_tracks(orc.h, 0, None, None, None, None)
    ids = np.zeros(max(n, 1), np.int32)
    state = np.zeros(max(n, 1), np.int32)
    mean = np.zeros((max(n, 1), 8))
    cov = np.zeros((max(n, 1), 8, 8))
    L.bxo_ss_tracks(orc.h, n, ids.ctypes.data, state.ctypes.data, mean.ctypes.data,
                    cov.ctypes.data)
    np.testing.assert_array_equal(g["id"], ids[:n])
    np.testing.assert_array_equal(g["state"], state[:n])
    np.testing.assert_array_equal(g["mean"], mean[:n])
    np.testing.assert_array_equal(g["covariance"], cov[:n])


def test_boosttrack_c5_bench_workload_vs_oracle(torch_cuda):
    """BASELINE configs[4] (`boosttrack_mot8`) on one GPU: its 8 sequences (MOT17-02/04 public
    detections + 6 synthetic) in one launch per frame, 100 frames, all 8 bitwise against the
    oracle every frame and their Kalman state at the end."""
    from boxmot_amd.workloads import CONFIGS

    _, _, F, params = CONFIGS["boosttrack_mot8"]
    n_frames = 100
    eng, frames, outs = drive_bench(torch_cuda, "boosttrack_mot8", 8, n_frames)
    L = po.lib()
    for s in range(8):
        orc = po.OracleTracker("boosttrack", **params)
        for t in range(1, n_frames + 1):
            dets, embs, rows = host_rows(frames, outs, s, t)
            assert embs.dtype == np.float64 and embs.shape[1] == F
            np.testing.assert_array_equal(rows, orc.update(dets, embs),
                                          err_msg=f"seq {s} frame {t}")
        g = eng.tracks(s)
        n = L.bxo_boost_tracks(orc.h, 0, None, None, None)
        ids = np.zeros(max(n, 1), np.int32)
        x = np.zeros((max(n, 1), 8))
        P = np.zeros((max(n, 1), 8, 8))
        L.bxo_boost_tracks(orc.h, n, ids.ctypes.data, x.ctypes.data, P.ctypes.data)
        np.testing.assert_array_equal(g["id"], ids[:n], err_msg=f"seq {s}")
        np.testing.assert_array_equal(g["x"], x[:n], err_msg=f"seq {s}")
        np.testing.assert_array_equal(g["P"], P[:n], err_msg=f"seq {s}")


def _compare_sampled(torch, config, n_seq, n_frames, sample, kf_keys, oracle_state):
    """Drive ``config`` at its bench shape and compare the sampled sequences bitwise with the
    oracle every frame, then their Kalman state (``oracle_state(orc)`` vs ``eng.tracks(s)``)."""
    from boxmot_amd.workloads import CONFIGS

    kind, _, F, params = CONFIGS[config]
    eng, frames, outs = drive_bench(torch, config, n_seq, n_frames)
    for s in sample:
        orc = po.OracleTracker(kind, **params)
        for t in range(1, n_frames + 1):
            dets, embs, rows = host_rows(frames, outs, s, t)
            exp = orc.update(dets, embs if F else None)
            np.testing.assert_array_equal(rows, exp, err_msg=f"{config} seq {s} frame {t}")
        g, r = eng.tracks(s), oracle_state(orc)
        for k in kf_keys:
            np.testing.assert_array_equal(g[k], r[k], err_msg=f"{config} seq {s} {k}")
    return eng


def test_botsort_crowded_bench_workload_vs_oracle(torch_cuda):
    """SURVEY §8(d)'s crowded variant of C3 (`botsort_crowded`) as bench.py times it: 1024
    sequences x 256 objects on the crowded layout, caps 512/256, overlap mode, 60 frames.  The
    sparse LAP (matching.py:30-108 restated) must have handed components to its
    per-lane SSP (past the register path) and components of more than 3 rows to its wave SSP
    (on the helper waves 1..3 when a LAP has more than 32 roots, else on wave 0) somewhere in
    the batch; the sampled sequences are spread over the batch (0, 511, 1023, ...) plus the ones
    with the most components on each of those two paths, all bitwise vs the oracle every frame
    (botsort.py:200-250) and in their final Kalman state."""
    from boxmot_amd.workloads import CONFIGS

    kind, _, F, params = CONFIGS["botsort_crowded"]
    n_frames = 60
    eng, frames, outs = drive_bench(torch_cuda, "botsort_crowded", 1024, n_frames, lap_stats=True)
    tot = eng.lap_components()
    assert tot["lane"] > 0 and tot["wave"] > 0, tot
    per = [eng.lap_components(s, 1) for s in range(1024)]
    lane_s = max(range(1024), key=lambda s: per[s]["lane"])
    wave_s = max(range(1024), key=lambda s: per[s]["wave"])
    both = [s for s in range(1024) if per[s]["lane"] and per[s]["wave"]]
    sample = sorted({0, 1, 511, 512, 1023, lane_s, wave_s, *(both[:1])})
    assert per[lane_s]["lane"] > 0 and per[wave_s]["wave"] > 0
    print(f"crowded LAP components: {tot}; sampled {sample}")
    for s in sample:
        orc = po.OracleTracker(kind, **params)
        for t in range(1, n_frames + 1):
            dets, embs, rows = host_rows(frames, outs, s, t)
            np.testing.assert_array_equal(rows, orc.update(dets, embs),
                                          err_msg=f"crowded seq {s} frame {t}")
        g, r = eng.tracks(s), orc.tracks()
        for k in ("id", "state", "mean", "covariance"):
            np.testing.assert_array_equal(g[k], r[k], err_msg=f"crowded seq {s} {k}")


def test_botsort_crowded_forced_assoc_builds_identical(torch_cuda):
    """The association kernel ships in two builds (wave 0 only / helper waves 1..3 for the wave
    SSP), picked per launch from a device cue (bx_engine_force_assoc_build -1).  Forced to each
    build for the whole run, the crowded C3 workload (60 frames, 1024 sequences) gives the same
    output rows in every sequence on every frame and the same final Kalman state; the helper
    build really solved components on waves 1..3 (comp_stats helper > 0) and the wave-0 build
    none; and the sequences with the most helper-solved components equal the oracle bitwise."""
    from boxmot_amd.workloads import CONFIGS

    torch = torch_cuda
    kind, _, F, params = CONFIGS["botsort_crowded"]
    n_frames = 60
    runs = {}
    for b in (0, 1):
        eng, frames, outs = drive_bench(torch, "botsort_crowded", 1024, n_frames, lap_stats=True,
                                        assoc_build=b)
        runs[b] = (eng, frames, outs, eng.lap_components())
    (e0, f0, o0, c0), (e1, f1, o1, c1) = runs[0], runs[1]
    print(f"forced builds: wave-0 {c0}, helper {c1}")
    assert c0["helper"] == 0 and c0["wave"] > 0, c0
    assert c1["helper"] > 0 and c1["helper"] <= c1["wave"], c1
    assert c0["wave"] == c1["wave"] and c0["lane"] == c1["lane"], (c0, c1)
    for t in range(n_frames):
        off = f0[t][1]
        assert torch.equal(off, f1[t][1])
        assert torch.equal(o0[t][1], o1[t][1]), f"counts differ at frame {t + 1}"
        # the rows each sequence wrote: [off[s], off[s] + cnt[s]) (the rest of its slice is unset)
        n = int(off[-1].item())
        idx = torch.arange(n, device=off.device)
        sq = torch.searchsorted(off[1:].long(), idx, right=True)
        valid = (idx - off[sq]) < o0[t][1].long()[sq]
        assert torch.equal(o0[t][0][:n][valid], o1[t][0][:n][valid]), f"rows differ, frame {t + 1}"
    for s in range(0, 1024, 97):
        g0, g1 = e0.tracks(s), e1.tracks(s)
        for k in ("id", "state", "mean", "covariance"):
            np.testing.assert_array_equal(g0[k], g1[k], err_msg=f"seq {s} {k}")
    per = [e1.lap_components(s, 1)["helper"] for s in range(1024)]
    top = sorted(range(1024), key=lambda s: -per[s])[:3]
    assert per[top[0]] > 0
    for s in top:
        orc = po.OracleTracker(kind, **params)
        for t in range(1, n_frames + 1):
            dets, embs, rows = host_rows(f1, o1, s, t)
            np.testing.assert_array_equal(rows, orc.update(dets, embs),
                                          err_msg=f"helper build seq {s} frame {t}")


def test_bytetrack_c2_bench_workload_vs_oracle(torch_cuda):
    """BASELINE configs[1] (`bytetrack`) as bench.py times it: 1024 sequences x 256 objects,
    caps 512/256, 60 frames; 8 sequences bitwise vs the oracle every frame
    (bytetrack.py:158-302) and in their final Kalman state."""
    _compare_sampled(torch_cuda, "bytetrack", 1024, 60, (0, 1, 255, 511, 512, 700, 1022, 1023),
                     ("id", "state", "mean", "covariance"), lambda o: o.tracks())


def test_ocsort_bench_workload_vs_oracle(torch_cuda):
    """The `ocsort` bench line (configs[0]'s tracker at 1024 sequences x ~40 objects, YAML
    defaults), 60 frames; 8 sequences bitwise vs the oracle every frame (ocsort.py:246-439) and
    in their final XYSR Kalman state."""
    _compare_sampled(torch_cuda, "ocsort", 1024, 60, (0, 1, 255, 511, 512, 700, 1022, 1023),
                     ("id", "x", "P"), lambda o: o.ocsort_tracks())


def _boost_state(orc):
    L = po.lib()
    n = L.bxo_boost_tracks(orc.h, 0, None, None, None)
    ids = np.zeros(max(n, 1), np.int32)
    x = np.zeros((max(n, 1), 8))
    P = np.zeros((max(n, 1), 8, 8))
    L.bxo_boost_tracks(orc.h, n, ids.ctypes.data, x.ctypes.data, P.ctypes.data)
    return {"id": ids[:n], "x": x[:n], "P": P[:n]}


def test_boosttrack_c2_bench_workload_vs_oracle(torch_cuda):
    """The `boosttrack` bench line (BoostTrack++ at 1024 sequences x 60 objects x 512-d f64: two
    waves per sequence at this launch width), 40 frames; 4 sequences bitwise vs the oracle
    every frame (boosttrack.py:221-336) and in their final Kalman state."""
    _compare_sampled(torch_cuda, "boosttrack", 1024, 40, (0, 511, 512, 1023), ("id", "x", "P"),
                     _boost_state)


def _ss_state(orc):
    L = po.lib()
    n = L.bxo_ss_tracks(orc.h, 0, None, None, None, None)
    ids = np.zeros(max(n, 1), np.int32)
    st = np.zeros(max(n, 1), np.int32)
    mean = np.zeros((max(n, 1), 8))
    cov = np.zeros((max(n, 1), 8, 8))
    L.bxo_ss_tracks(orc.h, n, ids.ctypes.data, st.ctypes.data, mean.ctypes.data, cov.ctypes.data)
    return {"id": ids[:n], "state": st[:n], "mean": mean[:n], "covariance": cov[:n]}


def test_strongsort_256_bench_workload_vs_oracle(torch_cuda):
    """The `strongsort` bench line (256 sequences x 48 objects x 512-d), 40 frames; 4 sequences
    bitwise vs the oracle every frame (strongsort.py:120-181, sort/tracker.py:183-298) and in
    their final Kalman state."""
    _compare_sampled(torch_cuda, "strongsort", 256, 40, (0, 127, 128, 255),
                     ("id", "state", "mean", "covariance"), _ss_state)
