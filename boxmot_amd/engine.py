"""Python handle over the native engine (``bx_engine_*`` in include/bxassoc.h).

An ``Engine`` holds ``n_seq`` independent sequences resident in HBM.  ``step`` advances one frame
of a contiguous range of sequences in a single kernel launch (device tensors in, device tensors
out); ``update_host`` is the single-sequence numpy path the drop-in tracker classes use.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _native as N

KINDS = {"bytetrack": 0, "botsort": 1}


@dataclass
class EngineParams:
    """Tracker parameters with the reference constructors' defaults."""

    # ByteTrack (bytetrack.py:132-140)
    min_conf: float = 0.1
    track_thresh: float = 0.45
    match_thresh: float = 0.8
    track_buffer: int | None = None  # None → the tracker's own default: 25 ByteTrack, 30 BoT-SORT
    frame_rate: int = 30
    # BoT-SORT (botsort.py:49-66)
    track_high_thresh: float = 0.5
    track_low_thresh: float = 0.1
    new_track_thresh: float = 0.6
    proximity_thresh: float = 0.5
    appearance_thresh: float = 0.25
    fuse_first_associate: bool = False
    with_reid: bool = True


class Engine:
    def __init__(self, kind: str, n_seq: int = 1, track_cap: int = 1024, det_cap: int = 384,
                 emb_dim: int = 0, emb_f64: bool = False, params: EngineParams | None = None):
        if kind not in KINDS:
            raise KeyError(kind)
        p = params or EngineParams()
        if p.track_buffer is None:
            p = EngineParams(**{**p.__dict__, "track_buffer": 25 if kind == "bytetrack" else 30})
        self.kind, self.n_seq, self.track_cap, self.det_cap = kind, n_seq, track_cap, det_cap
        self.emb_dim, self.emb_f64, self.params = emb_dim, bool(emb_f64), p
        self.with_reid = kind == "botsort" and p.with_reid
        cfg = N.BxConfig(
            kind=KINDS[kind], n_seq=n_seq, track_cap=track_cap, det_cap=det_cap,
            emb_dim=emb_dim if self.with_reid else 0, emb_f64=int(emb_f64),
            min_conf=p.min_conf, track_thresh=p.track_thresh, match_thresh=p.match_thresh,
            track_buffer=int(p.track_buffer), frame_rate=int(p.frame_rate),
            track_high_thresh=p.track_high_thresh, track_low_thresh=p.track_low_thresh,
            new_track_thresh=p.new_track_thresh, proximity_thresh=p.proximity_thresh,
            appearance_thresh=p.appearance_thresh,
            fuse_first_associate=int(bool(p.fuse_first_associate)), with_reid=int(self.with_reid))
        self._L = N.load()
        self._overlap, self._inflight = False, None
        h = C.c_void_p()
        N.check(self._L.bx_engine_create(C.byref(cfg), C.byref(h)), "bx_engine_create")
        self._h = h

    # ----------------------------------------------------------------------------- lifecycle
    def close(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.bx_engine_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, seq0: int = 0, nseq: int | None = None, stream: int | None = None):
        nseq = self.n_seq - seq0 if nseq is None else nseq
        N.check(self._L.bx_engine_reset(self._h, seq0, nseq, stream), "bx_engine_reset")

    # ------------------------------------------------------------------------------- frames
    def step(self, dets, det_off, embs=None, warps=None, out=None, out_count=None, seq0: int = 0,
             nseq: int | None = None, stream=None):
        """One frame for sequences [seq0, seq0+nseq): torch device tensors (or raw pointers).

        dets [sum N,6] float32, det_off [nseq+1] int32, embs [sum N,F] float32/64 or None,
        warps [nseq,6] float64 or None, out [sum N,8] float64, out_count [nseq] int32.
        """
        nseq = self.n_seq - seq0 if nseq is None else nseq
        ptr = _ptr
        if stream is None:
            stream = _current_stream()
        N.check(self._L.bx_engine_step(self._h, seq0, nseq, ptr(dets), ptr(det_off), ptr(embs),
                                       ptr(warps), ptr(out), ptr(out_count), stream),
                "bx_engine_step")
        # overlap mode: this step's K5 still reads its inputs after the call returns — hold them
        # so the caching allocator cannot hand their memory out before the next step
        self._inflight = (dets, det_off, embs) if self._overlap else None

    def slots_used(self, seq: int = 0) -> int:
        """Track slots of sequence ``seq`` in use (bx_engine_slots_used_host)."""
        u = C.c_int(0)
        N.check(self._L.bx_engine_slots_used_host(self._h, seq, C.byref(u)), "slots_used")
        return u.value

    def grown(self, track_cap: int, det_cap: int) -> "Engine":
        """A new engine with larger capacities holding this one's tracker state
        (bx_engine_copy_state): the reference's lists are unbounded."""
        e = Engine(self.kind, self.n_seq, track_cap, det_cap, self.emb_dim, self.emb_f64,
                   self.params)
        N.check(self._L.bx_engine_copy_state(e._h, self._h), "bx_engine_copy_state")
        if self._overlap:
            e.set_overlap(True)
        return e

    def inputs_released(self, stream=None) -> None:
        """Overlap mode: order ``stream`` after the last step's last read of its inputs
        (bx_engine_inputs_released) — before refilling a reused input buffer in place."""
        if stream is None:
            stream = _current_stream()
        N.check(self._L.bx_engine_inputs_released(self._h, stream), "bx_engine_inputs_released")

    def lap_ties(self, seq0: int = 0, nseq: int | None = None) -> int:
        """Associations re-solved by lapx's lapjv because their optimum was tied
        (bx_engine_lap_ties_host), summed over sequences [seq0, seq0+nseq)."""
        nseq = self.n_seq - seq0 if nseq is None else nseq
        t = C.c_int64(0)
        N.check(self._L.bx_engine_lap_ties_host(self._h, seq0, nseq, C.byref(t)), "lap_ties")
        return int(t.value)

    def lap_components(self, seq0: int = 0, nseq: int | None = None) -> dict:
        """LAP components solved by the per-lane SSP (past the register path) and by the
        wave-parallel SSP (more than 3 rows) since creation (bx_engine_lap_components_host), over
        [seq0, seq0+nseq)."""
        nseq = self.n_seq - seq0 if nseq is None else nseq
        a = (C.c_int64 * 3)()
        N.check(self._L.bx_engine_lap_components_host(self._h, seq0, nseq, a), "lap_components")
        return {"lane": int(a[0]), "wave": int(a[1]), "helper": int(a[2])}

    def force_assoc_build(self, mode: int) -> None:
        """-1: the association kernel build is picked per launch from the helper-wave cue
        (default); 0 / 1: always the wave-0-only / helper-wave build (bx_engine_force_assoc_build)."""
        N.check(self._L.bx_engine_force_assoc_build(self._h, int(mode)), "force_assoc_build")

    def set_lap_stats(self, on: bool = True) -> None:
        """Count LAP components for lap_components (bx_engine_set_lap_stats; off by default)."""
        N.check(self._L.bx_engine_set_lap_stats(self._h, int(bool(on))), "bx_engine_set_lap_stats")

    def update_host(self, seq: int, dets: np.ndarray, embs: np.ndarray | None = None,
                    warp: np.ndarray | None = None) -> np.ndarray:
        """One frame of one sequence from host arrays; returns float64 [M, 8]."""
        d = np.ascontiguousarray(dets, dtype=np.float32).reshape(-1, 6)
        n = d.shape[0]
        e = None
        if self.with_reid and n:
            if embs is None:
                raise ValueError("BoT-SORT with_reid needs embeddings (ReID inference is outside "
                                 "the association engine)")
            e = np.ascontiguousarray(embs, dtype=np.float64 if self.emb_f64 else np.float32)
            if e.shape != (n, self.emb_dim):
                raise ValueError(f"embs shape {e.shape} != ({n}, {self.emb_dim})")
        w = None if warp is None else np.ascontiguousarray(warp, np.float64).reshape(6)
        out = np.empty((max(n, 1), 8), np.float64)
        m = C.c_int(0)
        N.check(self._L.bx_engine_update_host(
            self._h, seq, d.ctypes.data if n else None, n,
            e.ctypes.data if e is not None else None, w.ctypes.data if w is not None else None,
            out.ctypes.data, C.byref(m), None), "bx_engine_update_host")
        return out[: m.value].copy()

    def update_classes_host(self, seq: int, dets: np.ndarray, embs: np.ndarray | None = None,
                            warp: np.ndarray | None = None, n_classes: int = 80) -> np.ndarray:
        """per_class=True frame of one sequence (bx_engine_update_classes_host): one update per
        class id on that class's detections, active lists per class, lost list shared.  ``warp``:
        None, one 2x3 warp for every class call, or [n_classes, 2, 3] — the reference calls
        cmc.apply once per class call (botsort.py:218)."""
        d = np.ascontiguousarray(dets, dtype=np.float32).reshape(-1, 6)
        n = d.shape[0]
        e = None
        if self.with_reid and n:
            if embs is None:
                raise ValueError("BoT-SORT with_reid needs embeddings (ReID inference is outside "
                                 "the association engine)")
            e = np.ascontiguousarray(embs, dtype=np.float64 if self.emb_f64 else np.float32)
            if e.shape != (n, self.emb_dim):
                raise ValueError(f"embs shape {e.shape} != ({n}, {self.emb_dim})")
        w = _class_warps(warp, n_classes)
        out = np.empty((max(n, 1), 8), np.float64)
        m = C.c_int(0)
        N.check(self._L.bx_engine_update_classes_host(
            self._h, seq, d.ctypes.data if n else None, n,
            e.ctypes.data if e is not None else None, w.ctypes.data if w is not None else None,
            int(n_classes), out.ctypes.data, C.byref(m), None), "bx_engine_update_classes_host")
        return out[: m.value].copy()

    # ---------------------------------------------------------------------------- state I/O
    def status(self) -> int:
        s = C.c_int(0)
        N.check(self._L.bx_engine_status(self._h, C.byref(s)), "bx_engine_status")
        return s.value

    STAGES = ["det_features", "predict", "gate", "cosine", "assoc", "update", "cov_predict",
              "features", "finish"]  # bx_stage order (include/bxassoc.h)

    def probe(self, stage) -> None:
        """Time every launch of one pipeline stage with HIP events (None/-1 disables)."""
        k = -1 if stage is None else (self.STAGES.index(stage) if isinstance(stage, str) else stage)
        N.check(self._L.bx_engine_probe(self._h, k), "bx_engine_probe")

    def set_early_features(self, on: bool = True) -> None:
        """Start each full step's detection-feature kernel at once on a stream of its own
        (bx_engine_set_early_features): the caller guarantees a step's inputs are complete when
        the step is called."""
        N.check(self._L.bx_engine_set_early_features(self._h, int(bool(on))),
                "bx_engine_set_early_features")

    def set_overlap(self, on: bool = True) -> None:
        """Leave each step's feature EMA (K5) unjoined on the side stream (bx_engine_set_overlap):
        the caller keeps a step's input tensors unmodified until the next step is enqueued."""
        N.check(self._L.bx_engine_set_overlap(self._h, int(bool(on))), "bx_engine_set_overlap")
        self._overlap = bool(on)
        if not on:
            self._inflight = None

    def probe_read(self):
        """(total ms, launches) of the probed stage since the last read."""
        t, n = C.c_double(), C.c_int()
        N.check(self._L.bx_engine_probe_read(self._h, C.byref(t), C.byref(n)), "probe_read")
        return t.value, n.value

    def frame_stats(self, seq0: int = 0, nseq: int = None) -> dict:
        """Last frame's unit counts summed over sequences (bench byte accounting)."""
        nseq = self.n_seq - seq0 if nseq is None else nseq
        a = (C.c_int64 * 7)()
        N.check(self._L.bx_engine_frame_stats_host(self._h, seq0, nseq, a), "frame_stats")
        keys = ["dets", "high", "active", "lost", "records", "pairs", "frame"]
        return dict(zip(keys, [int(x) for x in a]))

    def counters(self, seq: int = 0) -> dict:
        fc, idc, na, nl = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        N.check(self._L.bx_engine_counters_host(self._h, seq, C.byref(fc), C.byref(idc),
                                                C.byref(na), C.byref(nl)), "counters")
        return {"frame_count": fc.value, "id_count": idc.value, "n_active": na.value,
                "n_lost": nl.value}

    def set_id_count(self, seq: int, value: int):
        N.check(self._L.bx_engine_set_id_count(self._h, seq, int(value), None), "set_id_count")

    def tracks(self, seq: int = 0) -> dict:
        """Host snapshot of the live tracks: active list then lost list."""
        cap = self.track_cap
        ids = np.zeros(cap, np.int32)
        st = np.zeros(cap, np.int32)
        act = np.zeros(cap, np.int32)
        fid = np.zeros(cap, np.int32)
        sf = np.zeros(cap, np.int32)
        mean = np.zeros((cap, 8))
        cov = np.zeros((cap, 8, 8))
        na, nl = C.c_int(), C.c_int()
        N.check(self._L.bx_engine_tracks_host(
            self._h, seq, cap, ids.ctypes.data, st.ctypes.data, act.ctypes.data, fid.ctypes.data,
            sf.ctypes.data, mean.ctypes.data, cov.ctypes.data, C.byref(na), C.byref(nl)),
            "tracks")
        n = na.value + nl.value
        return {"n_active": na.value, "n_lost": nl.value, "id": ids[:n], "state": st[:n],
                "is_activated": act[:n].astype(bool), "frame_id": fid[:n],
                "start_frame": sf[:n], "mean": mean[:n], "covariance": cov[:n]}

    def class_tracks(self, seq: int, n_classes: int) -> list:
        """per_class mode: each class's active list (``per_class_active_tracks``), as
        ``tracks``-style dicts in class order."""
        cap = self.track_cap
        off = np.zeros(n_classes + 1, np.int32)
        ids = np.zeros(cap, np.int32)
        st = np.zeros(cap, np.int32)
        act = np.zeros(cap, np.int32)
        fid = np.zeros(cap, np.int32)
        sf = np.zeros(cap, np.int32)
        mean = np.zeros((cap, 8))
        cov = np.zeros((cap, 8, 8))
        N.check(self._L.bx_engine_class_tracks_host(
            self._h, seq, n_classes, cap, off.ctypes.data, ids.ctypes.data, st.ctypes.data,
            act.ctypes.data, fid.ctypes.data, sf.ctypes.data, mean.ctypes.data, cov.ctypes.data),
            "class_tracks")
        out = []
        for c in range(n_classes):
            a, b = int(off[c]), int(off[c + 1])
            out.append({"n_active": b - a, "n_lost": 0, "id": ids[a:b], "state": st[a:b],
                        "is_activated": act[a:b].astype(bool), "frame_id": fid[a:b],
                        "start_frame": sf[a:b], "mean": mean[a:b], "covariance": cov[a:b]})
        return out

    def state_set(self, seq: int, ids, mean=None, covariance=None) -> None:
        """Write the Kalman mean [n,8] / covariance [n,8,8] of live tracks by id (host code
        editing STrack.mean / .covariance in the reference)."""
        n, ids, m, c = _state_arrays(ids, mean, covariance, 8, 64)
        N.check(self._L.bx_engine_state_set_host(self._h, seq, n, ids.ctypes.data, _p(m), _p(c)),
                "state_set")



def _class_warps(warp, n_classes: int):
    """Per-class-call warps as the C ABI takes them: [n_classes][6] float64 or None."""
    if warp is None:
        return None
    w = np.asarray(warp, np.float64)
    if w.size == 6:
        w = np.broadcast_to(w.reshape(1, 6), (int(n_classes), 6))
    if w.shape[0] != int(n_classes) or w.size != 6 * int(n_classes):
        raise ValueError(f"warps must be one 2x3 warp or [n_classes, 2, 3], got {w.shape}")
    return np.ascontiguousarray(w.reshape(int(n_classes), 6))


def _state_arrays(ids, a, b, na, nb):
    ids = np.ascontiguousarray(ids, np.int32).reshape(-1)
    n = ids.size
    a = None if a is None else np.ascontiguousarray(a, np.float64).reshape(n, na)
    b = None if b is None else np.ascontiguousarray(b, np.float64).reshape(n, nb)
    return n, ids, a, b


def _p(a):
    return None if a is None else a.ctypes.data

def _asso_kind(name: str) -> int:
    from .iou import KINDS

    if name not in KINDS:
        raise ValueError(f"Invalid association mode: {name}. Choose from {list(KINDS)}")
    return KINDS[name]


@dataclass
class OcsortParams:
    """OcSort constructor parameters (ocsort.py:197-235 names; YAML defaults)."""

    min_conf: float = 0.1
    det_thresh: float = 0.6
    max_age: int = 30
    min_hits: int = 3
    asso_threshold: float = 0.3
    delta_t: int = 3
    inertia: float = 0.1
    use_byte: bool = False
    Q_xy_scaling: float = 0.01
    Q_s_scaling: float = 0.0001
    asso_func: str = "iou"      # utils/iou.py registry mode (BaseTracker asso_func)
    frame_w: float = 1920.0     # centroid normalisation until set_frame_size latches the image
    frame_h: float = 1080.0


class OcsortEngine:
    """Handle over ``bx_ocsort_*`` (include/bxocsort.h): ``n_seq`` OCSort sequences in HBM, one
    kernel launch (one wave per sequence) per frame."""

    def __init__(self, n_seq: int = 1, track_cap: int = 256, det_cap: int = 256,
                 params: OcsortParams | None = None):
        p = params or OcsortParams()
        self.n_seq, self.track_cap, self.det_cap, self.params = n_seq, track_cap, det_cap, p
        cfg = N.BxOcsortConfig(
            n_seq=n_seq, track_cap=track_cap, det_cap=det_cap, min_conf=p.min_conf,
            det_thresh=p.det_thresh, asso_threshold=p.asso_threshold, inertia=p.inertia,
            q_xy_scaling=p.Q_xy_scaling, q_s_scaling=p.Q_s_scaling, max_age=int(p.max_age),
            min_hits=int(p.min_hits), delta_t=int(p.delta_t), use_byte=int(bool(p.use_byte)),
            asso_kind=_asso_kind(p.asso_func), frame_w=float(p.frame_w), frame_h=float(p.frame_h))
        self._L = N.load()
        h = C.c_void_p()
        N.check(self._L.bx_ocsort_create(C.byref(cfg), C.byref(h)), "bx_ocsort_create")
        self._h = h

    def slots_used(self, seq: int = 0) -> int:
        return self.counters(seq)["n_tracks"]

    def grown(self, track_cap: int, det_cap: int) -> "OcsortEngine":
        """A new engine with larger capacities holding this one's state (bx_ocsort_copy_state)."""
        e = OcsortEngine(self.n_seq, track_cap, det_cap, self.params)
        N.check(self._L.bx_ocsort_copy_state(e._h, self._h), "bx_ocsort_copy_state")
        return e

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.bx_ocsort_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, seq0: int = 0, nseq: int | None = None, stream=None):
        nseq = self.n_seq - seq0 if nseq is None else nseq
        N.check(self._L.bx_ocsort_reset(self._h, seq0, nseq, stream), "bx_ocsort_reset")

    def step(self, dets, det_off, out, out_count, seq0: int = 0, nseq: int | None = None,
             stream=None):
        """One frame for sequences [seq0, seq0+nseq) from device tensors (see bx_ocsort_step)."""
        nseq = self.n_seq - seq0 if nseq is None else nseq
        if stream is None:
            stream = _current_stream()
        N.check(self._L.bx_ocsort_step(self._h, seq0, nseq, _ptr(dets), _ptr(det_off), _ptr(out),
                                       _ptr(out_count), stream), "bx_ocsort_step")

    def update_host(self, seq: int, dets: np.ndarray) -> np.ndarray:
        d = np.ascontiguousarray(dets, dtype=np.float32).reshape(-1, 6)
        n = d.shape[0]
        out = np.empty((max(n, 1), 8), np.float64)
        m = C.c_int(0)
        N.check(self._L.bx_ocsort_update_host(self._h, seq, d.ctypes.data if n else None, n,
                                              out.ctypes.data, C.byref(m), None),
                "bx_ocsort_update_host")
        return out[: m.value].copy()

    def update_classes_host(self, seq0: int, n_classes: int, dets: np.ndarray, id_count: int):
        """per_class=True frame (bx_ocsort_update_classes_host): class c is sequence seq0 + c, one
        launch; returns (rows with class-global ids, the advanced class-global id counter)."""
        d = np.ascontiguousarray(dets, dtype=np.float32).reshape(-1, 6)
        n = d.shape[0]
        out = np.empty((max(n, 1), 8), np.float64)
        m, g = C.c_int(0), C.c_int(int(id_count))
        N.check(self._L.bx_ocsort_update_classes_host(
            self._h, seq0, int(n_classes), d.ctypes.data if n else None, n, C.byref(g),
            out.ctypes.data, C.byref(m), None), "bx_ocsort_update_classes_host")
        return out[: m.value].copy(), g.value

    def status(self) -> int:
        s = C.c_int(0)
        N.check(self._L.bx_ocsort_status(self._h, C.byref(s)), "bx_ocsort_status")
        return s.value

    def counters(self, seq: int = 0) -> dict:
        fc, idc, nt = C.c_int(), C.c_int(), C.c_int()
        N.check(self._L.bx_ocsort_counters_host(self._h, seq, C.byref(fc), C.byref(idc),
                                                C.byref(nt)), "counters")
        return {"frame_count": fc.value, "id_count": idc.value, "n_tracks": nt.value}

    def set_id_count(self, seq: int, value: int):
        N.check(self._L.bx_ocsort_set_id_count(self._h, seq, int(value), None), "set_id_count")

    def set_frame_size(self, seq: int, w: float, h: float):
        N.check(self._L.bx_ocsort_set_frame_size(self._h, seq, float(w), float(h), None),
                "set_frame_size")

    def tracks(self, seq: int = 0) -> dict:
        """Host snapshot of the track list (list order): ids, XYSR means x [7], covariances."""
        cap = self.track_cap
        ids = np.zeros(cap, np.int32)
        x = np.zeros((cap, 7))
        P = np.zeros((cap, 7, 7))
        n = C.c_int()
        N.check(self._L.bx_ocsort_tracks_host(self._h, seq, cap, ids.ctypes.data, x.ctypes.data,
                                              P.ctypes.data, C.byref(n)), "tracks")
        k = min(n.value, cap)
        return {"id": ids[:k], "x": x[:k], "P": P[:k]}

    def state_set(self, seq: int, ids, x=None, P=None) -> None:
        """Write KalmanBoxTracker.kf.x [n,7] / .kf.P [n,7,7] of live tracks by id."""
        n, ids, a, b = _state_arrays(ids, x, P, 7, 49)
        N.check(self._L.bx_ocsort_state_set_host(self._h, seq, n, ids.ctypes.data, _p(a), _p(b)),
                "state_set")

    def frame_stats(self, seq0: int = 0, nseq: int | None = None) -> dict:
        """Last frame over sequences [seq0, seq0+nseq): live tracks, output rows, frame."""
        nseq = self.n_seq - seq0 if nseq is None else nseq
        a = (C.c_int64 * 3)()
        N.check(self._L.bx_ocsort_frame_stats_host(self._h, seq0, nseq, a), "frame_stats")
        return dict(zip(["tracks", "outputs", "frame"], [int(x) for x in a]))

    def probe(self, on: bool = True) -> None:
        N.check(self._L.bx_ocsort_probe(self._h, int(bool(on))), "bx_ocsort_probe")

    def probe_read(self):
        t, n = C.c_double(), C.c_int()
        N.check(self._L.bx_ocsort_probe_read(self._h, C.byref(t), C.byref(n)), "probe_read")
        return t.value, n.value


@dataclass
class BoostParams:
    """BoostTrack constructor parameters (boosttrack.py:154-181 names; YAML defaults)."""

    max_age: int = 60
    min_hits: int = 3
    det_thresh: float = 0.6
    iou_threshold: float = 0.3
    use_ecc: bool = True
    min_box_area: float = 10
    aspect_ratio_thresh: float = 1.6
    lambda_iou: float = 0.5
    lambda_mhd: float = 0.25
    lambda_shape: float = 0.25
    use_dlo_boost: bool = True
    use_duo_boost: bool = True
    dlo_boost_coef: float = 0.65
    s_sim_corr: bool = False
    use_rich_s: bool = True
    use_sb: bool = True
    use_vt: bool = True
    with_reid: bool = True


class BoostEngine:
    """Handle over ``bx_boost_*`` (include/bxboost.h): ``n_seq`` BoostTrack sequences in HBM;
    per frame a ReID contraction (fp64 MFMA), the frame kernel (a 1-4 wave workgroup per
    sequence) and the embedding update."""

    def __init__(self, n_seq: int = 1, track_cap: int = 256, det_cap: int = 256,
                 emb_dim: int = 0, params: BoostParams | None = None):
        p = params or BoostParams()
        if p.with_reid and emb_dim <= 0:
            raise ValueError("with_reid BoostTrack needs emb_dim > 0")
        self.n_seq, self.track_cap, self.det_cap, self.params = n_seq, track_cap, det_cap, p
        self.emb_dim = emb_dim if p.with_reid else 0
        cfg = N.BxBoostConfig(
            n_seq=n_seq, track_cap=track_cap, det_cap=det_cap, emb_dim=self.emb_dim,
            max_age=int(p.max_age), min_hits=int(p.min_hits), det_thresh=float(p.det_thresh),
            iou_threshold=float(p.iou_threshold), min_box_area=float(p.min_box_area),
            aspect_ratio_thresh=float(p.aspect_ratio_thresh), lambda_iou=float(p.lambda_iou),
            lambda_mhd=float(p.lambda_mhd), lambda_shape=float(p.lambda_shape),
            dlo_boost_coef=float(p.dlo_boost_coef), use_ecc=int(bool(p.use_ecc)),
            use_dlo_boost=int(bool(p.use_dlo_boost)), use_duo_boost=int(bool(p.use_duo_boost)),
            s_sim_corr=int(bool(p.s_sim_corr)), use_rich_s=int(bool(p.use_rich_s)),
            use_sb=int(bool(p.use_sb)), use_vt=int(bool(p.use_vt)),
            with_reid=int(bool(p.with_reid)))
        self._L = N.load()
        h = C.c_void_p()
        N.check(self._L.bx_boost_create(C.byref(cfg), C.byref(h)), "bx_boost_create")
        self._h = h

    def slots_used(self, seq: int = 0) -> int:
        return self.counters(seq)["n_tracks"]

    def grown(self, track_cap: int, det_cap: int) -> "BoostEngine":
        """A new engine with larger capacities holding this one's state (bx_boost_copy_state)."""
        e = BoostEngine(self.n_seq, track_cap, det_cap, self.emb_dim or 0, self.params)
        N.check(self._L.bx_boost_copy_state(e._h, self._h), "bx_boost_copy_state")
        return e

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.bx_boost_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, seq0: int = 0, nseq: int | None = None, stream=None):
        nseq = self.n_seq - seq0 if nseq is None else nseq
        N.check(self._L.bx_boost_reset(self._h, seq0, nseq, stream), "bx_boost_reset")

    def step(self, dets, det_off, embs, warps, out, out_count, seq0: int = 0,
             nseq: int | None = None, stream=None):
        """One frame for sequences [seq0, seq0+nseq) from device tensors (see bx_boost_step)."""
        nseq = self.n_seq - seq0 if nseq is None else nseq
        if stream is None:
            stream = _current_stream()
        N.check(self._L.bx_boost_step(self._h, seq0, nseq, _ptr(dets), _ptr(det_off), _ptr(embs),
                                      _ptr(warps), _ptr(out), _ptr(out_count), stream),
                "bx_boost_step")

    def update_host(self, seq: int, dets: np.ndarray, embs: np.ndarray | None = None,
                    warp: np.ndarray | None = None) -> np.ndarray:
        d = np.ascontiguousarray(dets, dtype=np.float32).reshape(-1, 6)
        n = d.shape[0]
        e = None
        if self.emb_dim:
            if n and embs is None:
                raise ValueError("with_reid BoostTrack needs embeddings")
            if n:
                e = np.ascontiguousarray(embs, dtype=np.float64).reshape(n, -1)
                if e.shape[1] != self.emb_dim:
                    raise ValueError(f"embedding dim {e.shape[1]} != engine emb_dim {self.emb_dim}")
        w = None if warp is None else np.ascontiguousarray(warp, np.float64).reshape(6)
        out = np.empty((max(n, 1), 8), np.float64)
        m = C.c_int(0)
        N.check(self._L.bx_boost_update_host(
            self._h, seq, d.ctypes.data if n else None, n, None if e is None else e.ctypes.data,
            None if w is None else w.ctypes.data, out.ctypes.data, C.byref(m), None),
            "bx_boost_update_host")
        return out[: m.value].copy()

    def update_classes_host(self, seq: int, dets: np.ndarray, embs: np.ndarray | None = None,
                            warp: np.ndarray | None = None, n_classes: int = 80) -> np.ndarray:
        """per_class=True frame of one sequence (bx_boost_update_classes_host)."""
        d = np.ascontiguousarray(dets, dtype=np.float32).reshape(-1, 6)
        n = d.shape[0]
        e = None
        if self.emb_dim and n:
            if embs is None:
                raise ValueError("with_reid BoostTrack needs embeddings")
            e = np.ascontiguousarray(embs, dtype=np.float64).reshape(n, -1)
            if e.shape[1] != self.emb_dim:
                raise ValueError(f"embedding dim {e.shape[1]} != engine emb_dim {self.emb_dim}")
        w = _class_warps(warp, n_classes)
        out = np.empty((max(n, 1), 8), np.float64)
        m = C.c_int(0)
        N.check(self._L.bx_boost_update_classes_host(
            self._h, seq, d.ctypes.data if n else None, n, None if e is None else e.ctypes.data,
            None if w is None else w.ctypes.data, int(n_classes), out.ctypes.data, C.byref(m),
            None), "bx_boost_update_classes_host")
        return out[: m.value].copy()

    def status(self) -> int:
        s = C.c_int(0)
        N.check(self._L.bx_boost_status(self._h, C.byref(s)), "bx_boost_status")
        return s.value

    def counters(self, seq: int = 0) -> dict:
        fc, idc, nt = C.c_int(), C.c_int(), C.c_int()
        N.check(self._L.bx_boost_counters_host(self._h, seq, C.byref(fc), C.byref(idc),
                                               C.byref(nt)), "counters")
        return {"frame_count": fc.value, "id_count": idc.value, "n_tracks": nt.value}

    def set_id_count(self, seq: int, value: int):
        N.check(self._L.bx_boost_set_id_count(self._h, seq, int(value), None), "set_id_count")

    def tracks(self, seq: int = 0) -> dict:
        """Host snapshot of the track list (list order): ids, means x [8], covariances [8, 8],
        embeddings [F] (with_reid)."""
        cap = self.track_cap
        ids = np.zeros(cap, np.int32)
        x = np.zeros((cap, 8))
        P = np.zeros((cap, 8, 8))
        E = np.zeros((cap, max(self.emb_dim, 1)))
        n = C.c_int()
        N.check(self._L.bx_boost_tracks_host(self._h, seq, cap, ids.ctypes.data, x.ctypes.data,
                                             P.ctypes.data, E.ctypes.data if self.emb_dim else None,
                                             C.byref(n)), "tracks")
        k = min(n.value, cap)
        snap = {"id": ids[:k], "x": x[:k], "P": P[:k]}
        if self.emb_dim:
            snap["emb"] = E[:k]
        return snap

    def state_set(self, seq: int, ids, x=None, P=None) -> None:
        """Write KalmanBoxTracker.kf.x [n,8] / .kf.covariance [n,8,8] of live tracks by id."""
        n, ids, a, b = _state_arrays(ids, x, P, 8, 64)
        N.check(self._L.bx_boost_state_set_host(self._h, seq, n, ids.ctypes.data, _p(a), _p(b)),
                "state_set")

    def frame_stats(self, seq0: int = 0, nseq: int | None = None) -> dict:
        nseq = self.n_seq - seq0 if nseq is None else nseq
        a = (C.c_int64 * 7)()
        N.check(self._L.bx_boost_frame_stats_host(self._h, seq0, nseq, a), "frame_stats")
        return dict(zip(["dets", "kept", "tracks", "outputs", "records", "frame", "pairs"],
                        [int(x) for x in a]))

    STAGES = ["embcost", "frame", "feature"]

    def probe(self, stage) -> None:
        """Time one stage per step (name from STAGES or index); None = off."""
        idx = -1 if stage is None else (self.STAGES.index(stage) if isinstance(stage, str)
                                        else int(stage))
        N.check(self._L.bx_boost_probe(self._h, idx), "bx_boost_probe")

    def probe_read(self):
        t, n = C.c_double(), C.c_int()
        N.check(self._L.bx_boost_probe_read(self._h, C.byref(t), C.byref(n)), "probe_read")
        return t.value, n.value


@dataclass
class SsParams:
    """StrongSort constructor parameters (strongsort.py:45-66 names and defaults)."""

    min_conf: float = 0.1
    max_cos_dist: float = 0.15
    max_iou_dist: float = 0.7
    max_age: int = 50
    n_init: int = 2
    nn_budget: int = 150
    mc_lambda: float = 0.995
    ema_alpha: float = 0.9
    conf_thresh_high: float = 0.7
    conf_thresh_low: float = 0.3
    id_preservation_weight: float = 0.1
    crowd_detection: bool = True
    born_confirmed: bool = False


class SsEngine:
    """Handle over ``bx_ss_*`` (include/bxstrongsort.h): ``n_seq`` StrongSort sequences in HBM;
    per frame the detection-feature kernel, the NN-gallery distance (fp64 MFMA), the recovery
    similarities and the frame kernel (one wave per sequence)."""

    STAGES = ["prep", "nn", "recovery", "pre", "cost", "match", "update", "post", "fit"]

    def __init__(self, n_seq: int = 1, track_cap: int = 256, det_cap: int = 256,
                 emb_dim: int = 512, vec_cap: int = 32, params: SsParams | None = None):
        p = params or SsParams()
        self.n_seq, self.track_cap, self.det_cap, self.params = n_seq, track_cap, det_cap, p
        self.emb_dim = emb_dim
        cfg = N.BxSsConfig(
            n_seq=n_seq, track_cap=track_cap, det_cap=det_cap, emb_dim=emb_dim, vec_cap=vec_cap,
            min_conf=float(p.min_conf), max_cos_dist=float(p.max_cos_dist),
            max_iou_dist=float(p.max_iou_dist), max_age=int(p.max_age), n_init=int(p.n_init),
            nn_budget=int(p.nn_budget), mc_lambda=float(p.mc_lambda),
            ema_alpha=float(p.ema_alpha), conf_thresh_high=float(p.conf_thresh_high),
            conf_thresh_low=float(p.conf_thresh_low),
            id_preservation_weight=float(p.id_preservation_weight),
            crowd_detection=int(bool(p.crowd_detection)),
            born_confirmed=int(bool(p.born_confirmed)))
        self._L = N.load()
        h = C.c_void_p()
        N.check(self._L.bx_ss_create(C.byref(cfg), C.byref(h)), "bx_ss_create")
        self._h = h
        self.vec_cap = vec_cap

    def slots_used(self, seq: int = 0) -> int:
        """Listed tracks plus the lost buffer's (their galleries keep their slots)."""
        c = self.counters(seq)
        return c["n_tracks"] + c["n_lost"]

    def grown(self, track_cap: int, det_cap: int) -> "SsEngine":
        """A new engine with larger capacities holding this one's state (bx_ss_copy_state)."""
        e = SsEngine(self.n_seq, track_cap, det_cap, self.emb_dim, self.vec_cap, self.params)
        N.check(self._L.bx_ss_copy_state(e._h, self._h), "bx_ss_copy_state")
        return e

    def close(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.bx_ss_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, seq0: int = 0, nseq: int | None = None, stream=None):
        nseq = self.n_seq - seq0 if nseq is None else nseq
        N.check(self._L.bx_ss_reset(self._h, seq0, nseq, stream), "bx_ss_reset")

    def step(self, dets, det_off, embs, warps, out, out_count, seq0: int = 0,
             nseq: int | None = None, stream=None):
        """One frame for sequences [seq0, seq0+nseq) from device tensors (see bx_ss_step):
        dets [sumN, 6] f64, det_off [S+1] i32, embs [sumN, F] f64, out [sumN, 10] f64."""
        nseq = self.n_seq - seq0 if nseq is None else nseq
        if stream is None:
            stream = _current_stream()
        N.check(self._L.bx_ss_step(self._h, seq0, nseq, _ptr(dets), _ptr(det_off), _ptr(embs),
                                   _ptr(warps), _ptr(out), _ptr(out_count), stream), "bx_ss_step")

    def update_host(self, seq: int, dets: np.ndarray, embs: np.ndarray,
                    warp: np.ndarray | None = None) -> np.ndarray:
        d = np.ascontiguousarray(dets, dtype=np.float64).reshape(-1, 6)
        n = d.shape[0]
        e = np.ascontiguousarray(embs, dtype=np.float64).reshape(n, -1) if n else None
        if n and e.shape[1] != self.emb_dim:
            raise ValueError(f"embedding dim {e.shape[1]} != engine emb_dim {self.emb_dim}")
        w = None if warp is None else np.ascontiguousarray(warp, np.float64).reshape(6)
        out = np.empty((max(n, 1), 10), np.float64)
        m = C.c_int(0)
        N.check(self._L.bx_ss_update_host(
            self._h, seq, d.ctypes.data if n else None, n, e.ctypes.data if n else None,
            None if w is None else w.ctypes.data, out.ctypes.data, C.byref(m), None),
            "bx_ss_update_host")
        return out[: m.value].copy()

    def status(self) -> int:
        s = C.c_int(0)
        N.check(self._L.bx_ss_status(self._h, C.byref(s)), "bx_ss_status")
        return s.value

    def counters(self, seq: int = 0) -> dict:
        fc, nid, nt, nl = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        N.check(self._L.bx_ss_counters_host(self._h, seq, C.byref(fc), C.byref(nid), C.byref(nt),
                                            C.byref(nl)), "counters")
        return {"frame_count": fc.value, "next_id": nid.value, "n_tracks": nt.value,
                "n_lost": nl.value}

    def tracks(self, seq: int = 0) -> dict:
        cap = self.track_cap
        ids = np.zeros(cap, np.int32)
        st = np.zeros(cap, np.int32)
        mean = np.zeros((cap, 8))
        cov = np.zeros((cap, 8, 8))
        n = C.c_int()
        N.check(self._L.bx_ss_tracks_host(self._h, seq, cap, ids.ctypes.data, st.ctypes.data,
                                          mean.ctypes.data, cov.ctypes.data, C.byref(n)),
                "tracks")
        k = min(n.value, cap)
        return {"id": ids[:k], "state": st[:k], "mean": mean[:k], "covariance": cov[:k]}

    def state_set(self, seq: int, ids, mean=None, covariance=None) -> None:
        """Write Track.mean [n,8] / Track.covariance [n,8,8] of live tracks by id."""
        n, ids, m, c = _state_arrays(ids, mean, covariance, 8, 64)
        N.check(self._L.bx_ss_state_set_host(self._h, seq, n, ids.ctypes.data, _p(m), _p(c)),
                "state_set")

    def track_attrs(self, seq: int = 0) -> dict:
        """Per track in list order: id, quality_score, conf, _max_age, len(features)."""
        cap = self.track_cap
        ids, mx, nf = (np.zeros(cap, np.int32) for _ in range(3))
        q, cf = np.zeros(cap), np.zeros(cap)
        n = C.c_int()
        N.check(self._L.bx_ss_track_attrs_host(self._h, seq, cap, ids.ctypes.data, q.ctypes.data,
                                               cf.ctypes.data, mx.ctypes.data, nf.ctypes.data,
                                               C.byref(n)), "track_attrs")
        k = min(n.value, cap)
        return {"id": ids[:k], "quality": q[:k], "conf": cf[:k], "max_age": mx[:k],
                "n_features": nf[:k]}

    def track_attrs_set(self, seq: int, ids, quality=None, conf=None, max_age=None) -> None:
        ids = np.ascontiguousarray(ids, np.int32).reshape(-1)
        q = None if quality is None else np.ascontiguousarray(quality, np.float64).reshape(-1)
        c = None if conf is None else np.ascontiguousarray(conf, np.float64).reshape(-1)
        m = None if max_age is None else np.ascontiguousarray(max_age, np.int32).reshape(-1)
        N.check(self._L.bx_ss_track_attrs_set_host(self._h, seq, ids.size, ids.ctypes.data,
                                                   _p(q), _p(c), _p(m)), "track_attrs_set")

    def last_features(self, seq: int, ids) -> np.ndarray:
        """features[-1] of the tracks `ids` ([n, emb_dim] float64)."""
        ids = np.ascontiguousarray(ids, np.int32).reshape(-1)
        out = np.zeros((ids.size, self.emb_dim))
        if ids.size:
            N.check(self._L.bx_ss_last_feature_host(self._h, seq, ids.size, ids.ctypes.data,
                                                    out.ctypes.data), "last_features")
        return out

    def last_features_set(self, seq: int, ids, feats, normalize: bool = True) -> None:
        ids = np.ascontiguousarray(ids, np.int32).reshape(-1)
        f = np.ascontiguousarray(feats, np.float64).reshape(ids.size, self.emb_dim)
        N.check(self._L.bx_ss_last_feature_set_host(self._h, seq, ids.size, ids.ctypes.data,
                                                    f.ctypes.data, int(bool(normalize))),
                "last_features_set")

    def frame_stats(self, seq0: int = 0, nseq: int | None = None) -> dict:
        nseq = self.n_seq - seq0 if nseq is None else nseq
        a = (C.c_int64 * 7)()
        N.check(self._L.bx_ss_frame_stats_host(self._h, seq0, nseq, a), "frame_stats")
        return dict(zip(["dets", "tracks", "queried", "rows", "outputs", "frame", "matches"],
                        [int(x) for x in a]))

    def set_lsap_mode(self, fast: bool) -> None:
        """Solve + certify the cascade LSAPs (default) or always solve them in scipy's row order
        (bx_ss_set_lsap_mode)."""
        N.check(self._L.bx_ss_set_lsap_mode(self._h, int(bool(fast))), "bx_ss_set_lsap_mode")

    def lsap_stats(self, seq0: int = 0, nseq: int | None = None) -> dict:
        """LSAP counters since creation (bx_ss_lsap_stats_host): solves, certified unique,
        unique up to rejected pairs, ties re-solved in scipy's order, stages restarted."""
        nseq = self.n_seq - seq0 if nseq is None else nseq
        a = (C.c_int64 * 5)()
        N.check(self._L.bx_ss_lsap_stats_host(self._h, seq0, nseq, a), "lsap_stats")
        return dict(zip(["solves", "unique", "unique_up_to_rejected", "ties", "restarts"],
                        [int(x) for x in a]))

    def probe(self, stage) -> None:
        idx = -1 if stage is None else (self.STAGES.index(stage) if isinstance(stage, str)
                                        else int(stage))
        N.check(self._L.bx_ss_probe(self._h, idx), "bx_ss_probe")

    def probe_read(self):
        t, n = C.c_double(), C.c_int()
        N.check(self._L.bx_ss_probe_read(self._h, C.byref(t), C.byref(n)), "probe_read")
        return t.value, n.value


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(type(x))


def _current_stream():
    try:
        import torch

        if torch.cuda.is_available():
            return torch.cuda.current_stream().cuda_stream
    except Exception:
        pass
    return None
