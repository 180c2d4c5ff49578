"""StrongSort's occlusion handling (``handle_occlusions=True``) as a host post-process over the
engine's track state.

The reference runs ``OcclusionAwareTracker.update_with_occlusion_handling`` on the host after
every tracker update (``trackers/strongsort/strongsort.py:150-154, 195-201``;
``utils/occlusion_handler.py:312-439``): an O(T^2) overlap analysis of the track boxes, then
per-track edits — ``_max_age`` doubled and ``quality_score`` floored at 0.6 while occluded, the
Kalman position replaced by the occluders' mean centre (covariance x1.5) when more than 80 %
hidden, the last feature buffered and, when the track re-emerges, its confidence raised by 0.1
and ``features[-1]`` blended with the strongest buffered feature.  Here the analysis runs in
numpy on the host and the edits go back through the engine's state calls
(``bx_ss_state_set_host``, ``bx_ss_track_attrs_set_host``, ``bx_ss_last_feature_set_host``).

Reference behaviour kept on purpose:
* ``OverlapAnalyzer`` reads the tlwh rows it is given as xyxy (``:49-56, :109-113``), so boxes
  only overlap for tracks near the top-left corner (x < w, y < h);
* a MUTUAL occlusion (size ratio in [0.8, 1.2]) reaches ``_resolve_mutual_occlusion``, whose
  ``list(int)`` raises ``TypeError`` — raised here at the same point;
* occluder centres are averaged in the iteration order of the reference's Python ``set``.
Deviations: ``_max_age`` is held at 2^30 instead of growing without bound (the engine stores an
int32; deletion thresholds that large are never reached); the blended feature is normalised in
the engine's wave order, like every other 1-D norm of the engine (numpy's BLAS order is unpinned).
"""
from __future__ import annotations

import math
from collections import defaultdict, deque

import numpy as np

MAX_AGE_CAP = 1 << 30
_PERM = [np.arange(64) ^ d for d in (32, 16, 8, 4, 2, 1)]
_TYPES = ("NO_OCCLUSION", "PARTIAL_OCCLUSION", "FULL_OCCLUSION", "MUTUAL_OCCLUSION")


def wave_norm(x: np.ndarray) -> float:
    """||x|| in the engine's wave order (64 lane-strided partial sums, xor butterfly)."""
    s = np.zeros(64)
    for k in range(0, x.size, 64):
        c = x[k:k + 64]
        s[:c.size] += c * c
    for p in _PERM:
        s = s + s[p]
    return math.sqrt(s[0])


def tlwh(mean: np.ndarray) -> np.ndarray:
    """Track.to_tlwh (sort/track.py:137-149)."""
    r = mean[:4].copy()
    r[2] *= r[3]
    r[:2] -= r[2:] / 2
    return r


def _pair_tables(boxes: np.ndarray):
    """compute_overlap_matrix (:45-87) and the size-ratio matrix of analyze_spatial_relationships
    (:101-141), both reading each row as (x1, y1, x2, y2)."""
    n = boxes.shape[0]
    x1, y1, x2, y2 = boxes.T
    area = (x2 - x1) * (y2 - y1)
    iu = np.triu_indices(n, 1)
    i, j = iu
    with np.errstate(divide="ignore", invalid="ignore"):
        w = np.maximum(0, np.minimum(x2[i], x2[j]) - np.maximum(x1[i], x1[j]))
        h = np.maximum(0, np.minimum(y2[i], y2[j]) - np.maximum(y1[i], y1[j]))
        inter = w * h
        o = np.where(inter > 0, np.maximum(inter / area[i], inter / area[j]), 0.0)
        r = np.where(area[j] > 0, area[i] / area[j], 1.0)
        rinv = 1.0 / r
    ov = np.zeros((n, n))
    sr = np.zeros((n, n))
    ov[i, j] = ov[j, i] = o
    sr[i, j], sr[j, i] = r, rinv
    return ov, sr


class OcclusionHandler:
    """OcclusionAwareTracker + OcclusionStateManager over one engine sequence."""

    def __init__(self, engine, seq: int = 0, occlusion_threshold: float = 0.3):
        self.engine, self.seq, self.thr = engine, seq, occlusion_threshold
        self.visibility = {}                 # track id -> visibility score (kept across frames)
        self.current = defaultdict(set)      # occluded id -> occluder ids (this frame)
        self.buffer = {}                     # occlusion_buffer: id -> deque(maxlen=10)
        self.events = defaultdict(list)      # occluded id -> [occluder, type, start, end, ratio]

    def level(self, tid: int) -> float:
        return 1.0 - self.visibility.get(int(tid), 1.0)

    # -------------------------------------------------------------------- state analysis
    def _analyse(self, ids, boxes, frame_id):
        """update_occlusion_state (:143-207): visibility of every track, current occluders."""
        ov, sr = _pair_tables(boxes)
        self.current.clear()
        for i, ti in enumerate(ids):
            vis = 1.0
            for j in np.flatnonzero(ov[i] > self.thr):
                if j == i:
                    continue
                o, r = ov[i, j], sr[i, j]
                kind = 1 if o < 0.6 else (2 if r > 1.5 else 3)  # detect_occlusion_type
                if r > 1.2:
                    occluder, occluded = ti, ids[j]
                elif r < 0.8:
                    occluder, occluded = ids[j], ti
                else:  # _resolve_mutual_occlusion: `list(int)`
                    raise TypeError("'int' object is not iterable")
                self.current[occluded].add(occluder)
                if ti == occluded:
                    vis *= (1.0 - o)
                self._record(occluder, occluded, kind, o, frame_id)
            self.visibility[ti] = vis

    def _record(self, occluder, occluded, kind, ratio, frame_id):
        """_record_occlusion_event (:209-232), kept for occlusion_stats."""
        ev = self.events[occluded]
        if ev and ev[-1][0] == occluder and ev[-1][3] is None and frame_id - ev[-1][2] < 10:
            ev[-1][4] = max(ev[-1][4], ratio)
            return
        ev.append([occluder, kind, frame_id, None, ratio])

    # ----------------------------------------------------------------------- the frame
    def __call__(self, frame_id: int, rows: np.ndarray) -> np.ndarray:
        """Run after the engine's frame; returns the output rows with the edited boxes, conf,
        quality and the occlusion level column (strongsort.py:324-354)."""
        eng, seq = self.engine, self.seq
        snap, attrs = eng.tracks(seq), eng.track_attrs(seq)
        ids = [int(t) for t in snap["id"]]
        if not ids:
            return rows
        means = snap["mean"].copy()
        covs = snap["covariance"].copy()
        self._analyse(ids, np.array([tlwh(m) for m in means]), frame_id)
        quality = attrs["quality"].copy()
        conf = attrs["conf"].copy()
        max_age = attrs["max_age"].astype(np.int64)
        levels = np.array([self.level(t) for t in ids])
        occl = [k for k in range(len(ids)) if levels[k] > 0.3 and attrs["n_features"][k] > 0]
        emer = [k for k in range(len(ids)) if levels[k] <= 0.3 and ids[k] in self.buffer
                and attrs["n_features"][k] > 0]
        last = eng.last_features(seq, [ids[k] for k in occl + emer])
        feat = {ids[k]: last[q] for q, k in enumerate(occl + emer)}
        moved, edited, blends = [], [], {}
        for k, tid in enumerate(ids):  # _apply_occlusion_modifications (:341-371)
            if levels[k] > 0.3 or tid in self.buffer:
                edited.append(k)
            if levels[k] > 0.3:
                max_age[k] = min(int(max_age[k] * 2.0), MAX_AGE_CAP)
                if tid in feat:
                    self.buffer.setdefault(tid, deque(maxlen=10)).append(feat[tid])
                quality[k] = max(quality[k], 0.6)
                if levels[k] > 0.8 and self.current.get(tid):
                    centres = [[(b[0] + b[2]) / 2, (b[1] + b[3]) / 2]
                               for b in (tlwh(means[ids.index(o)]) for o in self.current[tid])]
                    mc = np.mean(centres, axis=0)
                    x, y, w, h = np.array([mc[0] - 50 / 2, mc[1] - 100 / 2, 50, 100])
                    means[k, :4] = [x + w / 2, y + h / 2, w / h, h]
                    covs[k, :4, :4] *= 1.5
                    moved.append(k)
            elif tid in self.buffer:  # _handle_emerging_track (:394-417)
                conf[k] = min(conf[k] + 0.1, 1.0)
                stored = list(self.buffer[tid])
                if stored and tid in feat:
                    best = max(stored, key=wave_norm)
                    blends[tid] = 0.7 * feat[tid] + 0.3 * best
                del self.buffer[tid]
        if moved:
            eng.state_set(seq, [ids[k] for k in moved], means[moved], covs[moved])
        if edited:
            eng.track_attrs_set(seq, [ids[k] for k in edited], quality=quality[edited],
                                conf=conf[edited], max_age=max_age[edited])
        if blends:
            eng.last_features_set(seq, list(blends), np.stack(list(blends.values())),
                                  normalize=True)
        # output rows: boxes of moved tracks, conf / quality after the edits, occlusion level
        rows = np.array(rows, np.float64).reshape(-1, 10)
        pos = {t: k for k, t in enumerate(ids)}
        for r in rows:
            k = pos[int(r[4])]
            if k in moved:
                b = tlwh(means[k])
                b[2:] = b[:2] + b[2:]
                r[:4] = b
            r[5], r[8], r[9] = conf[k], quality[k], levels[k]
        return rows

    def statistics(self) -> dict:
        """get_occlusion_statistics (:419-439)."""
        types = defaultdict(int)
        for evs in self.events.values():
            for e in evs:
                types[_TYPES[e[1]]] += 1
        return {
            "currently_occluded_tracks": sum(1 for v in self.current.values() if v),
            "total_occlusion_events": sum(len(v) for v in self.events.values()),
            "average_visibility": (np.mean(list(self.visibility.values()))
                                   if self.visibility else 1.0),
            "tracks_in_occlusion_buffer": len(self.buffer),
            "occlusion_type_distribution": dict(types),
        }
