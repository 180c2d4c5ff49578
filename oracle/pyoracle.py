"""ctypes binding of the C oracle (oracle/build/libbxoracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — never by the product package boxmot_amd/.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "libbxoracle.so"

_dp = C.POINTER(C.c_double)
_fp = C.POINTER(C.c_float)
_ip = C.POINTER(C.c_int)


def build(force: bool = False) -> Path:
    srcs = [HERE / n for n in ("bxo_ops.c", "bxo_track.c", "bxo_ocsort.c", "bxo_boost.c",
                               "bxo_strongsort.c", "bxo.h", "bxo_internal.h")]
    if force or not LIB_PATH.exists() or any(
        s.stat().st_mtime > LIB_PATH.stat().st_mtime for s in srcs
    ):
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


class BoostParams(C.Structure):
    """bxo_boost_params (oracle/bxo.h)."""

    _fields_ = [("max_age", C.c_int), ("min_hits", C.c_int), ("det_thresh", C.c_double),
                ("iou_threshold", C.c_double), ("min_box_area", C.c_double),
                ("aspect_ratio_thresh", C.c_double), ("lambda_iou", C.c_double),
                ("lambda_mhd", C.c_double), ("lambda_shape", C.c_double),
                ("dlo_boost_coef", C.c_double), ("use_ecc", C.c_int), ("use_dlo_boost", C.c_int),
                ("use_duo_boost", C.c_int), ("s_sim_corr", C.c_int), ("use_rich_s", C.c_int),
                ("use_sb", C.c_int), ("use_vt", C.c_int), ("with_reid", C.c_int)]


class SsParams(C.Structure):
    """bxo_ss_params (oracle/bxo.h)."""

    _fields_ = [("min_conf", C.c_double), ("max_cos_dist", C.c_double),
                ("max_iou_dist", C.c_double), ("max_age", C.c_int), ("n_init", C.c_int),
                ("nn_budget", C.c_int), ("mc_lambda", C.c_double), ("ema_alpha", C.c_double),
                ("conf_thresh_high", C.c_double), ("conf_thresh_low", C.c_double),
                ("id_preservation_weight", C.c_double), ("crowd_detection", C.c_int),
                ("born_confirmed", C.c_int)]


# StrongSort.__init__ defaults (strongsort.py:43-66)
SS_DEFAULTS = dict(min_conf=0.1, max_cos_dist=0.15, max_iou_dist=0.7, max_age=50, n_init=2,
                   nn_budget=150, mc_lambda=0.995, ema_alpha=0.9, conf_thresh_high=0.7,
                   conf_thresh_low=0.3, id_preservation_weight=0.1, crowd_detection=True,
                   born_confirmed=True)


def ss_params(**p):
    q = dict(SS_DEFAULTS)
    q.update({k: v for k, v in p.items() if k in SS_DEFAULTS})
    return SsParams(**{k: (float(v) if isinstance(SS_DEFAULTS[k], float) else int(v))
                       for k, v in q.items()})


def lsap(cost):
    """scipy.optimize.linear_sum_assignment restated (rows, cols)."""
    c = np.ascontiguousarray(cost, np.float64)
    nr, nc = c.shape
    k = max(1, min(nr, nc))
    r = np.zeros(k, np.int32)
    cc = np.zeros(k, np.int32)
    n = lib().bxo_lsap(_d(c), nr, nc, r.ctypes.data_as(_ip), cc.ctypes.data_as(_ip))
    return r[:max(n, 0)], cc[:max(n, 0)]


def lapjv(cost, extend_cost=False, cost_limit=np.inf):
    """lapx.lapjv (0.5.11 _lapjv.pyx wrapper rules) around the restated lapjv_internal
    (bxo_lapjv): returns (x [nr], y [nc]) int32 with -1 for unmatched when extended."""
    c = np.ascontiguousarray(cost, np.float64)
    nr, nc = c.shape
    if nr != nc and not extend_cost:
        raise ValueError("Square cost array expected. If cost is intentionally non-square, "
                         "pass extend_cost=True.")
    if cost_limit < np.inf:
        n = nr + nc
        E = np.full((n, n), cost_limit / 2.0)
        E[nr:, nc:] = 0
        E[:nr, :nc] = c
    elif extend_cost:
        n = max(nr, nc)
        E = np.zeros((n, n))
        E[:nr, :nc] = c
    else:
        n, E = nr, c
    x = np.zeros(n, np.int32)
    y = np.zeros(n, np.int32)
    if n:
        lib().bxo_lapjv(n, _d(np.ascontiguousarray(E)), x.ctypes.data_as(_ip),
                        y.ctypes.data_as(_ip))
    if cost_limit < np.inf or extend_cost:
        x[x >= nc] = -1
        y[y >= nr] = -1
        x, y = x[:nr], y[:nc]
    return x, y


# BoostTrack.__init__ defaults (boosttrack.py:154-181)
BOOST_DEFAULTS = dict(max_age=60, min_hits=3, det_thresh=0.6, iou_threshold=0.3, use_ecc=True,
                      min_box_area=10, aspect_ratio_thresh=1.6, lambda_iou=0.5, lambda_mhd=0.25,
                      lambda_shape=0.25, use_dlo_boost=True, use_duo_boost=True,
                      dlo_boost_coef=0.65, s_sim_corr=False, use_rich_s=False, use_sb=False,
                      use_vt=False, with_reid=False)


def boost_params(**p):
    q = dict(BOOST_DEFAULTS)
    q.update({k: v for k, v in p.items() if k in BOOST_DEFAULTS})
    return BoostParams(**{k: (type(getattr(BoostParams, k)) is not None and
                              (float(v) if isinstance(BOOST_DEFAULTS[k], float) else int(v)))
                          for k, v in q.items()})


_lib = None


def set_threads(n: int) -> None:
    """Threads for the oracle's parallel loops (StrongSort NN rows); results do not depend on it."""
    lib().bxo_set_threads(int(n))


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(str(LIB_PATH))
        L.bxo_set_threads.argtypes = [C.c_int]
        L.bxo_iou_batch.argtypes = [_dp, C.c_int, _dp, C.c_int, _dp]
        L.bxo_fuse_score.argtypes = [_dp, C.c_int, C.c_int, _dp]
        L.bxo_embedding_distance.argtypes = [_fp, C.c_int, _fp, C.c_int, C.c_int, _dp]
        L.bxo_np_norm_f32.argtypes = [_fp, C.c_int]
        L.bxo_np_norm_f32.restype = C.c_float
        L.bxo_kf_initiate.argtypes = [C.c_int, _dp, _dp, _dp]
        L.bxo_kf_multi_predict.argtypes = [C.c_int, C.c_int, _dp, _dp]
        L.bxo_kf_update.argtypes = [C.c_int, _dp, _dp, _dp, C.c_double]
        L.bxo_kf_gating_distance.argtypes = [C.c_int, _dp, _dp, _dp, C.c_int, _dp]
        L.bxo_lapjv.argtypes = [C.c_int, _dp, _ip, _ip]
        L.bxo_linear_assignment.argtypes = [_dp, C.c_int, C.c_int, C.c_double, _ip, _ip, _ip,
                                            _ip, _ip, _ip]
        L.bxo_bytetrack_new.argtypes = [C.c_double, C.c_double, C.c_double, C.c_int, C.c_int]
        L.bxo_bytetrack_new.restype = C.c_void_p
        L.bxo_botsort_new.argtypes = [C.c_double, C.c_double, C.c_double, C.c_int, C.c_double,
                                      C.c_double, C.c_double, C.c_int, C.c_int, C.c_int]
        L.bxo_botsort_new.restype = C.c_void_p
        L.bxo_update.argtypes = [C.c_void_p, _dp, C.c_int, C.c_void_p, C.c_int, C.c_int, _dp,
                                 _dp, C.c_int]
        L.bxo_id_count.argtypes = [C.c_void_p]
        L.bxo_frame_count.argtypes = [C.c_void_p]
        for fn in ("bxo_kf_xysr_initiate", "bxo_kf_xysr_update", "bxo_kf_boost_initiate",
                   "bxo_kf_boost_update"):
            getattr(L, fn).argtypes = [C.c_int, _dp, _dp, _dp]
        L.bxo_kf_xysr_predict.argtypes = [C.c_int, _dp, _dp, C.c_double, C.c_double]
        L.bxo_kf_boost_predict.argtypes = [C.c_int, _dp, _dp]
        L.bxo_kf_boost_mh_dist.argtypes = [C.c_int, _dp, C.c_int, _dp, _dp, _dp]
        L.bxo_select_class.argtypes = [C.c_void_p, C.c_int]
        L.bxo_ss_set_occlusion.argtypes = [C.c_void_p, C.c_int, C.c_double]
        L.bxo_pyset_order.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.bxo_set_frame_count.argtypes = [C.c_void_p, C.c_int]
        L.bxo_ocsort_set_id_count.argtypes = [C.c_void_p, C.c_int]
        L.bxo_boost_set_frame_count.argtypes = [C.c_void_p, C.c_int]
        L.bxo_free.argtypes = [C.c_void_p]
        L.bxo_ocsort_new.argtypes = [C.c_double, C.c_double, C.c_int, C.c_int, C.c_double,
                                     C.c_int, C.c_double, C.c_int, C.c_double, C.c_double]
        L.bxo_ocsort_new.restype = C.c_void_p
        L.bxo_ocsort_free.argtypes = [C.c_void_p]
        L.bxo_ocsort_set_asso.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double]
        L.bxo_ocsort_id_count.argtypes = [C.c_void_p]
        L.bxo_ocsort_update.argtypes = [C.c_void_p, _dp, C.c_int, _dp, C.c_int]
        L.bxo_tracks.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p]
        for fn in ("bxo_state_set", "bxo_ocsort_state_set", "bxo_boost_state_set",
                   "bxo_ss_state_set"):
            getattr(L, fn).argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.bxo_ocsort_tracks.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.bxo_nn_cosine_distance.argtypes = [_dp, _ip, C.c_int, _dp, C.c_int, C.c_int, _dp]
        L.bxo_np_norm_f64.argtypes = [_dp, C.c_int]
        L.bxo_np_norm_f64.restype = C.c_double
        L.bxo_acos.argtypes = [C.c_double]
        L.bxo_acos.restype = C.c_double
        L.bxo_boost_new.argtypes = [C.POINTER(BoostParams)]
        L.bxo_boost_new.restype = C.c_void_p
        L.bxo_boost_free.argtypes = [C.c_void_p]
        L.bxo_boost_id_count.argtypes = [C.c_void_p]
        L.bxo_boost_set_id_count.argtypes = [C.c_void_p, C.c_int]
        L.bxo_boost_tracks.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
        L.bxo_boost_update.argtypes = [C.c_void_p, _dp, C.c_int, C.c_void_p, C.c_int, _dp, _dp,
                                       C.c_int]
        L.bxo_ss_new.argtypes = [C.POINTER(SsParams)]
        L.bxo_ss_new.restype = C.c_void_p
        L.bxo_ss_free.argtypes = [C.c_void_p]
        L.bxo_ss_next_id.argtypes = [C.c_void_p]
        L.bxo_ss_tracks.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p]
        L.bxo_ss_update.argtypes = [C.c_void_p, _dp, C.c_int, C.c_void_p, C.c_int, _dp, _dp,
                                    C.c_int]
        L.bxo_lsap.argtypes = [_dp, C.c_int, C.c_int, _ip, _ip]
        L.bxo_asso_batch.argtypes = [C.c_int, _dp, C.c_int, _dp, C.c_int, C.c_double,
                                     C.c_double, _dp]
        L.bxo_aw_max_metric.argtypes = [_dp, C.c_int, C.c_int, C.c_double, C.c_double, _dp]
        L.bxo_atan.argtypes = [C.c_double]
        L.bxo_atan.restype = C.c_double
        L.bxo_exp.argtypes = [C.c_double]
        L.bxo_exp.restype = C.c_double
        L.bxo_pow15.argtypes = [C.c_double]
        L.bxo_pow15.restype = C.c_double
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(_dp)


def iou_batch(a, b):
    a = np.ascontiguousarray(a, np.float64).reshape(-1, 4)
    b = np.ascontiguousarray(b, np.float64).reshape(-1, 4)
    out = np.zeros((a.shape[0], b.shape[0]))
    lib().bxo_iou_batch(_d(a), a.shape[0], _d(b), b.shape[0], _d(out))
    return out


ASSO_KIND = {"iou": 0, "hmiou": 1, "giou": 2, "diou": 3, "ciou": 4, "centroid": 5}


def asso_batch(kind, a, b, w=1920, h=1080):
    """AssociationFunction.<kind>_batch (utils/iou.py) restated."""
    a = np.ascontiguousarray(a, np.float64).reshape(-1, 4)
    b = np.ascontiguousarray(b, np.float64).reshape(-1, 4)
    out = np.zeros((a.shape[0], b.shape[0]))
    lib().bxo_asso_batch(ASSO_KIND[kind], _d(a), a.shape[0], _d(b), b.shape[0], float(w),
                         float(h), _d(out))
    return out


def aw_max_metric(emb_cost, w_assoc, bottom=0.5):
    """compute_aw_max_metric (utils/association.py:320-374) restated."""
    e = np.ascontiguousarray(emb_cost, np.float64)
    out = np.zeros_like(e)
    lib().bxo_aw_max_metric(_d(e), e.shape[0], e.shape[1], float(w_assoc), float(bottom),
                            _d(out))
    return out


def fuse_score(cost, confs):
    c = np.array(cost, np.float64, order="C", copy=True)
    confs = np.ascontiguousarray(confs, np.float64)
    lib().bxo_fuse_score(_d(c), c.shape[0], c.shape[1], _d(confs))
    return c


def embedding_distance(trk, det):
    trk = np.ascontiguousarray(trk, np.float32)
    det = np.ascontiguousarray(det, np.float32)
    out = np.zeros((trk.shape[0], det.shape[0]))
    lib().bxo_embedding_distance(trk.ctypes.data_as(_fp), trk.shape[0], det.ctypes.data_as(_fp),
                                 det.shape[0], trk.shape[1], _d(out))
    return out


def nn_cosine_distance(samples, off, feats):
    """StrongSort NN gallery distance: samples [G,F] f64 with per-target offsets off [T+1],
    feats [D,F] -> [T,D]."""
    samples = np.ascontiguousarray(samples, np.float64)
    feats = np.ascontiguousarray(feats, np.float64)
    off = np.ascontiguousarray(off, np.int32)
    T, D = off.shape[0] - 1, feats.shape[0]
    F = feats.shape[1] if feats.ndim == 2 else samples.shape[1]
    out = np.zeros((T, D))
    lib().bxo_nn_cosine_distance(_d(samples), off.ctypes.data_as(_ip), T, _d(feats), D, F, _d(out))
    return out


KF_KIND = {"xyah": 0, "xywh": 1}


def kf_initiate(kind, meas):
    meas = np.ascontiguousarray(meas, np.float64)
    mean, cov = np.zeros(8), np.zeros((8, 8))
    lib().bxo_kf_initiate(KF_KIND[kind], _d(meas), _d(mean), _d(cov))
    return mean, cov


def kf_multi_predict(kind, mean, cov):
    mean = np.array(mean, np.float64, order="C", copy=True)
    cov = np.array(cov, np.float64, order="C", copy=True)
    lib().bxo_kf_multi_predict(KF_KIND[kind], mean.shape[0], _d(mean), _d(cov))
    return mean, cov


def kf_update(kind, mean, cov, z, conf=0.0):
    mean = np.array(mean, np.float64, order="C", copy=True)
    cov = np.array(cov, np.float64, order="C", copy=True)
    z = np.ascontiguousarray(z, np.float64)
    lib().bxo_kf_update(KF_KIND[kind], _d(mean), _d(cov), _d(z), float(conf))
    return mean, cov


def kf_gating_distance(kind, mean, cov, z):
    mean = np.ascontiguousarray(mean, np.float64)
    cov = np.ascontiguousarray(cov, np.float64)
    z = np.ascontiguousarray(z, np.float64).reshape(-1, 4)
    out = np.zeros(z.shape[0])
    lib().bxo_kf_gating_distance(KF_KIND[kind], _d(mean), _d(cov), _d(z), z.shape[0], _d(out))
    return out


def linear_assignment(cost, thresh):
    cost = np.ascontiguousarray(cost, np.float64)
    nr, nc = cost.shape
    k = max(1, min(nr, nc))
    m = np.zeros(2 * k, np.int32)
    ua = np.zeros(max(nr, 1), np.int32)
    ub = np.zeros(max(nc, 1), np.int32)
    nm, nua, nub = C.c_int(), C.c_int(), C.c_int()
    ip = lambda a: a.ctypes.data_as(_ip)  # noqa: E731
    lib().bxo_linear_assignment(_d(cost), nr, nc, float(thresh), ip(m), C.byref(nm), ip(ua),
                                C.byref(nua), ip(ub), C.byref(nub))
    return m[: 2 * nm.value].reshape(-1, 2), ua[: nua.value], ub[: nub.value]


def pyset_order(adds):
    """The oracle's emulation of CPython's set iteration order (bxo_pyset_order)."""
    a = np.ascontiguousarray(adds, np.int64)
    out = np.zeros(max(a.size, 1), np.int64)
    m = lib().bxo_pyset_order(a.ctypes.data, a.size, out.ctypes.data)
    return out[:m].tolist()


def kf_xysr(op, x, P, arg=None, q_xy=0.01, q_s=0.0001):
    """Op-level XYSR filter (bxo_kf_xysr_*): op in initiate (arg = boxes [n,4]), predict,
    update (arg = z [n,4]); returns new (x [n,7], P [n,7,7])."""
    L = lib()
    n = (arg if op == "initiate" else x).shape[0]
    x = np.zeros((n, 7)) if op == "initiate" else np.array(x, np.float64).reshape(n, 7)
    P = np.zeros((n, 7, 7)) if op == "initiate" else np.array(P, np.float64).reshape(n, 7, 7)
    if op == "initiate":
        L.bxo_kf_xysr_initiate(n, _d(np.ascontiguousarray(arg, np.float64)), _d(x), _d(P))
    elif op == "predict":
        L.bxo_kf_xysr_predict(n, _d(x), _d(P), q_xy, q_s)
    else:
        L.bxo_kf_xysr_update(n, _d(x), _d(P), _d(np.ascontiguousarray(arg, np.float64)))
    return x, P


def kf_boost(op, x, P, arg=None):
    """Op-level BoostTrack filter (bxo_kf_boost_*): initiate (arg = z [n,4]), predict, update
    (arg = z), mh_dist (arg = xyxy detections [m,4]; returns [m,n])."""
    L = lib()
    if op == "mh_dist":
        d = np.ascontiguousarray(arg, np.float64)
        x = np.ascontiguousarray(x, np.float64)
        P = np.ascontiguousarray(P, np.float64)
        out = np.zeros((d.shape[0], x.shape[0]))
        L.bxo_kf_boost_mh_dist(d.shape[0], _d(d), x.shape[0], _d(x), _d(P), _d(out))
        return out
    n = (arg if op == "initiate" else x).shape[0]
    x = np.zeros((n, 8)) if op == "initiate" else np.array(x, np.float64).reshape(n, 8)
    P = np.zeros((n, 8, 8)) if op == "initiate" else np.array(P, np.float64).reshape(n, 8, 8)
    if op == "initiate":
        L.bxo_kf_boost_initiate(n, _d(np.ascontiguousarray(arg, np.float64)), _d(x), _d(P))
    elif op == "predict":
        L.bxo_kf_boost_predict(n, _d(x), _d(P))
    else:
        L.bxo_kf_boost_update(n, _d(x), _d(P), _d(np.ascontiguousarray(arg, np.float64)))
    return x, P


NR_CLASSES = 80  # BaseTracker(nr_classes=80) (basetracker.py:23)


class OracleTracker:
    """Per-sequence CPU oracle tracker with the reference ``update`` contract.

    ``per_class=True`` restates BaseTracker.per_class_decorator (basetracker.py:155-201): one
    update per class id 0..79 on that class's detections with the frame counter held; ByteTrack /
    BoT-SORT swap only the active list (lost list and ids shared), OCSort runs one tracker per
    class with the class-global id counter, BoostTrack calls its one tracker per class (D10)."""

    def __init__(self, kind: str, **p):
        L = lib()
        self.kind = kind
        self.per_class = bool(p.pop("per_class", False))
        if self.per_class and kind == "strongsort":
            raise NotImplementedError("StrongSort has no per-class mode (tracker_zoo.py:85-86)")
        self._p = dict(p)
        self._oc = {}  # OCSort per-class trackers
        self._frame = 0
        if kind == "bytetrack":
            self.h = L.bxo_bytetrack_new(
                p.get("min_conf", 0.1), p.get("track_thresh", 0.45), p.get("match_thresh", 0.8),
                int(p.get("track_buffer", 25)), int(p.get("frame_rate", 30)))
        elif kind == "botsort":
            self.h = L.bxo_botsort_new(
                p.get("track_high_thresh", 0.5), p.get("track_low_thresh", 0.1),
                p.get("new_track_thresh", 0.6), int(p.get("track_buffer", 30)),
                p.get("match_thresh", 0.8), p.get("proximity_thresh", 0.5),
                p.get("appearance_thresh", 0.25), int(p.get("frame_rate", 30)),
                int(bool(p.get("fuse_first_associate", False))), int(bool(p.get("with_reid", True))))
        elif kind == "ocsort":  # YAML defaults (configs/trackers/ocsort.yaml)
            self.h = L.bxo_ocsort_new(
                p.get("min_conf", 0.1), p.get("det_thresh", 0.6), int(p.get("max_age", 30)),
                int(p.get("min_hits", 3)), p.get("asso_threshold", 0.3), int(p.get("delta_t", 3)),
                p.get("inertia", 0.1), int(bool(p.get("use_byte", False))),
                p.get("Q_xy_scaling", 0.01), p.get("Q_s_scaling", 0.0001))
            # asso_func (utils/iou.py registry); centroid normalises by the fixtures' 1920x1080
            # frame (make_golden.run_tracker's image), overridable with frame_w / frame_h
            L.bxo_ocsort_set_asso(self.h, ASSO_KIND[p.get("asso_func", "iou")],
                                  float(p.get("frame_w", 1920)), float(p.get("frame_h", 1080)))
        elif kind == "boosttrack":
            self._bp = boost_params(**p)
            self.h = L.bxo_boost_new(C.byref(self._bp))
        elif kind == "strongsort":
            self._sp = ss_params(**p)
            self.h = L.bxo_ss_new(C.byref(self._sp))
            if p.get("handle_occlusions", False):  # OcclusionAwareTracker post-process
                L.bxo_ss_set_occlusion(self.h, 1, float(p.get("occlusion_threshold", 0.3)))
        else:
            raise KeyError(kind)
        self._cap = 1024

    def update(self, dets, embs=None, warp=None):
        if self.per_class:
            return self._update_per_class(dets, embs, warp)
        return self._update_one(dets, embs, warp)

    def _update_per_class(self, dets, embs, warp):
        """``warp``: None, one 2x3 warp for every class call, or [NR_CLASSES, 2, 3] — one per
        class call, as the reference calls cmc.apply in each (botsort.py:218,
        boosttrack.py:243-246)."""
        L = lib()
        dets = np.asarray(dets, np.float64).reshape(-1, 6)
        fc = self._frame
        outs = []
        wall = None if warp is None else np.asarray(warp, np.float64)
        for c in range(NR_CLASSES):
            warp = None if wall is None else (wall[c] if wall.ndim == 3 else wall)
            idx = np.flatnonzero(dets[:, 5].astype(np.float32) == c)
            cd = dets[idx]
            ce = None if embs is None else np.asarray(embs)[idx]
            if self.kind == "ocsort":
                if c not in self._oc:
                    self._oc[c] = OracleTracker("ocsort", **self._p)
                    self._oc[c]._frame_sync(fc)
                t = self._oc[c]
                L.bxo_ocsort_set_id_count(t.h, self._ids_shared())
                o = t._update_one(cd, ce, warp)
                self._oc_ids = L.bxo_ocsort_id_count(t.h)
            else:
                if self.kind == "boosttrack":
                    L.bxo_boost_set_frame_count(self.h, fc)
                else:
                    L.bxo_select_class(self.h, c)
                    L.bxo_set_frame_count(self.h, fc)
                o = self._update_one(cd, ce, warp)
            if o.size:
                outs.append(o)
        self._frame = fc + 1
        return np.vstack(outs) if outs else np.empty((0, 8))

    def _ids_shared(self):
        return getattr(self, "_oc_ids", 0)

    def _frame_sync(self, fc):
        """A per-class OCSort tracker created at frame fc+1 has seen fc (empty) frames before."""
        for _ in range(fc):
            self._update_one(np.empty((0, 6)), None, None)

    def _update_one(self, dets, embs=None, warp=None):
        dets = np.ascontiguousarray(np.asarray(dets, np.float64).reshape(-1, 6))
        n = dets.shape[0]
        e_ptr, f, is64 = None, 0, 0
        if embs is not None and n:
            embs = np.ascontiguousarray(embs)
            if embs.dtype == np.float64:
                is64 = 1
            else:
                embs = embs.astype(np.float32, copy=False)
            f = embs.shape[1]
            e_ptr = embs.ctypes.data_as(C.c_void_p)
        if self.kind == "ocsort":
            # BaseTracker.setup_decorator rounds dets to float32 (basetracker.py:122-128)
            d32 = np.ascontiguousarray(dets.astype(np.float32).astype(np.float64))
            cap = max(self._cap, 2 * n + 64)
            out = np.zeros((cap, 8))
            m = lib().bxo_ocsort_update(self.h, _d(d32), n, _d(out), cap)
            if m < 0:
                raise RuntimeError(f"oracle update failed ({m})")
            return out[:m].copy()
        w = None if warp is None else _d(np.ascontiguousarray(warp, np.float64).reshape(6))
        if self.kind == "strongsort":  # no setup_decorator: dets stay float64
            ep, fd = None, 0
            if embs is not None and n:
                e64 = np.ascontiguousarray(embs, np.float64)
                ep, fd = e64.ctypes.data_as(C.c_void_p), e64.shape[1]
            cap = max(self._cap, 2 * n + 64)
            out = np.zeros((cap, 10))
            m = lib().bxo_ss_update(self.h, _d(dets), n, ep, fd, w, _d(out), cap)
            if m == -5:  # the reference's _resolve_mutual_occlusion
                raise TypeError("'int' object is not iterable")
            if m < 0:
                raise RuntimeError(f"oracle update failed ({m})")
            return out[:m].copy()
        if self.kind == "boosttrack":
            d32 = np.ascontiguousarray(dets.astype(np.float32).astype(np.float64))
            ep, fd = None, 0
            if embs is not None and n and self._bp.with_reid:
                e64 = np.ascontiguousarray(embs, np.float64)
                ep, fd = e64.ctypes.data_as(C.c_void_p), e64.shape[1]
            cap = max(self._cap, 2 * n + 64)
            out = np.zeros((cap, 8))
            m = lib().bxo_boost_update(self.h, _d(d32), n, ep, fd, w, _d(out), cap)
            if m < 0:
                raise RuntimeError(f"oracle update failed ({m})")
            return out[:m].copy()
        while True:
            cap = max(self._cap, n + 16)
            out = np.zeros((cap, 8))
            m = lib().bxo_update(self.h, _d(dets), n, e_ptr, f, is64, w, _d(out), cap)
            if m == -2:
                raise RuntimeError("oracle output buffer too small")
            if m < 0:
                raise RuntimeError(f"oracle update failed ({m})")
            return out[:m].copy()

    @property
    def id_count(self):
        if self.kind == "ocsort":
            return lib().bxo_ocsort_id_count(self.h)
        if self.kind == "boosttrack":
            return lib().bxo_boost_id_count(self.h)
        if self.kind == "strongsort":
            return lib().bxo_ss_next_id(self.h) - 1
        return lib().bxo_id_count(self.h)

    def state_set(self, ids, a=None, b=None):
        """Kalman state edit by track id, as the engines' state_set (ByteTrack/BoT-SORT/StrongSort:
        mean, covariance; OCSort: x [7], P [49]; BoostTrack: x [8], P [64])."""
        ids = np.ascontiguousarray(ids, np.int32).reshape(-1)
        fn = {"bytetrack": "bxo_state_set", "botsort": "bxo_state_set",
              "ocsort": "bxo_ocsort_state_set", "boosttrack": "bxo_boost_state_set",
              "strongsort": "bxo_ss_state_set"}[self.kind]
        a = None if a is None else np.ascontiguousarray(a, np.float64)
        b = None if b is None else np.ascontiguousarray(b, np.float64)
        found = getattr(lib(), fn)(self.h, ids.size, ids.ctypes.data,
                                   None if a is None else a.ctypes.data,
                                   None if b is None else b.ctypes.data)
        assert found == ids.size, "state_set: unknown track id"

    def tracks(self):
        """ByteTrack / BoT-SORT: tracked then lost list — ids, states, means [n,8], covs [n,8,8]."""
        L = lib()
        n = L.bxo_tracks(self.h, 0, None, None, None, None)
        ids = np.zeros(max(n, 1), np.int32)
        st = np.zeros(max(n, 1), np.int32)
        mean = np.zeros((max(n, 1), 8))
        cov = np.zeros((max(n, 1), 8, 8))
        L.bxo_tracks(self.h, n, ids.ctypes.data, st.ctypes.data, mean.ctypes.data,
                     cov.ctypes.data)
        return {"id": ids[:n], "state": st[:n], "mean": mean[:n], "covariance": cov[:n]}

    def ocsort_tracks(self):
        """OCSort track list (list order): ids, XYSR means [n,7], covariances [n,7,7]."""
        n = lib().bxo_ocsort_tracks(self.h, 0, None, None, None)
        ids = np.zeros(max(n, 1), np.int32)
        x = np.zeros((max(n, 1), 7))
        P = np.zeros((max(n, 1), 7, 7))
        lib().bxo_ocsort_tracks(self.h, n, ids.ctypes.data, x.ctypes.data, P.ctypes.data)
        return {"id": ids[:n], "x": x[:n], "P": P[:n]}

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            free = {"ocsort": lib().bxo_ocsort_free, "boosttrack": lib().bxo_boost_free,
                    "strongsort": lib().bxo_ss_free}
            free.get(self.kind, lib().bxo_free)(h)
            self.h = None

