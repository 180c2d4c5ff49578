"""The bench workloads (BASELINE.json configs): tracker, objects per sequence,
ReID width and tracker parameters (the reference's YAML / constructor defaults) per bench.py
--config, plus the StrongSort engine capacities.  Shared by bench.py, the GPU tests that run a
config at its stated size (tests/test_gpu_parity.py) and the diagnostic tools, so a test does not
import the bench script."""
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

CONFIGS = {
    # name: (tracker, n_obj, emb_dim, tracker params (YAML defaults))
    "botsort": ("botsort", 256, 512, dict(track_high_thresh=0.6, track_low_thresh=0.1,
                                          new_track_thresh=0.7, track_buffer=30,
                                          match_thresh=0.8, proximity_thresh=0.5,
                                          appearance_thresh=0.25)),
    # C3's tracker and sizes on the crowded layout (random centres, heavy overlap: many gated
    # pairs per track, non-trivial LAP components) — SURVEY §8(d)'s crowded variant
    "botsort_crowded": ("botsort", 256, 512, dict(track_high_thresh=0.6, track_low_thresh=0.1,
                                                  new_track_thresh=0.7, track_buffer=30,
                                                  match_thresh=0.8, proximity_thresh=0.5,
                                                  appearance_thresh=0.25)),
    "bytetrack": ("bytetrack", 256, 0, dict(min_conf=0.1, track_thresh=0.6, match_thresh=0.9,
                                            track_buffer=30)),
    # OCSort (configs[0]'s tracker, YAML defaults): ~20 tracks/frame like MOT17-mini, and the
    # 256-track geometry of configs[1]; detection confidences span both BYTE splits
    "ocsort": ("ocsort", 40, 0, dict(min_conf=0.1, det_thresh=0.6, max_age=30, min_hits=3,
                                     asso_threshold=0.3, delta_t=3, inertia=0.1, use_byte=False,
                                     Q_xy_scaling=0.01, Q_s_scaling=0.0001)),
    "ocsort256": ("ocsort", 256, 0, dict(min_conf=0.1, det_thresh=0.6, max_age=30, min_hits=3,
                                         asso_threshold=0.3, delta_t=3, inertia=0.1,
                                         use_byte=False, Q_xy_scaling=0.01, Q_s_scaling=0.0001)),
    # BoostTrack++ (configs[4]'s tracker, YAML defaults) on MOT17-ablation-sized sequences
    # (T ~ 20-40 live tracks, D ~ 30 dets, 512-d ReID)
    "boosttrack": ("boosttrack", 60, 512, dict(
        max_age=60, min_hits=3, det_thresh=0.6, iou_threshold=0.3, use_ecc=True,
        min_box_area=10, aspect_ratio_thresh=1.6, lambda_iou=0.5, lambda_mhd=0.25,
        lambda_shape=0.25, use_dlo_boost=True, use_duo_boost=True, dlo_boost_coef=0.65,
        s_sim_corr=False, use_rich_s=True, use_sb=True, use_vt=True, with_reid=True)),
    # StrongSort (configs[3]'s tracker, constructor defaults, born Confirmed): many MOT-sized
    # sequences with 512-d ReID, and configs[3] itself (1024 tracks x ~512 dets x 2048-d) as one
    # sequence
    "strongsort": ("strongsort", 48, 512, dict(
        min_conf=0.1, max_cos_dist=0.15, max_iou_dist=0.7, max_age=50, n_init=2, nn_budget=150,
        mc_lambda=0.995, ema_alpha=0.9, conf_thresh_high=0.7, conf_thresh_low=0.3,
        id_preservation_weight=0.1, crowd_detection=True, born_confirmed=True)),
    # C5 (BASELINE.json configs[4]): BoostTrack++ on 8 MOT17-ablation-like sequences sharded
    # over the ranks (strong scaling of a fixed set): MOT17-02 / MOT17-04 public detections with
    # identity-linked synthetic ReID + 6 synthetic 60-object sequences (SURVEY §8(d) stand-in)
    "boosttrack_mot8": ("boosttrack", 60, 512, dict(
        max_age=60, min_hits=3, det_thresh=0.6, iou_threshold=0.3, use_ecc=True,
        min_box_area=10, aspect_ratio_thresh=1.6, lambda_iou=0.5, lambda_mhd=0.25,
        lambda_shape=0.25, use_dlo_boost=True, use_duo_boost=True, dlo_boost_coef=0.65,
        s_sim_corr=False, use_rich_s=True, use_sb=True, use_vt=True, with_reid=True)),
    "strongsort_c4": ("strongsort", 1024, 2048, dict(
        min_conf=0.1, max_cos_dist=0.15, max_iou_dist=0.7, max_age=50, n_init=2, nn_budget=150,
        mc_lambda=0.995, ema_alpha=0.9, conf_thresh_high=0.7, conf_thresh_low=0.3,
        id_preservation_weight=0.1, crowd_detection=True, born_confirmed=True)),
}
DEFAULT_SEQS = {"strongsort": 256, "strongsort_c4": 1}
MOT_DETS = ROOT / "tests" / "golden" / "mot17_public_dets.npz"  # C5's real-data sequences
C5_TOTAL = 8
# StrongSort engine capacities (track slots, detections per frame, pool vectors per slot); the C4
# ones are also tests/test_gpu_parity.py::test_strongsort_c4_size_vs_oracle's
SS_C4_CAPS = dict(track_cap=1024, det_cap=1024, vec_cap=64)


def ss_caps(config, n_obj):
    if config == "strongsort_c4":
        return dict(SS_C4_CAPS)
    return dict(track_cap=min(1024, max(96, 2 * n_obj)), det_cap=min(1024, max(64, n_obj)),
                vec_cap=64)


OCS_CONF_LO = 0.3  # OCSort / BoostTrack scenes: confidences U(0.3, 1) -> ~40% below det_thresh


def bench_engine(config, n_seq, track_cap=512, det_cap=256, overlap=True, early=False):
    """The engine bench.py times for ``config`` with ``n_seq`` sequences per launch, and its
    pipeline stages (the probe targets).  BoT-SORT / ByteTrack: ``track_cap`` / ``det_cap`` slots
    and overlap mode (each step's feature EMA left unjoined: the caller keeps a step's inputs
    alive until the next step is enqueued)."""
    import os

    from .engine import (BoostEngine, BoostParams, Engine, EngineParams, OcsortEngine,
                         OcsortParams, SsEngine, SsParams)

    kind, n_obj, F, params = CONFIGS[config]
    if kind == "strongsort":
        return (SsEngine(n_seq=n_seq, emb_dim=F, params=SsParams(**params),
                         **ss_caps(config, n_obj)), list(SsEngine.STAGES))
    if kind == "boosttrack":
        return (BoostEngine(n_seq=n_seq, track_cap=128, det_cap=max(64, n_obj), emb_dim=F,
                            params=BoostParams(**params)), list(BoostEngine.STAGES))
    if kind == "ocsort":
        tcap = int(os.environ.get("BX_OCS_TRACK_CAP", max(64, 2 * n_obj)))
        return (OcsortEngine(n_seq=n_seq, track_cap=tcap, det_cap=max(64, n_obj),
                             params=OcsortParams(**params)), [])
    eng = Engine(kind, n_seq=n_seq, track_cap=track_cap, det_cap=det_cap, emb_dim=F,
                 params=EngineParams(**params))
    eng.set_overlap(overlap)
    if early and F:
        eng.set_early_features(True)
    return eng, [s for s in Engine.STAGES
                 if F or s not in ("det_features", "gate", "cosine", "features")]


class BenchFrames:
    """bench.py's input stream for ``config`` on ``device``: ``frame(t)`` (t = 1, 2, ... in order:
    the GPU generator draws frames sequentially) -> ``(dets, det_off, embs)`` device tensors in
    the dtypes the engine consumes (BoT-SORT / ByteTrack / OCSort: float32 detections, float32
    embeddings; BoostTrack: float64 embeddings; StrongSort: float64 detections and embeddings).

    Synthetic configs draw ``n_seq`` sequences from ``TorchSceneBatch(seed=1000 + rank)``; C5
    (``boosttrack_mot8``) plays this rank's LPT shard of its eight sequences (``self.mine``, global
    indices into ``self.c5``), so ``self.n_seq`` is that shard's size."""

    def __init__(self, config, n_seq, device, rank=0, world=1):
        import numpy as np

        self.config, self.device = config, device
        kind, n_obj, F, _ = CONFIGS[config]
        self.kind, self.emb_dim = kind, F
        self.c5 = self.mine = None
        if config == "boosttrack_mot8":
            from .shard import shard_sequences
            from .synth import c5_sequences

            if world > C5_TOTAL:
                raise SystemExit(f"boosttrack_mot8 has {C5_TOTAL} sequences: at most {C5_TOTAL} "
                                 "ranks")
            self.c5 = c5_sequences(MOT_DETS, F)
            self.mine = shard_sequences([nf for _, _, nf in self.c5], world, rank)
            self.n_seq = len(self.mine)
            self.n_frames_max = min(self.c5[g][2] for g in self.mine)
            self.layout = "MOT17-02/04 public dets + synthetic"
            self._np = np
        else:
            from .synth import TorchSceneBatch

            self.n_seq = n_seq
            self.n_frames_max = None
            self.layout = "crowded" if config.endswith("_crowded") else "grid"
            lo = kind in ("ocsort", "boosttrack", "strongsort")
            self.gen = TorchSceneBatch(n_seq, n_obj, emb_dim=F, seed=1000 + rank, device=device,
                                       layout=self.layout,
                                       **(dict(conf_lo=OCS_CONF_LO) if lo else {}))
        self._next = 1

    def frame(self, t):
        if t != self._next:
            raise ValueError(f"frames are drawn in order: expected frame {self._next}, got {t}")
        self._next += 1
        if self.c5 is not None:
            import torch

            np = self._np
            fr = [self.c5[g][1].frame(t) for g in self.mine]
            off = np.zeros(self.n_seq + 1, np.int32)
            off[1:] = np.cumsum([f[0].shape[0] for f in fr])
            d = np.concatenate([f[0] for f in fr], 0).astype(np.float32)
            e = np.concatenate([f[1] for f in fr], 0).astype(np.float64)
            return (torch.from_numpy(d).to(self.device), torch.from_numpy(off).to(self.device),
                    torch.from_numpy(e).to(self.device))
        d, o, e = self.gen.frame(t)
        if self.kind == "boosttrack":
            e = e.double()
        elif self.kind == "strongsort":
            d, e = d.double(), e.double()
        return d, o, e
