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
