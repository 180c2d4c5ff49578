"""ctypes binding of libbxassoc.so (include/bxassoc.h).

The HIP library is the product: there is no CPU fallback.  Importing this module never needs a
GPU, but any call into the engine on a machine without the built library or without a HIP
device raises ``NativeUnavailable`` — loudly, so a silent eager/CPU path can never stand in.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
CSRC = PKG / "csrc"
LIB_DIR = PKG / "lib"
LIB_PATH = LIB_DIR / "libbxassoc.so"
HEADER = REPO / "include" / "bxassoc.h"
HEADER_OCS = REPO / "include" / "bxocsort.h"
HEADER_BOOST = REPO / "include" / "bxboost.h"
HEADER_SS = REPO / "include" / "bxstrongsort.h"
HEADER_IO = REPO / "include" / "bxio.h"

HIPCC_FLAGS = [
    "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
    # numpy-identical rounding: no FMA contraction, IEEE f32 division/sqrt
    "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
    # MFMA accumulators in the VGPR form: the compiler otherwise copies the StrongSort NN
    # kernel's accumulator tiles between VGPRs and AGPRs around every k-block
    "-mllvm", "-amdgpu-mfma-vgpr-form=1",
]
SOURCES = ["bx_engine.hip", "bx_ops.hip", "bx_ocsort.hip", "bx_nn.hip", "bx_boost.hip",
           "bx_strongsort.hip", "bx_io.cpp"]


class NativeUnavailable(RuntimeError):
    pass


def _deps(src: Path, seen=None) -> list:
    """src and the in-tree headers it includes (transitively)."""
    import re

    seen = set() if seen is None else seen
    if src in seen or not src.exists():
        return []
    seen.add(src)
    out = [src]
    for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', src.read_text(), re.M):
        for d in (src.parent, REPO / "include"):
            if (d / inc).exists():
                out += _deps((d / inc).resolve(), seen)
                break
    return out


def _toolchain_stamp(hipcc: str, flags: list) -> str:
    """Hash of the compile flags and the compiler's version: objects built under another stamp
    are stale even when their sources did not change."""
    import hashlib

    try:
        ver = subprocess.run([hipcc, "--version"], capture_output=True, text=True).stdout
    except OSError:
        ver = ""
    return hashlib.sha256(("\0".join(flags) + "\0" + ver).encode()).hexdigest()[:16]


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile the HIP extension for gfx950 in-tree (boxmot_amd/lib/libbxassoc.so): one object per
    translation unit (compiled in parallel, and only when it or a header it includes changed, or
    the flags / compiler did), then one link.  Temporary outputs carry the process id, so two
    processes building at once never replace each other's half-written file."""
    from concurrent.futures import ThreadPoolExecutor

    objdir = LIB_DIR / "obj"
    objdir.mkdir(parents=True, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    # BX_HIPCC_EXTRA: extra compile flags for a debug build (e.g. -DBX_CHECK: device-side bounds
    # checks latched as engine errors); part of the toolchain stamp, so switching rebuilds
    flags = [f for f in HIPCC_FLAGS if f != "-shared"] + os.environ.get("BX_HIPCC_EXTRA", "").split()
    link_flags = [f for f in HIPCC_FLAGS if f.startswith("--offload-arch")] + ["-shared", "-fPIC"]
    stamp_file = objdir / "toolchain.stamp"
    stamp = _toolchain_stamp(hipcc, flags)
    if not stamp_file.exists() or stamp_file.read_text().strip() != stamp:
        force = True
    stale = []
    objs = []
    for s in SOURCES:
        src = CSRC / s
        obj = objdir / (s + ".o")
        objs.append(obj)
        if force or not obj.exists() or any(d.stat().st_mtime > obj.stat().st_mtime
                                            for d in _deps(src)):
            stale.append((src, obj))

    def compile_one(so):
        src, obj = so
        tmp = obj.with_suffix(f".o.{os.getpid()}.tmp")
        r = subprocess.run([hipcc, *flags, "-c", "-o", str(tmp), str(src)], capture_output=True,
                           text=True)
        if r.returncode != 0:
            tmp.unlink(missing_ok=True)
            raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stderr}")
        if verbose and r.stderr:
            print(r.stderr)
        os.replace(tmp, obj)

    if stale:
        with ThreadPoolExecutor(max_workers=min(len(stale), os.cpu_count() or 1)) as ex:
            list(ex.map(compile_one, stale))
        stamp_file.write_text(stamp + "\n")
    if not stale and LIB_PATH.exists() and all(
            o.stat().st_mtime <= LIB_PATH.stat().st_mtime for o in objs):
        return LIB_PATH
    LIB_DIR.mkdir(exist_ok=True)
    tmp = LIB_PATH.with_suffix(f".so.{os.getpid()}.tmp")
    r = subprocess.run([hipcc, *link_flags, "-o", str(tmp), *[str(o) for o in objs]],
                       capture_output=True, text=True)
    if r.returncode != 0:
        tmp.unlink(missing_ok=True)
        raise RuntimeError(f"hipcc link failed:\n{r.stderr}")
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


class BxConfig(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("n_seq", C.c_int32), ("track_cap", C.c_int32),
        ("det_cap", C.c_int32), ("emb_dim", C.c_int32), ("emb_f64", C.c_int32),
        ("min_conf", C.c_double), ("track_thresh", C.c_double), ("match_thresh", C.c_double),
        ("track_buffer", C.c_int32), ("frame_rate", C.c_int32),
        ("track_high_thresh", C.c_double), ("track_low_thresh", C.c_double),
        ("new_track_thresh", C.c_double), ("proximity_thresh", C.c_double),
        ("appearance_thresh", C.c_double),
        ("fuse_first_associate", C.c_int32), ("with_reid", C.c_int32),
    ]


class BxOcsortConfig(C.Structure):
    _fields_ = [
        ("n_seq", C.c_int32), ("track_cap", C.c_int32), ("det_cap", C.c_int32),
        ("min_conf", C.c_double), ("det_thresh", C.c_double), ("asso_threshold", C.c_double),
        ("inertia", C.c_double), ("q_xy_scaling", C.c_double), ("q_s_scaling", C.c_double),
        ("max_age", C.c_int32), ("min_hits", C.c_int32), ("delta_t", C.c_int32),
        ("use_byte", C.c_int32), ("asso_kind", C.c_int32), ("frame_w", C.c_double),
        ("frame_h", C.c_double),
    ]


class BxBoostConfig(C.Structure):
    _fields_ = [
        ("n_seq", C.c_int32), ("track_cap", C.c_int32), ("det_cap", C.c_int32),
        ("emb_dim", C.c_int32), ("max_age", C.c_int32), ("min_hits", C.c_int32),
        ("det_thresh", C.c_double), ("iou_threshold", C.c_double), ("min_box_area", C.c_double),
        ("aspect_ratio_thresh", C.c_double), ("lambda_iou", C.c_double),
        ("lambda_mhd", C.c_double), ("lambda_shape", C.c_double), ("dlo_boost_coef", C.c_double),
        ("use_ecc", C.c_int32), ("use_dlo_boost", C.c_int32), ("use_duo_boost", C.c_int32),
        ("s_sim_corr", C.c_int32), ("use_rich_s", C.c_int32), ("use_sb", C.c_int32),
        ("use_vt", C.c_int32), ("with_reid", C.c_int32),
    ]


class BxSsConfig(C.Structure):
    _fields_ = [
        ("n_seq", C.c_int32), ("track_cap", C.c_int32), ("det_cap", C.c_int32),
        ("emb_dim", C.c_int32), ("vec_cap", C.c_int32), ("min_conf", C.c_double),
        ("max_cos_dist", C.c_double), ("max_iou_dist", C.c_double), ("max_age", C.c_int32),
        ("n_init", C.c_int32), ("nn_budget", C.c_int32), ("mc_lambda", C.c_double),
        ("ema_alpha", C.c_double), ("conf_thresh_high", C.c_double),
        ("conf_thresh_low", C.c_double), ("id_preservation_weight", C.c_double),
        ("crowd_detection", C.c_int32), ("born_confirmed", C.c_int32),
    ]


# every symbol include/*.h declares (checked by tests/test_native_abi.py)
EXPORTS = [
    "bx_last_error", "bx_device_count", "bx_engine_create", "bx_engine_destroy",
    "bx_engine_reset", "bx_engine_step", "bx_engine_update_host", "bx_engine_status",
    "bx_engine_counters_host", "bx_engine_set_id_count", "bx_engine_tracks_host", "bx_engine_class_tracks_host",
    "bx_engine_state_set_host", "bx_ocsort_state_set_host", "bx_boost_state_set_host",
    "bx_ss_state_set_host",
    "bx_engine_probe", "bx_engine_probe_read", "bx_engine_set_overlap", "bx_engine_frame_stats_host",
    "bx_iou_batch", "bx_pairwise_cost", "bx_aw_max_metric", "bx_fuse_score", "bx_embedding_distance", "bx_kf_initiate",
    "bx_kf_multi_predict", "bx_kf_update", "bx_kf_gating_distance", "bx_linear_assignment", "bx_lapjv",
    "bx_linear_assignment_ex", "bx_engine_lap_ties_host", "bx_engine_lap_components_host", "bx_engine_set_lap_stats",
    "bx_engine_force_assoc_build", "bx_legacy_lap_pair", "bx_engine_set_early_features",
    "bx_engine_inputs_released",
    "bx_engine_copy_state", "bx_engine_slots_used_host", "bx_ocsort_copy_state",
    "bx_boost_copy_state", "bx_ss_copy_state",
    "bx_nn_cosine_distance", "bx_ocsort_create", "bx_ocsort_destroy", "bx_ocsort_reset", "bx_ocsort_step",
    "bx_ocsort_update_host", "bx_ocsort_status", "bx_ocsort_counters_host",
    "bx_ocsort_set_id_count", "bx_ocsort_set_frame_size", "bx_ocsort_tracks_host", "bx_ocsort_probe", "bx_ocsort_probe_read",
    "bx_ocsort_frame_stats_host", "bx_boost_create", "bx_boost_destroy", "bx_boost_reset",
    "bx_boost_step", "bx_boost_update_host", "bx_boost_status", "bx_boost_counters_host",
    "bx_boost_set_id_count", "bx_boost_tracks_host", "bx_boost_frame_stats_host",
    "bx_boost_probe", "bx_boost_probe_read", "bx_ss_create", "bx_ss_destroy", "bx_ss_reset",
    "bx_ss_step", "bx_ss_update_host", "bx_ss_status", "bx_ss_counters_host",
    "bx_ss_tracks_host", "bx_ss_frame_stats_host", "bx_ss_probe", "bx_ss_probe_read",
    "bx_ss_set_lsap_mode", "bx_ss_lsap_stats_host", "bx_ss_lsap_op",
    "bx_txt_shape", "bx_txt_read", "bx_mot_format", "bx_mot_write",
    "bx_engine_update_classes_host", "bx_ocsort_update_classes_host",
    "bx_boost_update_classes_host", "bx_kf_xysr_initiate", "bx_kf_xysr_predict",
    "bx_kf_xysr_update", "bx_kf_boost_initiate", "bx_kf_boost_predict", "bx_kf_boost_update",
    "bx_kf_boost_mh_dist", "bx_ss_track_attrs_host", "bx_ss_track_attrs_set_host",
    "bx_ss_last_feature_host", "bx_ss_last_feature_set_host",
]

_vp, _ip, _dp, _fp = C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_double), C.POINTER(C.c_float)

_SIGS = {
    "bx_last_error": ([], C.c_char_p),
    "bx_device_count": ([_ip], C.c_int),
    "bx_engine_create": ([C.POINTER(BxConfig), C.POINTER(C.c_void_p)], C.c_int),
    "bx_engine_destroy": ([_vp], C.c_int),
    "bx_engine_reset": ([_vp, C.c_int, C.c_int, _vp], C.c_int),
    "bx_engine_step": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "bx_engine_update_host": ([_vp, C.c_int, _vp, C.c_int, _vp, _vp, _vp, _ip, _vp], C.c_int),
    "bx_engine_status": ([_vp, _ip], C.c_int),
    "bx_engine_probe": ([_vp, C.c_int], C.c_int),
    "bx_engine_set_overlap": ([_vp, C.c_int], C.c_int),
    "bx_engine_set_early_features": ([_vp, C.c_int], C.c_int),
    "bx_engine_probe_read": ([_vp, _dp, _ip], C.c_int),
    "bx_engine_frame_stats_host": ([_vp, C.c_int, C.c_int, C.POINTER(C.c_int64)], C.c_int),
    "bx_engine_counters_host": ([_vp, C.c_int, _ip, _ip, _ip, _ip], C.c_int),
    "bx_engine_set_id_count": ([_vp, C.c_int, C.c_int, _vp], C.c_int),
    "bx_engine_tracks_host": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _ip,
                               _ip], C.c_int),
    "bx_engine_class_tracks_host": ([_vp, C.c_int, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp,
                                     _vp, _vp, _vp], C.c_int),
    "bx_iou_batch": ([_vp, C.c_int, _vp, C.c_int, _vp, _vp], C.c_int),
    "bx_pairwise_cost": ([C.c_int, _vp, C.c_int, C.c_int, _vp, C.c_int, C.c_int, C.c_double,
                          C.c_double, _vp, _vp], C.c_int),
    "bx_txt_shape": ([C.c_char_p, C.POINTER(C.c_int64), C.POINTER(C.c_int32)], C.c_int),
    "bx_txt_read": ([C.c_char_p, _vp, C.c_int64, C.c_int32], C.c_int),
    "bx_mot_format": ([_vp, C.c_int64, C.c_int32, C.c_int32, _vp], C.c_int),
    "bx_mot_write": ([C.c_char_p, _vp, C.c_int64, C.c_int32], C.c_int),
    "bx_aw_max_metric": ([_vp, C.c_int, C.c_int, C.c_double, C.c_double, _vp, _vp], C.c_int),
    "bx_fuse_score": ([_vp, C.c_int, C.c_int, _vp, _vp], C.c_int),
    "bx_embedding_distance": ([_vp, C.c_int, _vp, C.c_int, C.c_int, _vp, _vp], C.c_int),
    "bx_kf_initiate": ([C.c_int, C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "bx_kf_multi_predict": ([C.c_int, C.c_int, _vp, _vp, _vp], C.c_int),
    "bx_kf_update": ([C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "bx_kf_gating_distance": ([C.c_int, C.c_int, _vp, _vp, _vp, C.c_int, _vp, _vp], C.c_int),
    "bx_linear_assignment": ([_vp, C.c_int, C.c_int, C.c_double, _vp, _vp, _vp], C.c_int),
    "bx_linear_assignment_ex": ([_vp, C.c_int, C.c_int, C.c_double, _vp, _vp, _vp, _vp], C.c_int),
    "bx_engine_lap_ties_host": ([_vp, C.c_int, C.c_int, C.POINTER(C.c_int64)], C.c_int),
    "bx_engine_lap_components_host": ([_vp, C.c_int, C.c_int, C.POINTER(C.c_int64)], C.c_int),
    "bx_engine_set_lap_stats": ([_vp, C.c_int], C.c_int),
    "bx_engine_force_assoc_build": ([_vp, C.c_int], C.c_int),
    "bx_legacy_lap_pair": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "bx_engine_inputs_released": ([_vp, _vp], C.c_int),
    "bx_engine_copy_state": ([_vp, _vp], C.c_int),
    "bx_ocsort_copy_state": ([_vp, _vp], C.c_int),
    "bx_boost_copy_state": ([_vp, _vp], C.c_int),
    "bx_ss_copy_state": ([_vp, _vp], C.c_int),
    "bx_engine_slots_used_host": ([_vp, C.c_int, _ip], C.c_int),
    "bx_lapjv": ([_vp, C.c_int, C.c_int, C.c_int, C.c_double, _vp, _vp, _vp], C.c_int),
    "bx_nn_cosine_distance": ([_vp, C.c_int, _vp, C.c_int, _vp, C.c_int, C.c_int, C.c_int, _vp,
                               _vp], C.c_int),
    "bx_ocsort_create": ([C.POINTER(BxOcsortConfig), C.POINTER(C.c_void_p)], C.c_int),
    "bx_ocsort_destroy": ([_vp], C.c_int),
    "bx_ocsort_reset": ([_vp, C.c_int, C.c_int, _vp], C.c_int),
    "bx_ocsort_step": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "bx_ocsort_update_host": ([_vp, C.c_int, _vp, C.c_int, _vp, _ip, _vp], C.c_int),
    "bx_ocsort_status": ([_vp, _ip], C.c_int),
    "bx_ocsort_counters_host": ([_vp, C.c_int, _ip, _ip, _ip], C.c_int),
    "bx_ocsort_set_id_count": ([_vp, C.c_int, C.c_int, _vp], C.c_int),
    "bx_ocsort_set_frame_size": ([_vp, C.c_int, C.c_double, C.c_double, _vp], C.c_int),
    "bx_ocsort_tracks_host": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp, _ip], C.c_int),
    "bx_ocsort_probe": ([_vp, C.c_int], C.c_int),
    "bx_ocsort_frame_stats_host": ([_vp, C.c_int, C.c_int, C.POINTER(C.c_int64)], C.c_int),
    "bx_ocsort_probe_read": ([_vp, _dp, _ip], C.c_int),
    "bx_boost_create": ([C.POINTER(BxBoostConfig), C.POINTER(C.c_void_p)], C.c_int),
    "bx_boost_destroy": ([_vp], C.c_int),
    "bx_boost_reset": ([_vp, C.c_int, C.c_int, _vp], C.c_int),
    "bx_boost_step": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "bx_boost_update_host": ([_vp, C.c_int, _vp, C.c_int, _vp, _vp, _vp, _ip, _vp], C.c_int),
    "bx_boost_status": ([_vp, _ip], C.c_int),
    "bx_boost_counters_host": ([_vp, C.c_int, _ip, _ip, _ip], C.c_int),
    "bx_boost_set_id_count": ([_vp, C.c_int, C.c_int, _vp], C.c_int),
    "bx_boost_tracks_host": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _ip], C.c_int),
    "bx_boost_frame_stats_host": ([_vp, C.c_int, C.c_int, C.POINTER(C.c_int64)], C.c_int),
    "bx_boost_probe": ([_vp, C.c_int], C.c_int),
    "bx_boost_probe_read": ([_vp, _dp, _ip], C.c_int),
    "bx_ss_create": ([C.POINTER(BxSsConfig), C.POINTER(C.c_void_p)], C.c_int),
    "bx_ss_destroy": ([_vp], C.c_int),
    "bx_ss_reset": ([_vp, C.c_int, C.c_int, _vp], C.c_int),
    "bx_ss_step": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp], C.c_int),
    "bx_ss_update_host": ([_vp, C.c_int, _vp, C.c_int, _vp, _vp, _vp, _ip, _vp], C.c_int),
    "bx_ss_status": ([_vp, _ip], C.c_int),
    "bx_ss_counters_host": ([_vp, C.c_int, _ip, _ip, _ip, _ip], C.c_int),
    "bx_ss_tracks_host": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _ip], C.c_int),
    "bx_engine_state_set_host": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp], C.c_int),
    "bx_ocsort_state_set_host": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp], C.c_int),
    "bx_boost_state_set_host": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp], C.c_int),
    "bx_ss_state_set_host": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp], C.c_int),
    "bx_ss_frame_stats_host": ([_vp, C.c_int, C.c_int, C.POINTER(C.c_int64)], C.c_int),
    "bx_ss_set_lsap_mode": ([_vp, C.c_int], C.c_int),
    "bx_ss_lsap_op": ([_vp, C.c_int, C.c_int, C.c_double, C.c_int, _vp, _vp, _vp, _vp, _vp],
                      C.c_int),
    "bx_ss_lsap_stats_host": ([_vp, C.c_int, C.c_int, C.POINTER(C.c_int64)], C.c_int),
    "bx_ss_probe": ([_vp, C.c_int], C.c_int),
    "bx_ss_probe_read": ([_vp, _dp, _ip], C.c_int),
    "bx_engine_update_classes_host": ([_vp, C.c_int, _vp, C.c_int, _vp, _vp, C.c_int, _vp, _ip,
                                       _vp], C.c_int),
    "bx_ocsort_update_classes_host": ([_vp, C.c_int, C.c_int, _vp, C.c_int, _ip, _vp, _ip, _vp],
                                      C.c_int),
    "bx_boost_update_classes_host": ([_vp, C.c_int, _vp, C.c_int, _vp, _vp, C.c_int, _vp, _ip,
                                      _vp], C.c_int),
    "bx_kf_xysr_initiate": ([C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "bx_kf_xysr_predict": ([C.c_int, _vp, _vp, C.c_double, C.c_double, _vp], C.c_int),
    "bx_kf_xysr_update": ([C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "bx_kf_boost_initiate": ([C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "bx_kf_boost_predict": ([C.c_int, _vp, _vp, _vp], C.c_int),
    "bx_kf_boost_update": ([C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "bx_kf_boost_mh_dist": ([C.c_int, _vp, C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "bx_ss_track_attrs_host": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp, _vp, _ip], C.c_int),
    "bx_ss_track_attrs_set_host": ([_vp, C.c_int, C.c_int, _vp, _vp, _vp, _vp], C.c_int),
    "bx_ss_last_feature_host": ([_vp, C.c_int, C.c_int, _vp, _vp], C.c_int),
    "bx_ss_last_feature_set_host": ([_vp, C.c_int, C.c_int, _vp, _vp, C.c_int], C.c_int),
}

_lib = None


def load(path: Path | None = None):
    """Load libbxassoc.so (raises NativeUnavailable when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    # BX_LIB_PATH: load a diagnostic build (e.g. the -DBX_PHASE_TIMING stamps library)
    p = Path(path) if path else Path(os.environ.get("BX_LIB_PATH", LIB_PATH))
    if not p.exists():
        raise NativeUnavailable(
            f"{p} is missing: build the HIP extension first (python -c 'import __graft_entry__ "
            "as g; g.build()' or boxmot_amd._native.build())")
    L = C.CDLL(str(p))
    for name, (args, res) in _SIGS.items():
        fn = getattr(L, name, None)
        if fn is None and not path and "BX_LIB_PATH" in os.environ:
            continue  # (an older diagnostic build for an A/B: entry points it predates stay unset)
        if fn is None:
            raise NativeUnavailable(f"{p} does not export {name}: rebuild the HIP extension")
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


STATUS = {0: "ok", 1: "invalid argument", 2: "capacity exceeded", 3: "track slots exhausted",
          4: "HIP error", 5: "no HIP device", 6: "shape mismatch"}


def check(rc: int, what: str = ""):
    if rc == 0:
        return
    msg = load().bx_last_error().decode(errors="replace")
    text = f"{what}: {STATUS.get(rc, rc)} ({msg})"
    if rc == 5:
        raise NativeUnavailable(text)
    if rc in (1, 2, 6):
        raise ValueError(text)
    raise RuntimeError(text)


def device_count() -> int:
    n = C.c_int(0)
    load().bx_device_count(C.byref(n))
    return n.value
