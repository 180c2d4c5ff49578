"""Helpers to replay golden fixtures (tests only)."""
import ast

import numpy as np

from boxmot_amd.synth import SyntheticScene


def fixture_id(path) -> str:
    """Test id of a tracker fixture.  Fixtures whose captured LAP calls tie (``lap_degenerate`` >
    0: OCSort / BoostTrack full matchings, the duplicate-detection captures) were resolved by
    the restated lapx lapjv (make_golden.use_restated_lapx_jv), so their tie order is lapx's
    published algorithm as restated, not a lapx binary: the id says "parity-unpinned-ties<N>"
    with N the tie-sensitive call count, so a green run is not read as lapx parity."""
    from pathlib import Path

    stem = Path(path).stem[4:]
    with np.load(path) as fx:
        n = int(fx["lap_degenerate"]) if "lap_degenerate" in fx.files else 0
    return f"{stem}-parity-unpinned-ties{n}" if n else stem


def fixture_frames(fx):
    """Yield (frame_no, dets[N,6], embs|None) for a tracker fixture."""
    if "dets" in fx.files:
        D = fx["dets"]
        for f in np.unique(D[:, 0]).astype(int):
            yield int(f), D[D[:, 0] == f][:, 1:], None
    else:
        sc = SyntheticScene(**ast.literal_eval(str(fx["scene"])))
        for t in range(1, int(fx["n_frames"]) + 1):
            d, e, _ = sc.frame(t)
            yield t, d, e


def fixture_crash(fx):
    """(frame_no, dets, embs) of the frame where the reference raised TypeError (the StrongSort
    occlusion handler's mutual-occlusion crash, D7), or None."""
    if "crash_frame" not in fx.files or not int(fx["crash_frame"]):
        return None
    t = int(fx["crash_frame"])
    d, e, _ = SyntheticScene(**ast.literal_eval(str(fx["scene"]))).frame(t)
    return t, d, e


def fixture_warp(fx, f):
    """The 2x3 CMC warp a fixture's frame ``f`` was captured with (None = identity CMC)."""
    if "warps" not in fx.files:
        return None
    return np.asarray(fx["warps"][int(f) - 1], np.float64)


def fixture_tracker_args(fx):
    return str(fx["kind"]), ast.literal_eval(str(fx["tracker_args"]))


def compare_outputs(got, ref, box_atol=1e-6, conf_atol=None):
    """Integer columns (frame, id, cls, det_ind) bit-exact; boxes (and StrongSort's quality /
    occlusion columns) within box_atol; conf bit-exact unless conf_atol is given (BoostTrack's boosted confidences are functions of the Kalman
    state, so they inherit its tolerance)."""
    assert got.shape == ref.shape, (got.shape, ref.shape)
    np.testing.assert_array_equal(got[:, [0, 5, 7, 8]], ref[:, [0, 5, 7, 8]])
    if conf_atol is None:
        np.testing.assert_array_equal(got[:, 6], ref[:, 6])
    else:
        np.testing.assert_allclose(got[:, 6], ref[:, 6], rtol=0, atol=conf_atol)
    np.testing.assert_allclose(got[:, 1:5], ref[:, 1:5], rtol=0, atol=box_atol)
    if ref.shape[1] > 9:  # StrongSort rows: track quality and occlusion level (functions of the
        # Kalman state and the detections, so they inherit the box tolerance)
        np.testing.assert_allclose(got[:, 9:], ref[:, 9:], rtol=0, atol=box_atol)
