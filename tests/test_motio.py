"""MOT evaluation I/O (boxmot_amd.motio, include/bxio.h) against numpy's own behaviour on the
reference's formats: val.py's np.savetxt('%f') det/emb files read back by MOT17.py's np.loadtxt,
and engine/utils.py's convert_to_mot_format + write_mot_results.  ``xyxy2ltwh`` there is
ultralytics' (not in the reference tree): restated as [x1, y1, x2 - x1, y2 - y1]."""
import numpy as np
import pytest

from boxmot_amd import motio


def _write_val_files(tmp_path, frames, n_per, F, seed=0):
    """engine/val.py:157-187: a '#' header, then per frame np.savetxt(fmt='%f') appends."""
    rng = np.random.default_rng(seed)
    det_p, emb_p = tmp_path / "dets.txt", tmp_path / "embs.txt"
    with open(det_p, "ab+") as f:
        np.savetxt(f, [], fmt="%f", header="/data/MOT17/train/MOT17-02-FRCNN/img1")
    open(emb_p, "w").close()
    for fr in frames:
        n = n_per(fr)
        xy = rng.uniform(-5, 1900, (n, 2))
        wh = rng.uniform(1, 300, (n, 2))
        dets = np.concatenate([np.full((n, 1), fr), xy, xy + wh, rng.uniform(0, 1, (n, 1)),
                               rng.integers(0, 3, (n, 1))], 1)
        embs = rng.standard_normal((n, F)) * 10 ** rng.uniform(-3, 3, (n, 1))
        with open(det_p, "ab+") as f:
            np.savetxt(f, dets, fmt="%f")
        with open(emb_p, "ab+") as f:
            np.savetxt(f, embs, fmt="%f")
    return det_p, emb_p


def test_load_txt_bit_identical_to_loadtxt(tmp_path):
    det_p, emb_p = _write_val_files(tmp_path, range(1, 30), lambda f: 1 + f % 7, 64)
    for p in (det_p, emb_p):
        np.testing.assert_array_equal(motio.load_txt(p), np.loadtxt(p, comments="#"))


def test_load_txt_rejects_ragged_rows(tmp_path):
    from boxmot_amd import _native as N

    p = tmp_path / "bad.txt"
    p.write_text("1 2 3\n4 5\n")
    with pytest.raises(ValueError):
        motio.load_txt(p)
    assert N is not None


def test_packed_sequence_matches_mot17_masks(tmp_path):
    """MOT17Sequence (MOT17.py:181-200): dets[mask, 1:], embs[mask] per image frame; frames
    without rows (and frames written out of order) included."""
    frames = [1, 2, 3, 5, 8, 9, 4, 12]  # 4 appended after 9: the mask selection reorders
    det_p, emb_p = _write_val_files(tmp_path, frames, lambda f: (f * 3) % 5, 32, seed=3)
    b = motio.BinSequence(motio.pack_sequence(det_p, emb_p, tmp_path / "seq.bxmot"))
    dets = np.loadtxt(det_p, comments="#")
    embs = np.loadtxt(emb_p, comments="#")
    for fid in range(0, 15):
        mask = dets[:, 0].astype(int) == fid
        d, e = b.frame(fid)
        np.testing.assert_array_equal(d, dets[mask, 1:])
        np.testing.assert_array_equal(e, embs[mask])
    assert b.emb_dim == 32 and b.rows == dets.shape[0]


def _reference_mot_rows(tracks, fid):
    """engine/utils.py:120-133 with numpy."""
    tlwh = tracks[:, 0:4].copy()
    tlwh[:, 2] = tracks[:, 2] - tracks[:, 0]
    tlwh[:, 3] = tracks[:, 3] - tracks[:, 1]
    return np.column_stack((np.full((tracks.shape[0], 1), fid, dtype=np.int32),
                            tracks[:, 4].astype(np.int32), tlwh.round().astype(np.int32),
                            np.ones((tracks.shape[0], 1), dtype=np.int32),
                            tracks[:, 6].astype(np.int32), tracks[:, 5]))


def test_mot_format_and_writer_match_numpy(tmp_path):
    rng = np.random.default_rng(5)
    n = 200
    x1 = rng.uniform(-50, 1900, n)
    x1[:40] = np.floor(x1[:40]) + 0.5  # exact halves: round half to even
    y1 = rng.uniform(-50, 1000, n)
    w = rng.uniform(0.5, 300, n)
    w[40:60] = np.floor(w[40:60]) + 0.5
    tracks = np.column_stack([x1, y1, x1 + w, y1 + rng.uniform(1, 400, n),
                              rng.integers(1, 500, n), rng.uniform(0, 1, n),
                              rng.integers(0, 5, n), rng.integers(0, 99, n)]).astype(np.float64)
    got = motio.convert_to_mot_format(tracks, 17)
    ref = _reference_mot_rows(tracks, 17)
    np.testing.assert_array_equal(got, ref)
    a, b = tmp_path / "a" / "seq.txt", tmp_path / "b.txt"
    motio.write_mot_results(a, got)
    motio.write_mot_results(a, got[:5])  # append mode
    with open(b, "a") as f:  # engine/utils.py:170-173
        np.savetxt(f, ref, fmt="%d,%d,%d,%d,%d,%d,%d,%d,%.6f")
        np.savetxt(f, ref[:5], fmt="%d,%d,%d,%d,%d,%d,%d,%d,%.6f")
    assert a.read_bytes() == b.read_bytes()
    motio.write_mot_results(tmp_path / "empty.txt", np.empty((0, 0)))
    assert (tmp_path / "empty.txt").read_bytes() == b""
