"""MOT evaluation I/O and the many-sequence runner.

Reference path replaced (muntherr/boxmot @ /root/reference):
  * detections / embeddings: ``engine/val.py:157-187`` appends ``np.savetxt(fmt='%f')`` text (a
    ``#`` header line, rows ``frame x1 y1 x2 y2 conf cls`` and ``F`` floats per row);
    ``utils/dataloaders/MOT17.py:147-200`` reloads them with ``np.loadtxt`` and selects each
    frame's rows by mask.  Here the text is parsed once by ``bx_txt_read`` (strtod: the same
    correctly rounded doubles as numpy) and packed into one binary file per sequence — header,
    frame table, float64 detection rows grouped by frame, float64 embeddings — that later runs
    memory-map.
  * results: ``engine/utils.py:101-173`` ``convert_to_mot_format`` + ``write_mot_results``
    (``bx_mot_format`` / ``bx_mot_write``, byte-identical lines).
  * the process pool of ``engine/val.py:357-405`` (one tracker per sequence per process):
    ``run_sequences`` drives ALL sequences through one batched engine handle, frame index by
    frame index; a sequence without detections at a frame is not updated (``val.py:347``).

Everything here is host code in libbxassoc.so; the trackers run on the MI355X engine.
"""
from __future__ import annotations

import ctypes as C
import struct
from pathlib import Path

import numpy as np

from . import _native as N

MAGIC = b"BXMOTSEQ"
_HDR = struct.Struct("<8sIIqII")  # magic, version, header bytes, rows, emb_dim, frames


def load_txt(path) -> np.ndarray:
    """``np.loadtxt(path, comments='#')`` as a 2-D float64 array (bit-identical values)."""
    L = N.load()
    rows, cols = C.c_int64(), C.c_int32()
    N.check(L.bx_txt_shape(str(path).encode(), C.byref(rows), C.byref(cols)), "bx_txt_shape")
    out = np.empty((rows.value, cols.value), np.float64)
    N.check(L.bx_txt_read(str(path).encode(), out.ctypes.data if out.size else None, rows.value,
                          cols.value), "bx_txt_read")
    return out


def pack_sequence(det_txt, emb_txt, out_path) -> Path:
    """Pack one sequence's det / emb text files (val.py's format) into the binary layout."""
    dets = load_txt(det_txt)
    embs = load_txt(emb_txt) if emb_txt is not None else np.empty((dets.shape[0], 0))
    if dets.shape[0] != embs.shape[0]:
        raise ValueError(f"Row mismatch in {det_txt}")  # MOT17.py:152-153
    if dets.shape[0] and dets.shape[1] != 7:
        raise ValueError("detection rows must be frame, x1, y1, x2, y2, conf, cls")
    fid = dets[:, 0].astype(int) if dets.shape[0] else np.empty(0, int)
    order = np.argsort(fid, kind="stable")  # per frame, the rows in file order (the mask's order)
    frames, first = np.unique(fid[order], return_index=True)
    offs = np.append(first, len(order)).astype(np.int64)
    out_path = Path(out_path)
    hdr_bytes = _HDR.size + 8 * len(frames) + 8 * len(offs)
    with open(out_path, "wb") as f:
        f.write(_HDR.pack(MAGIC, 1, hdr_bytes, dets.shape[0], embs.shape[1], len(frames)))
        f.write(frames.astype(np.int64).tobytes())
        f.write(offs.tobytes())
        f.write(np.ascontiguousarray(dets[order][:, 1:7], np.float64).tobytes())
        f.write(np.ascontiguousarray(embs[order], np.float64).tobytes())
    return out_path


class BinSequence:
    """A packed sequence, memory-mapped: ``frame(fid) -> (dets [n,6], embs [n,F])`` exactly as
    MOT17Sequence yields them (``dets[mask, 1:]``, ``embs[mask]``)."""

    def __init__(self, path):
        self.path = Path(path)
        with open(self.path, "rb") as f:
            magic, ver, hdr, rows, F, nf = _HDR.unpack(f.read(_HDR.size))
        if magic != MAGIC or ver != 1:
            raise ValueError(f"{path}: not a packed MOT sequence")
        self.rows, self.emb_dim, self.n_frames = rows, F, nf
        self.frame_ids = np.fromfile(self.path, np.int64, nf, offset=_HDR.size)
        self.offsets = np.fromfile(self.path, np.int64, nf + 1, offset=_HDR.size + 8 * nf)
        self._index = {int(k): i for i, k in enumerate(self.frame_ids)}
        self.dets = np.memmap(self.path, np.float64, "r", offset=hdr, shape=(rows, 6)) \
            if rows else np.empty((0, 6))
        self.embs = np.memmap(self.path, np.float64, "r", offset=hdr + 48 * rows,
                              shape=(rows, F)) if rows and F else np.empty((rows, F))

    def frame(self, fid: int):
        i = self._index.get(int(fid))
        if i is None:
            return np.empty((0, 6)), np.empty((0, self.emb_dim))
        a, b = self.offsets[i], self.offsets[i + 1]
        return np.asarray(self.dets[a:b]), np.asarray(self.embs[a:b])


def convert_to_mot_format(tracks: np.ndarray, frame_idx: int) -> np.ndarray:
    """engine/utils.py:101-133 (numpy branch): [n, >=7] tracker rows -> [n, 9] float64."""
    t = np.ascontiguousarray(np.asarray(tracks, np.float64))
    if t.size == 0:
        return np.empty((0, 9))
    t = t.reshape(t.shape[0], -1)
    out = np.empty((t.shape[0], 9), np.float64)
    N.check(N.load().bx_mot_format(t.ctypes.data, t.shape[0], t.shape[1], int(frame_idx),
                                   out.ctypes.data), "bx_mot_format")
    return out


def write_mot_results(txt_path, mot_results: np.ndarray | None) -> None:
    """engine/utils.py:152-173: create the file (and its directory), append the rows."""
    if mot_results is None:
        return
    p = Path(txt_path)
    p.parent.mkdir(parents=True, exist_ok=True)
    p.touch(exist_ok=True)
    m = np.ascontiguousarray(np.asarray(mot_results, np.float64))
    if m.size:
        N.check(N.load().bx_mot_write(str(p).encode(), m.ctypes.data, m.shape[0], 1),
                "bx_mot_write")


# ------------------------------------------------------------------------------ the runner
def _batched_engine(tracker_type: str, n_seq: int, emb_dim: int, tracker_kwargs: dict):
    """One engine handle for n_seq sequences, parameterised exactly as the drop-in tracker
    `tracker_type` is by `tracker_kwargs` (create_tracker's YAML defaults when empty)."""
    from .engine import BoostEngine, Engine, OcsortEngine, SsEngine
    from .tracker_zoo import create_tracker

    tr = create_tracker(tracker_type, evolve_param_dict=tracker_kwargs or None) \
        if tracker_kwargs else create_tracker(tracker_type)
    if tracker_type == "bytetrack":
        e = tr.engine
        return Engine("bytetrack", n_seq=n_seq, track_cap=e.track_cap, det_cap=e.det_cap,
                      params=e.params), np.float32, 8
    if tracker_type == "botsort":
        tc, dc = tr._caps
        return Engine("botsort", n_seq=n_seq, track_cap=tc, det_cap=dc, emb_dim=emb_dim,
                      emb_f64=True, params=tr._params), np.float32, 8
    if tracker_type == "ocsort":
        e = tr.engine
        return OcsortEngine(n_seq=n_seq, track_cap=e.track_cap, det_cap=e.det_cap,
                            params=e.params), np.float32, 8
    if tracker_type == "boosttrack":
        tc, dc = tr._caps
        return BoostEngine(n_seq=n_seq, track_cap=tc, det_cap=dc,
                           emb_dim=emb_dim if tr._params.with_reid else 0,
                           params=tr._params), np.float32, 8
    if tracker_type == "strongsort":
        tc, dc, vc = tr._caps
        eng = SsEngine(n_seq=n_seq, track_cap=tc, det_cap=dc, emb_dim=emb_dim, vec_cap=vc,
                       params=tr._params)
        # handle_occlusions: the host post-process runs per sequence after each batched step
        eng.occlusion_threshold = tr.occlusion_threshold if tr.handle_occlusions else None
        return eng, np.float64, 10
    raise NotImplementedError(f"{tracker_type} is not on the engine")


def run_sequences(tracker_type: str, sequences: dict, exp_dir, frame_ids: dict | None = None,
                  frame_sizes: dict | None = None, tracker_kwargs: dict | None = None) -> dict:
    """process_sequence (val.py:304-354) for every sequence at once.

    sequences: name -> packed file (pack_sequence) or BinSequence; frame_ids: name -> the frames
    to iterate (the image list; default: the frames that have detections); frame_sizes: name ->
    (w, h) of its images (OCSort's centroid mode).  Writes ``exp_dir/<name>.txt`` and returns
    name -> the frame ids iterated.  Sequence k's track ids start at 1, as in a fresh process.
    """
    import torch

    names = list(sequences)
    seqs = [s if isinstance(s, BinSequence) else BinSequence(s) for s in sequences.values()]
    S = len(seqs)
    F = max([s.emb_dim for s in seqs] + [0])
    eng, ddt, ncol = _batched_engine(tracker_type, S, F, tracker_kwargs or {})
    if tracker_type == "ocsort" and frame_sizes:
        for k, nm in enumerate(names):
            if nm in frame_sizes:
                eng.set_frame_size(k, *frame_sizes[nm])
    fids = [np.asarray(frame_ids[nm]) if frame_ids and nm in frame_ids else s.frame_ids
            for nm, s in zip(names, seqs)]
    results = [[] for _ in range(S)]
    occ = None
    if getattr(eng, "occlusion_threshold", None) is not None:
        from .occlusion import OcclusionHandler

        occ = [OcclusionHandler(eng, k, eng.occlusion_threshold) for k in range(S)]
    nupd = [0] * S
    dev = torch.device("cuda")
    for t in range(max([len(f) for f in fids] + [0])):
        frame = []
        for k in range(S):
            if t < len(fids[k]):
                d, e = seqs[k].frame(fids[k][t])
                frame.append((d, e) if d.size and (e.size or not F) else None)
            else:
                frame.append(None)
        k = 0
        while k < S:  # contiguous runs of sequences with an update at this frame index
            if frame[k] is None:
                k += 1
                continue
            k1 = k
            while k1 < S and frame[k1] is not None:
                k1 += 1
            ds = [frame[q][0] for q in range(k, k1)]
            off = np.zeros(k1 - k + 1, np.int32)
            off[1:] = np.cumsum([d.shape[0] for d in ds])
            dd = torch.from_numpy(np.concatenate(ds).astype(ddt)).to(dev)
            od = torch.from_numpy(off).to(dev)
            out = torch.empty((int(off[-1]), ncol), dtype=torch.float64, device=dev)
            cnt = torch.empty(k1 - k, dtype=torch.int32, device=dev)
            if tracker_type == "ocsort":
                eng.step(dd, od, out, cnt, seq0=k, nseq=k1 - k)
            else:
                emb = None
                if F and getattr(eng, "with_reid", True) and not (
                        tracker_type == "boosttrack" and not eng.emb_dim):
                    emb = torch.from_numpy(np.concatenate([frame[q][1] for q in range(k, k1)])
                                           .astype(np.float64)).to(dev)
                eng.step(dd, od, emb, None, out, cnt, seq0=k, nseq=k1 - k)
            o, c = out.cpu().numpy(), cnt.cpu().numpy()
            for q in range(k, k1):
                rows = o[off[q - k]: off[q - k] + c[q - k]]
                nupd[q] += 1
                if occ is not None:
                    rows = occ[q](nupd[q], rows)
                if rows.shape[0]:
                    results[q].append(convert_to_mot_format(rows, int(fids[q][t])))
            k = k1
    if eng.status() != 0:
        raise RuntimeError(f"engine status {eng.status()} (capacity overflow)")
    exp_dir = Path(exp_dir)
    for nm, res in zip(names, results):
        write_mot_results(exp_dir / f"{nm}.txt", np.vstack(res) if res else np.empty((0, 0)))
    return {nm: list(map(int, f)) for nm, f in zip(names, fids)}
