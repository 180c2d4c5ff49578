"""Seeded synthetic detection/embedding streams for the association benchmarks.

This is the build's own scene generator (SURVEY.md §8(d) "Synthetic inputs"): ``n_obj``
constant-velocity boxes over a 1920x1080 frame, each detected with probability ``p_det`` per
frame, jittered box corners, confidences U(conf_lo, conf_hi), class 0 (or a fixed class per
identity from ``classes``), and per-identity unit embeddings perturbed by 0.1*N(0,1)/sqrt(F)
and renormalised.

Every frame is generated from its own ``numpy.random.default_rng([seed, frame])`` stream, so a
frame can be produced independently of the frames before it (bench shards, GPU-side staging and
the golden-fixture script all regenerate identical inputs from ``(seed, frame)``).

Three layouts:
* ``grid``   — objects on a regular grid, little overlap (the survey's C2/C3/C4 scene);
* ``crowded``— uniformly random centres with heavy overlap: many non-trivial LAP components and
  near-threshold costs (the stress variant §8(d) asks for);
* ``corner`` — ``crowded`` plus the ``corner`` objects held at the top-left corner (StrongSort's
  occlusion-handler fixtures).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

__all__ = ["SyntheticScene", "SyntheticCMC", "StatefulCMC", "TorchSceneBatch", "MotSequence",
           "c5_sequences", "load_mot_dets", "synth_warp"]


@dataclass
class SyntheticScene:
    n_obj: int
    seed: int = 0
    emb_dim: int = 0
    layout: str = "grid"
    p_det: float = 0.5
    conf_lo: float = 0.65
    conf_hi: float = 1.0
    jitter: float = 0.5
    width: float = 1920.0
    height: float = 1080.0
    emb_dtype: type = np.float32
    classes: tuple = ()  # per-identity class ids (identity k -> classes[k % len]); () = class 0
    corner: tuple = ()  # layout "corner": (width, a) of the objects parked at the top-left corner
    # every k-th detection is emitted twice (identical row and embedding, the copy right after
    # it) — a detector without NMS; the duplicates tie the linear assignment (0 = off)
    dup_every: int = 0

    def __post_init__(self):
        rng = np.random.default_rng([self.seed, 0x5CE7E])
        n = self.n_obj
        if self.layout == "grid":
            cols = max(1, math.ceil(math.sqrt(n * self.width / self.height)))
            rows = max(1, math.ceil(n / cols))
            cw, ch = self.width / cols, self.height / rows
            idx = np.arange(n)
            cx = (idx % cols + 0.5) * cw
            cy = (idx // cols + 0.5) * ch
            w = 0.45 * cw * rng.uniform(0.8, 1.2, n)
            h = 0.80 * ch * rng.uniform(0.8, 1.2, n)
        elif self.layout in ("crowded", "corner"):
            cx = rng.uniform(0.1, 0.9, n) * self.width
            cy = rng.uniform(0.1, 0.9, n) * self.height
            w = rng.uniform(30.0, 90.0, n)
            h = w * rng.uniform(1.5, 3.0, n)
            # corner: objects 0..k-1 nearly still at the top-left corner, where a tlwh row has
            # x < w and y < h — the only place OcclusionAwareTracker's xyxy reading of tlwh
            # boxes (occlusion_handler.py:49-56, 297-299) sees overlaps
            # (centre at a * size: the box's tlwh row reads as the xyxy rect [(a-.5)w, w] x ...)
            for i, (cw, a) in enumerate(self.corner if self.layout == "corner" else ()):
                w[i], h[i] = cw, 2.5 * cw
                cx[i], cy[i] = a * w[i], a * h[i]
        else:
            raise ValueError(f"unknown layout {self.layout!r}")
        self.c0 = np.stack([cx, cy], 1)
        self.size = np.stack([w, h], 1)
        self.vel = rng.uniform(-0.5, 0.5, (n, 2))
        if self.layout == "corner":
            self.vel[: len(self.corner)] *= 0.05
        if self.emb_dim:
            base = rng.standard_normal((n, self.emb_dim))
            self.base_emb = base / np.linalg.norm(base, axis=1, keepdims=True)
        else:
            self.base_emb = None

    def frame(self, t: int):
        """Detections of frame ``t`` (1-based like the reference's frame counter).

        Returns ``(dets[N,6] float64 (x1,y1,x2,y2,conf,cls), embs[N,F] or None, ids[N])``.
        """
        rng = np.random.default_rng([self.seed, int(t)])
        n = self.n_obj
        seen = rng.random(n) < self.p_det
        ids = np.flatnonzero(seen)
        rng.shuffle(ids)
        m = ids.size
        c = self.c0[ids] + self.vel[ids] * float(t)
        half = self.size[ids] * 0.5
        box = np.concatenate([c - half, c + half], 1) + rng.normal(0.0, self.jitter, (m, 4))
        conf = rng.uniform(self.conf_lo, self.conf_hi, m)
        dets = np.zeros((m, 6), np.float64)
        dets[:, :4] = box
        dets[:, 4] = conf
        if self.classes:  # per-class mode fixtures: the class is a fixed property of the identity
            dets[:, 5] = np.asarray(self.classes, np.float64)[ids % len(self.classes)]
        embs = None
        if self.base_emb is not None:
            e = self.base_emb[ids] + 0.1 * rng.standard_normal((m, self.emb_dim)) / math.sqrt(
                self.emb_dim
            )
            e /= np.linalg.norm(e, axis=1, keepdims=True)
            embs = e.astype(self.emb_dtype)
        if self.dup_every > 0 and m:
            rep = np.ones(m, np.int64)
            rep[:: self.dup_every] = 2
            order = np.repeat(np.arange(m), rep)
            dets, ids = dets[order], ids[order]
            embs = embs[order] if embs is not None else None
        return dets, embs, ids


def synth_warp(seed: int, t: int, rot: float = 0.003, scale: float = 0.002,
               shift: float = 2.0) -> np.ndarray:
    """Seeded 2x3 camera warp of frame ``t`` — a small similarity (rotation about the image
    origin, isotropic scale, shift in px) standing in for an ECC estimate (``motion/cmc/ecc.py``
    returns the same 2x3 affine form).  Drawn from ``default_rng([seed, t, 0xC3C])``."""
    rng = np.random.default_rng([int(seed), int(t), 0xC3C])
    a = rng.uniform(-rot, rot)
    s = 1.0 + rng.uniform(-scale, scale)
    tx, ty = rng.uniform(-shift, shift, 2)
    return np.array([[s * math.cos(a), -s * math.sin(a), tx],
                     [s * math.sin(a), s * math.cos(a), ty]], np.float64)


class SyntheticCMC:
    """A CMC object for the trackers' ``cmc`` slot (``apply(img, dets) -> 2x3``) that returns a
    per-frame warp from a table keyed by frame number: the caller sets ``t`` before each
    ``update``, so the warp a frame sees does not depend on which frames call ``apply``
    (StrongSort skips it when there are no tracks, ``strongsort.py:168-172``)."""

    def __init__(self, warps):
        self.warps = warps  # {frame: (2,3)} or a callable t -> (2,3)
        self.t = 0

    def apply(self, img, dets=None):
        w = self.warps(self.t) if callable(self.warps) else self.warps[self.t]
        return np.array(w, np.float64).reshape(2, 3)


class StatefulCMC(SyntheticCMC):
    """ECC-like state (``motion/cmc/ecc.py`` keeps the previous frame): the first ``apply`` of a
    frame returns that frame's warp, every later call on the same frame compares the image with
    itself and returns the identity.  Under ``per_class=True`` the reference calls ``apply`` once
    per class call (basetracker.py:175-189 -> botsort.py:218 / boosttrack.py:244), so only class
    0 sees the real inter-frame warp."""

    def __init__(self, warps):
        super().__init__(warps)
        self._last = None

    def apply(self, img, dets=None):
        if self._last == self.t:
            return np.eye(2, 3)
        self._last = self.t
        return super().apply(img, dets)


class TorchSceneBatch:
    """The scene process for ``n_seq`` independent sequences, generated on the GPU.

    Same geometry (``grid`` or ``crowded``), motion, detection probability, jitter, confidence and
    embedding model as ``SyntheticScene``, but drawn with torch's device RNG so that thousands of
    sequences × frames can be staged in HBM before a timed region (numbers differ from the numpy
    generator; the distribution does not).  ``frame(t)`` returns packed
    ``(dets[sum N,6] f32, det_off[n_seq+1] i32, embs[sum N,F] f32 | None)`` on ``device``.
    """

    def __init__(self, n_seq, n_obj, emb_dim=0, seed=0, device="cuda", p_det=0.5,
                 conf_lo=0.65, conf_hi=1.0, jitter=0.5, width=1920.0, height=1080.0,
                 layout="grid"):
        import torch

        self.torch, self.n_seq, self.n_obj, self.emb_dim = torch, n_seq, n_obj, emb_dim
        self.device, self.p_det, self.conf = device, p_det, (conf_lo, conf_hi)
        self.jitter = jitter
        g = torch.Generator(device=device)
        g.manual_seed(int(seed) * 7919 + 17)
        self.g = g
        cols = max(1, math.ceil(math.sqrt(n_obj * width / height)))
        rows = max(1, math.ceil(n_obj / cols))
        cw, ch = width / cols, height / rows
        idx = torch.arange(n_obj, device=device, dtype=torch.float64)
        cx = ((idx % cols) + 0.5) * cw
        cy = torch.div(idx, cols, rounding_mode="floor").add(0.5) * ch
        u = lambda *s: torch.rand(*s, generator=g, device=device, dtype=torch.float64)  # noqa
        if layout == "grid":
            w = 0.45 * cw * (0.8 + 0.4 * u(n_seq, n_obj))
            h = 0.80 * ch * (0.8 + 0.4 * u(n_seq, n_obj))
            self.c0 = torch.stack([cx.expand(n_seq, n_obj), cy.expand(n_seq, n_obj)], -1)
        elif layout == "crowded":  # SyntheticScene's crowded process: random centres, overlap
            self.c0 = torch.stack([(0.1 + 0.8 * u(n_seq, n_obj)) * width,
                                   (0.1 + 0.8 * u(n_seq, n_obj)) * height], -1)
            w = 30.0 + 60.0 * u(n_seq, n_obj)
            h = w * (1.5 + 1.5 * u(n_seq, n_obj))
        else:
            raise ValueError(f"unknown layout {layout!r}")
        self.half = torch.stack([w, h], -1) * 0.5
        self.vel = u(n_seq, n_obj, 2) - 0.5
        if emb_dim:
            b = torch.randn(n_seq, n_obj, emb_dim, generator=g, device=device)
            self.base = b / b.norm(dim=-1, keepdim=True)

    def frame(self, t):
        torch = self.torch
        g, dev, S, n = self.g, self.device, self.n_seq, self.n_obj
        seen = torch.rand(S, n, generator=g, device=dev) < self.p_det
        # random order of the detected objects inside each sequence
        key = torch.rand(S, n, generator=g, device=dev) + (~seen).float() * 2.0
        order = key.argsort(dim=1)
        counts = seen.sum(1)
        sel = torch.arange(n, device=dev).expand(S, n) < counts[:, None]
        sidx = torch.arange(S, device=dev)[:, None].expand(S, n)[sel]
        oidx = order[sel]
        c = self.c0[sidx, oidx] + self.vel[sidx, oidx] * float(t)
        hf = self.half[sidx, oidx]
        m = sidx.numel()
        box = torch.cat([c - hf, c + hf], 1) + self.jitter * torch.randn(
            m, 4, generator=g, device=dev, dtype=torch.float64)
        lo, hi = self.conf
        conf = lo + (hi - lo) * torch.rand(m, generator=g, device=dev, dtype=torch.float64)
        dets = torch.zeros(m, 6, device=dev, dtype=torch.float32)
        dets[:, :4] = box.float()
        dets[:, 4] = conf.float()
        off = torch.zeros(S + 1, dtype=torch.int32, device=dev)
        off[1:] = counts.cumsum(0).to(torch.int32)
        embs = None
        if self.emb_dim:
            e = self.base[sidx, oidx] + 0.1 * torch.randn(
                m, self.emb_dim, generator=g, device=dev) / math.sqrt(self.emb_dim)
            embs = (e / e.norm(dim=-1, keepdim=True)).contiguous()
        return dets, off, embs


def _iou_matrix(a, b):
    lt = np.maximum(a[:, None, :2], b[None, :, :2])
    rb = np.minimum(a[:, None, 2:4], b[None, :, 2:4])
    wh = np.clip(rb - lt, 0, None)
    inter = wh[..., 0] * wh[..., 1]
    area = lambda x: (x[:, 2] - x[:, 0]) * (x[:, 3] - x[:, 1])  # noqa: E731
    return inter / (area(a)[:, None] + area(b)[None, :] - inter)


class MotSequence:
    """A real detection stream (MOT17 public detections, packed [frame, x1, y1, x2, y2, conf])
    with synthetic ReID embeddings that follow object identity: consecutive frames' detections
    are linked greedily by IoU (>= 0.5, best pair first), a linked detection inherits its
    predecessor's identity, and each identity owns a random unit base vector; a detection's
    embedding is its identity's vector plus 10% noise, normalised.  Frames are renumbered
    1..n_frames (val.py feeds every frame that has detections).  ``frame(t)`` has
    SyntheticScene's contract."""

    def __init__(self, packed, emb_dim=0, seed=0, emb_dtype=np.float64):
        packed = np.asarray(packed, np.float64)
        fnos = np.unique(packed[:, 0]).astype(int)
        self.n_frames = len(fnos)
        self.dets, self.ids = [], []
        prev, prev_id, next_id = None, None, 0
        for f in fnos:
            r = packed[packed[:, 0] == f]
            d = np.zeros((r.shape[0], 6), np.float64)
            d[:, :5] = r[:, 1:6]
            ids = np.full(d.shape[0], -1, np.int64)
            if prev is not None and prev.shape[0] and d.shape[0]:
                iou = _iou_matrix(d, prev)
                order = np.argsort(-iou, axis=None, kind="stable")
                used_a, used_b = set(), set()
                for k in order:
                    i, j = divmod(int(k), prev.shape[0])
                    if iou[i, j] < 0.5:
                        break
                    if i in used_a or j in used_b:
                        continue
                    used_a.add(i)
                    used_b.add(j)
                    ids[i] = prev_id[j]
            for i in np.flatnonzero(ids < 0):
                ids[i] = next_id
                next_id += 1
            self.dets.append(d)
            self.ids.append(ids)
            prev, prev_id = d, ids
        self.emb_dim, self.seed, self.emb_dtype = emb_dim, seed, emb_dtype
        if emb_dim:
            rng = np.random.default_rng([seed, 0x307])
            base = rng.standard_normal((next_id, emb_dim))
            self.base_emb = base / np.linalg.norm(base, axis=1, keepdims=True)

    def frame(self, t: int):
        d, ids = self.dets[t - 1], self.ids[t - 1]
        embs = None
        if self.emb_dim:
            rng = np.random.default_rng([self.seed, int(t)])
            e = self.base_emb[ids] + 0.1 * rng.standard_normal((ids.size, self.emb_dim)) / \
                math.sqrt(self.emb_dim)
            e /= np.linalg.norm(e, axis=1, keepdims=True)
            embs = e.astype(self.emb_dtype)
        return d.copy(), embs, ids


def c5_sequences(mot_npz, emb_dim=512, n_synth=6, seed=0):
    """SURVEY §8(d)'s C5 stand-in (MOT17-ablation is a network download): MOT17-02 and MOT17-04
    public detections + ``n_synth`` synthetic MOT-sized sequences (60 objects detected w.p. 0.5:
    ~30 dets/frame, confidences U(0.3, 1)), float64 ReID embeddings.  Returns [(name, seq,
    n_frames)]."""
    z = np.load(mot_npz)
    out = []
    for k, name in enumerate(["MOT17-02-FRCNN", "MOT17-04-FRCNN"]):
        sq = MotSequence(z[name], emb_dim=emb_dim, seed=seed + k)
        out.append((name, sq, sq.n_frames))
    for k in range(n_synth):
        sq = SyntheticScene(n_obj=60, seed=seed + 100 + k, emb_dim=emb_dim, conf_lo=0.3,
                            emb_dtype=np.float64, layout="crowded" if k % 2 else "grid")
        out.append((f"synthetic-{k}", sq, 600 + 90 * k))
    return out


def load_mot_dets(path):
    """MOT17 ``det.txt`` (``frame,-1,x,y,w,h,conf``) → {frame: dets[N,6] xyxy,conf,cls=0}.

    Mirrors how the survey fed MOT17-mini public detections to the trackers (§8(c)).
    """
    raw = np.loadtxt(path, delimiter=",", dtype=np.float64, ndmin=2)
    out = {}
    for f in np.unique(raw[:, 0]).astype(int):
        r = raw[raw[:, 0] == f]
        d = np.zeros((r.shape[0], 6), np.float64)
        d[:, 0] = r[:, 2]
        d[:, 1] = r[:, 3]
        d[:, 2] = r[:, 2] + r[:, 4]
        d[:, 3] = r[:, 3] + r[:, 5]
        d[:, 4] = r[:, 6]
        out[int(f)] = d
    return out
