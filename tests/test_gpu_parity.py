"""GPU parity: libbxassoc.so (HIP, gfx950) against the oracle and the reference's golden vectors.

Bar (BASELINE.json north_star): integer outputs (track ids, det_ind) and conf/cls bit-exact;
Kalman state within fp32 1e-5 relative — the engine is fp64 and mirrors the oracle's operation
order, so boxes are compared to the oracle bitwise and to the reference at 1e-9 absolute.
"""
import glob
from pathlib import Path

import numpy as np
import pytest

from oracle import pyoracle as po
from tests.golden_util import (compare_outputs, fixture_crash, fixture_frames, fixture_id,
                               fixture_tracker_args, fixture_warp)

pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).parent / "golden"
TRK_FIXTURES = sorted(glob.glob(str(GOLDEN / "trk_*.npz")))


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected without a HIP device")
    from boxmot_amd import _native

    _native.load()  # must be the in-tree HIP library, never a fallback
    return torch


@pytest.fixture(scope="module")
def K():
    return np.load(GOLDEN / "kernels.npz")


def dev(torch, a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def host(t):
    import torch

    torch.cuda.synchronize()
    return t.cpu().numpy()


# ------------------------------------------------------------------------------- op level
@pytest.mark.parametrize("mode", ["iou", "hmiou", "giou", "diou", "ciou", "centroid"])
def test_pairwise_cost_registry(torch_cuda, mode):
    """bx_pairwise_cost vs the reference's vectors (utils/iou.py:79-307) and, bit for bit, vs
    the oracle — on the golden boxes, on strided rows (lda 6 / ldb 9: dets carry conf/cls)
    and at C4 size 1024 x 512."""
    torch = torch_cuda
    from boxmot_amd.iou import AssociationFunction, pairwise_cost

    g = np.load(GOLDEN / "asso_funcs.npz")
    af = AssociationFunction(int(g["w"]), int(g["h"]), mode)
    for which in ("rand", "edge"):
        a, b = g[f"{which}_a"], g[f"{which}_b"]
        got = af.asso_func(a, b)
        np.testing.assert_array_equal(got, po.asso_batch(mode, a, b, int(g["w"]), int(g["h"])))
        ref = g[f"{mode}_{which}"]
        if mode == "ciou":  # np.arctan vs fdlibm atan: <= 1 ulp
            np.testing.assert_allclose(got, ref, rtol=0, atol=4e-16)
        else:
            np.testing.assert_array_equal(got, ref)
    rng = np.random.default_rng(11)
    c = rng.uniform(0, 1900, (1024, 2))
    sz = rng.uniform(8, 200, (1024, 2))
    A = np.concatenate([c - sz / 2, c + sz / 2, rng.uniform(0, 1, (1024, 2))], 1)
    B = np.concatenate([A[:512, :4] + rng.normal(0, 6, (512, 4)), np.zeros((512, 5))], 1)
    ad = torch.from_numpy(A).cuda()
    bd = torch.from_numpy(B).cuda()
    out = pairwise_cost(mode, ad, bd, 1920, 1080)
    assert out.is_cuda and out.shape == (1024, 512)
    np.testing.assert_array_equal(host(out), po.asso_batch(mode, A[:, :4], B[:, :4], 1920, 1080))
    empty = pairwise_cost(mode, np.zeros((0, 4)), B[:, :4], 1920, 1080)
    assert empty.shape == (0, 512)


def test_aw_max_metric_exact(torch_cuda):
    """bx_aw_max_metric vs the reference's vectors (utils/association.py:320-374), bitwise."""
    torch = torch_cuda
    from boxmot_amd import _native as N

    L = N.load()
    g = np.load(GOLDEN / "asso_funcs.npz")
    for k in range(int(g["aw_count"])):
        e = dev(torch, g[f"aw{k}_in"])
        out = torch.empty_like(e)
        N.check(L.bx_aw_max_metric(e.data_ptr(), e.shape[0], e.shape[1], float(g[f"aw{k}_w"]),
                                   0.5, out.data_ptr(), None))
        np.testing.assert_array_equal(host(out), g[f"aw{k}_out"])


def test_iou_fuse_embedding_exact(torch_cuda, K):
    torch = torch_cuda
    from boxmot_amd import _native as N

    L = N.load()
    a, b = dev(torch, K["iou_a"]), dev(torch, K["iou_b"])
    out = torch.empty((a.shape[0], b.shape[0]), dtype=torch.float64, device="cuda")
    N.check(L.bx_iou_batch(a.data_ptr(), a.shape[0], b.data_ptr(), b.shape[0], out.data_ptr(),
                           None))
    np.testing.assert_array_equal(host(out), K["iou_out"])

    c = dev(torch, K["fuse_cost_in"])
    conf = dev(torch, K["fuse_conf"])
    N.check(L.bx_fuse_score(c.data_ptr(), c.shape[0], c.shape[1], conf.data_ptr(), None))
    np.testing.assert_array_equal(host(c), K["fuse_out"])

    t, d = dev(torch, K["emb_trk"]), dev(torch, K["emb_det"])
    out = torch.empty((t.shape[0], d.shape[0]), dtype=torch.float64, device="cuda")
    N.check(L.bx_embedding_distance(t.data_ptr(), t.shape[0], d.data_ptr(), d.shape[0],
                                    t.shape[1], out.data_ptr(), None))
    np.testing.assert_array_equal(host(out), K["emb_out"])  # scipy cdist order: bit-exact


@pytest.mark.parametrize("kind", ["xyah", "xywh"])
def test_kalman_ops(torch_cuda, K, kind):
    torch = torch_cuda
    from boxmot_amd import _native as N

    L = N.load()
    k = 0 if kind == "xyah" else 1
    meas = dev(torch, K[f"kf_{kind}_meas"])
    n = meas.shape[0]
    mean = torch.empty((n, 8), dtype=torch.float64, device="cuda")
    cov = torch.empty((n, 8, 8), dtype=torch.float64, device="cuda")
    N.check(L.bx_kf_initiate(k, n, meas.data_ptr(), mean.data_ptr(), cov.data_ptr(), None))
    np.testing.assert_array_equal(host(mean), K[f"kf_{kind}_init_mean"])
    np.testing.assert_array_equal(host(cov), K[f"kf_{kind}_init_cov"])

    mean = dev(torch, K[f"kf_{kind}_pred_in_mean"])
    cov = dev(torch, K[f"kf_{kind}_init_cov"])
    N.check(L.bx_kf_multi_predict(k, n, mean.data_ptr(), cov.data_ptr(), None))
    np.testing.assert_array_equal(host(mean), K[f"kf_{kind}_pred_mean"])
    np.testing.assert_array_equal(host(cov), K[f"kf_{kind}_pred_cov"])

    mean = dev(torch, K[f"kf_{kind}_pred_mean"])
    cov = dev(torch, K[f"kf_{kind}_pred_cov"])
    z = dev(torch, K[f"kf_{kind}_upd_z"])
    conf = dev(torch, K[f"kf_{kind}_upd_conf"])
    N.check(L.bx_kf_update(k, n, mean.data_ptr(), cov.data_ptr(), z.data_ptr(), conf.data_ptr(),
                           None))
    gm, gc = host(mean), host(cov)
    for i in range(n):
        om, oc = po.kf_update(kind, K[f"kf_{kind}_pred_mean"][i], K[f"kf_{kind}_pred_cov"][i],
                              K[f"kf_{kind}_upd_z"][i], K[f"kf_{kind}_upd_conf"][i])
        np.testing.assert_array_equal(gm[i], om)  # same op order as the oracle: bitwise
        np.testing.assert_array_equal(gc[i], oc)
    np.testing.assert_allclose(gm, K[f"kf_{kind}_upd_mean"], rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(gc, K[f"kf_{kind}_upd_cov"], rtol=1e-10, atol=1e-9)

    zg = dev(torch, K[f"kf_{kind}_gate_z"])
    mean = dev(torch, K[f"kf_{kind}_pred_mean"])
    cov = dev(torch, K[f"kf_{kind}_pred_cov"])
    out = torch.empty((n, zg.shape[0]), dtype=torch.float64, device="cuda")
    N.check(L.bx_kf_gating_distance(k, n, mean.data_ptr(), cov.data_ptr(), zg.data_ptr(),
                                    zg.shape[0], out.data_ptr(), None))
    np.testing.assert_allclose(host(out), K[f"kf_{kind}_gate_out"], rtol=1e-10)


@pytest.mark.gpu
def test_kf_xysr_boost_ops(torch_cuda):
    """Op-level XYSR (OCSort) and BoostTrack filters: bitwise equal to the oracle on the
    reference-captured chains of kf_ops.npz (initiate, predict incl. the clamp, update, MhDist),
    and through it pinned to the reference (tests/test_oracle.py)."""
    torch = torch_cuda
    from boxmot_amd import _native as N

    L = N.load()
    fx = np.load(GOLDEN / "kf_ops.npz")
    ptr = lambda t: t.data_ptr()  # noqa: E731
    n = fx["xysr_init_box"].shape[0]
    x = torch.empty((n, 7), dtype=torch.float64, device="cuda")
    P = torch.empty((n, 7, 7), dtype=torch.float64, device="cuda")
    N.check(L.bx_kf_xysr_initiate(n, ptr(dev(torch, fx["xysr_init_box"])), ptr(x), ptr(P), None))
    np.testing.assert_array_equal(host(x), fx["xysr_init_x"])
    np.testing.assert_array_equal(host(P), fx["xysr_init_P"])
    for s in range(int(fx["xysr_steps"])):
        x, P = dev(torch, fx[f"xysr_s{s}_in_x"]), dev(torch, fx[f"xysr_s{s}_in_P"])
        N.check(L.bx_kf_xysr_predict(n, ptr(x), ptr(P), 0.01, 0.0001, None))
        np.testing.assert_array_equal(host(x), fx[f"xysr_s{s}_pred_x"])
        np.testing.assert_array_equal(host(P), fx[f"xysr_s{s}_pred_P"])
        z = fx[f"xysr_s{s}_z"]
        N.check(L.bx_kf_xysr_update(n, ptr(x), ptr(P), ptr(dev(torch, z)), None))
        ox, oP = po.kf_xysr("update", fx[f"xysr_s{s}_pred_x"], fx[f"xysr_s{s}_pred_P"], z)
        np.testing.assert_array_equal(host(x), ox)
        np.testing.assert_array_equal(host(P), oP)
    n = fx["boost_init_z"].shape[0]
    x = torch.empty((n, 8), dtype=torch.float64, device="cuda")
    P = torch.empty((n, 8, 8), dtype=torch.float64, device="cuda")
    N.check(L.bx_kf_boost_initiate(n, ptr(dev(torch, fx["boost_init_z"])), ptr(x), ptr(P), None))
    np.testing.assert_array_equal(host(x), fx["boost_init_x"])
    np.testing.assert_array_equal(host(P), fx["boost_init_P"])
    for s in range(int(fx["boost_steps"])):
        x, P = dev(torch, fx[f"boost_s{s}_in_x"]), dev(torch, fx[f"boost_s{s}_in_P"])
        N.check(L.bx_kf_boost_predict(n, ptr(x), ptr(P), None))
        np.testing.assert_array_equal(host(x), fx[f"boost_s{s}_pred_x"])
        np.testing.assert_array_equal(host(P), fx[f"boost_s{s}_pred_P"])
        d = fx[f"boost_s{s}_mh_dets"]
        mh = torch.empty((d.shape[0], n), dtype=torch.float64, device="cuda")
        N.check(L.bx_kf_boost_mh_dist(d.shape[0], ptr(dev(torch, d)), n, ptr(x), ptr(P), ptr(mh),
                                      None))
        np.testing.assert_array_equal(host(mh), fx[f"boost_s{s}_mh"])
        z = fx[f"boost_s{s}_z"]
        N.check(L.bx_kf_boost_update(n, ptr(x), ptr(P), ptr(dev(torch, z)), None))
        ox, oP = po.kf_boost("update", fx[f"boost_s{s}_pred_x"], fx[f"boost_s{s}_pred_P"], z)
        np.testing.assert_array_equal(host(x), ox)
        np.testing.assert_array_equal(host(P), oP)


def gpu_linear_assignment(torch, cost, thr, tied=None):
    """bx_linear_assignment_ex -> (matches, unmatched_a, unmatched_b) as matching.py:56-61 builds
    them (x == -1 unmatched; -3 = assigned above thresh: neither).  `tied` (a list) receives
    whether the lapx re-solve ran."""
    from boxmot_amd import _native as N

    nr, nc = cost.shape
    c = dev(torch, cost.astype(np.float64))
    x = torch.empty(max(nr, 1), dtype=torch.int32, device="cuda")
    y = torch.empty(max(nc, 1), dtype=torch.int32, device="cuda")
    t = torch.zeros(1, dtype=torch.int32, device="cuda")
    N.check(N.load().bx_linear_assignment_ex(c.data_ptr(), nr, nc, float(thr), x.data_ptr(),
                                             y.data_ptr(), t.data_ptr(), None))
    x, y = host(x)[:nr], host(y)[:nc]
    if tied is not None:
        tied.append(int(host(t)[0]))
    rows = np.flatnonzero(x >= 0)
    return np.stack([rows, x[rows]], 1) if rows.size else np.empty((0, 2), int), \
        np.flatnonzero(x == -1), np.flatnonzero(y == -1)


def test_linear_assignment_golden(torch_cuda, K):
    for i in range(int(K["lap_count"])):
        m, ua, ub = gpu_linear_assignment(torch_cuda, K[f"lap{i}_cost"], float(K[f"lap{i}_thr"]))
        np.testing.assert_array_equal(m, K[f"lap{i}_matches"].reshape(-1, 2))
        np.testing.assert_array_equal(ua, K[f"lap{i}_ua"])
        np.testing.assert_array_equal(ub, K[f"lap{i}_ub"])


@pytest.mark.parametrize("shape", [(1, 1), (3, 7), (7, 3), (20, 20), (64, 31), (31, 64),
                                   (128, 128), (300, 150)])
def test_linear_assignment_random_vs_oracle(torch_cuda, shape):
    """Continuous costs: unique optima, solved sparse — the tie check must not fire (it would
    only cost time, but it is the fast path's precondition)."""
    rng = np.random.default_rng(hash(shape) % 2**32)
    for thr, power in [(0.8, 1.0), (0.5, 3.0), (0.9, 0.5), (0.3, 1.0)]:
        c = rng.uniform(0, 1, shape) ** power
        om, oua, oub = po.linear_assignment(c, thr)
        tied = []
        gm, gua, gub = gpu_linear_assignment(torch_cuda, c, thr, tied)
        np.testing.assert_array_equal(gm, om)
        np.testing.assert_array_equal(gua, oua)
        np.testing.assert_array_equal(gub, oub)
        assert tied == [0]


def tie_heavy_costs(rng, shape, rep):
    """Tied LAP inputs as trackers meet them: costs on a 0.1 grid (equal costs everywhere, some
    exactly at the limit), duplicated rows (two tracks predicted onto one box) and duplicated
    columns (duplicate detections) over sparse or continuous costs."""
    nr, nc = shape
    thr = (0.8, 0.5, 0.7, 0.9)[rep % 4]
    kind = rep % 3
    if kind == 0:
        c = rng.integers(0, 11, shape) / 10.0
    else:
        c = rng.uniform(0, 1, shape) if kind == 1 else np.ones(shape)
        if kind == 2:
            m = rng.uniform(size=shape) < 0.05
            c[m] = rng.uniform(0, thr, m.sum())
        for _ in range(max(1, nc // 6)):  # duplicate detections
            j1, j2 = rng.integers(0, nc, 2)
            c[:, j2] = c[:, j1]
        for _ in range(max(1, nr // 8)):  # tracks on the same box
            i1, i2 = rng.integers(0, nr, 2)
            c[i2] = c[i1]
        at = rng.uniform(size=shape) < 0.01  # costs exactly at the limit
        c[at] = thr
    return np.ascontiguousarray(c, np.float64), thr


@pytest.mark.parametrize("shape", [(1, 2), (2, 1), (3, 3), (8, 5), (5, 8), (40, 40), (128, 64),
                                   (256, 128), (150, 300)])
def test_linear_assignment_ties_vs_oracle(torch_cuda, shape):
    """Tied optima (VERDICT r2 Missing 1): the sparse solver's pick among equal optima is its
    own, so bx_linear_assignment detects a non-unique optimum (dual test, lap_tied_block) and
    re-solves with lapx's lapjv on the (nr+nc)^2 extension — GPU == the oracle's lapx
    (matching.py:54-61) on every matrix, ties included."""
    rng = np.random.default_rng(sum(shape) * 7919 + shape[0])
    n_tied = 0
    for rep in range(8):
        c, thr = tie_heavy_costs(rng, shape, rep)
        om, oua, oub = po.linear_assignment(c, thr)
        tied = []
        gm, gua, gub = gpu_linear_assignment(torch_cuda, c, thr, tied)
        np.testing.assert_array_equal(gm, om, err_msg=f"{shape} rep {rep}")
        np.testing.assert_array_equal(gua, oua, err_msg=f"{shape} rep {rep}")
        np.testing.assert_array_equal(gub, oub, err_msg=f"{shape} rep {rep}")
        n_tied += tied[0]
    assert n_tied > 0
    # the VERDICT's example: one track, two identical detections -> lapx gives det 1
    gm, _, gub = gpu_linear_assignment(torch_cuda, np.array([[0.3, 0.3]]), 0.8)
    np.testing.assert_array_equal(gm, [[0, 1]])
    np.testing.assert_array_equal(gub, [0])


@pytest.mark.parametrize("shape,density", [((64, 64), 0.02), ((256, 128), 0.01),
                                           ((256, 128), 0.03), ((128, 256), 0.02),
                                           ((200, 200), 0.008)])
def test_linear_assignment_sparse_components_vs_oracle(torch_cuda, shape, density):
    """Sparse candidate graphs like the trackers' (many single-edge rows, stars — several
    rows on one column — and small multi-edge components) against the oracle's dense solver."""
    rng = np.random.default_rng(int(density * 1e4) + shape[0])
    for rep in range(6):
        thr = 0.8
        c = np.ones(shape)
        mask = rng.uniform(size=shape) < density
        # stars: a few columns shared by several single-edge rows
        for j in rng.choice(shape[1], size=max(1, shape[1] // 16), replace=False):
            rows = rng.choice(shape[0], size=rng.integers(2, 5), replace=False)
            mask[rows, :] = False
            mask[rows, j] = True
        c[mask] = rng.uniform(0, thr, mask.sum())
        om, oua, oub = po.linear_assignment(c, thr)
        gm, gua, gub = gpu_linear_assignment(torch_cuda, c, thr)
        np.testing.assert_array_equal(gm, om)
        np.testing.assert_array_equal(gua, oua)
        np.testing.assert_array_equal(gub, oub)


def crowd_dup_costs(rng, nt, nd, dup_every=3):
    """1 - IoU of nt track boxes against nd detections near some of them, every dup_every-th
    detection emitted twice (a detector without NMS): duplicate columns, and most rows all 1.0 —
    the tie path's row classes (jv_wave_t's scan skip)."""
    def boxes(k):
        xy = rng.uniform(0, 1000, (k, 2))
        return np.hstack([xy, xy + rng.uniform(30, 80, (k, 2))])

    T = boxes(nt)
    D = T[rng.choice(nt, nd, replace=nd > nt)] + rng.normal(0, 5, (nd, 4))
    D = np.vstack([np.repeat(D[i:i + 1], 2 if i % dup_every == 0 else 1, 0) for i in range(nd)])
    x1 = np.maximum(T[:, None, 0], D[None, :, 0])
    y1 = np.maximum(T[:, None, 1], D[None, :, 1])
    x2 = np.minimum(T[:, None, 2], D[None, :, 2])
    y2 = np.minimum(T[:, None, 3], D[None, :, 3])
    inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
    area = lambda z: (z[:, 2] - z[:, 0]) * (z[:, 3] - z[:, 1])  # noqa: E731
    return np.ascontiguousarray(1.0 - inter / (area(T)[:, None] + area(D)[None, :] - inter))


@pytest.mark.gpu
def test_linear_assignment_equivalent_rows_vs_oracle(torch_cuda):
    """The tie re-solve skips a scan of a row whose cost row equals an already-scanned row's
    (dummy rows; real rows constant at the first constant row's value) when it provably changes
    nothing (jv_wave_t).  Problems made of such rows: crowded IoU with duplicated detections,
    all-equal costs, and mixed constant rows (some at the class value, some at another, some
    above the limit) — bx_linear_assignment_ex and bx_lapjv(cost_limit) == the oracle's lapx."""
    rng = np.random.default_rng(4242)
    cases = [crowd_dup_costs(rng, nt, nd, de) for nt, nd, de in
             [(64, 32, 3), (128, 64, 3), (256, 128, 3), (96, 80, 2), (40, 90, 3)]]
    cases += [np.full((n, m), 0.5) for n, m in [(64, 64), (100, 37), (30, 120)]]
    for t in range(4):
        nr, nc = [(80, 60), (60, 80), (150, 90), (33, 33)][t]
        c = crowd_dup_costs(rng, nr, max(1, nc * 2 // 3))[:, :nc]
        c = np.hstack([c, np.ones((nr, nc - c.shape[1]))]) if c.shape[1] < nc else c
        rows = rng.choice(nr, nr // 3, replace=False)
        c[rows[: len(rows) // 3]] = 0.5  # constant rows at another value (the first may set K)
        c[rows[len(rows) // 3: 2 * len(rows) // 3]] = 0.9  # constant above the limit
        cases.append(np.ascontiguousarray(c))
    n_tied = 0
    for k, c in enumerate(cases):
        thr = 0.8
        om, oua, oub = po.linear_assignment(c, thr)
        tied = []
        gm, gua, gub = gpu_linear_assignment(torch_cuda, c, thr, tied)
        np.testing.assert_array_equal(gm, om, err_msg=f"case {k} {c.shape}")
        np.testing.assert_array_equal(gua, oua, err_msg=f"case {k}")
        np.testing.assert_array_equal(gub, oub, err_msg=f"case {k}")
        n_tied += tied[0]
        ox, oy = po.lapjv(c, extend_cost=True, cost_limit=thr)
        gx, gy = gpu_lapjv(torch_cuda, c, extend_cost=True, cost_limit=thr)
        np.testing.assert_array_equal(gx, ox, err_msg=f"lapjv x case {k}")
        np.testing.assert_array_equal(gy, oy, err_msg=f"lapjv y case {k}")
    assert n_tied >= len(cases) // 2


def gpu_lapjv(torch, cost, extend_cost=False, cost_limit=float("inf")):
    from boxmot_amd import _native as N

    c = dev(torch, np.ascontiguousarray(cost, np.float64))
    nr, nc = cost.shape
    x = torch.empty(max(nr, 1), dtype=torch.int32, device="cuda")
    y = torch.empty(max(nc, 1), dtype=torch.int32, device="cuda")
    N.check(N.load().bx_lapjv(c.data_ptr(), nr, nc, int(extend_cost), float(cost_limit),
                              x.data_ptr(), y.data_ptr(), None), "bx_lapjv")
    torch.cuda.synchronize()
    return host(x)[:nr], host(y)[:nc]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["square", "extend", "limit"])
def test_lapjv_ties_vs_oracle(torch_cuda, mode):
    """lapx's own algorithm on the GPU (register wave for n <= 64, LDS wave above) returns the
    oracle's x / y bit for bit on tie-heavy problems: small-integer costs, zero padding
    (association.py:105-114 / boosttrack/assoc.py:106-114) and cost_limit extensions."""
    rng = np.random.default_rng({"square": 1, "extend": 2, "limit": 3}[mode])
    sizes = [(1, 1), (2, 2), (3, 5), (7, 4), (17, 30), (40, 63), (64, 64), (50, 65), (65, 40),
             (100, 120), (200, 130), (333, 178), (512, 300)]
    for t, (nr, nc) in enumerate(sizes * 3):
        if mode == "square":
            nc = nr
        if mode == "limit" and nr + nc > 512:
            nr, nc = nr // 2, nc // 2
        hi = 2 + t % 5
        c = rng.integers(0, hi, (nr, nc)).astype(np.float64)
        if t % 3 == 1:
            c = -c  # maximisation form, as assoc.match's lapjv(-cost)
        if t % 3 == 2:
            c = np.round(rng.uniform(-1, 1, (nr, nc)), 1)
        kw = dict(extend_cost=mode != "square")
        if mode == "limit":
            kw["cost_limit"] = float(hi) / 2
        ox, oy = po.lapjv(c, **kw)
        gx, gy = gpu_lapjv(torch_cuda, c, **kw)
        np.testing.assert_array_equal(gx, ox, err_msg=f"x {mode} {nr}x{nc} t={t}")
        np.testing.assert_array_equal(gy, oy, err_msg=f"y {mode} {nr}x{nc} t={t}")


@pytest.mark.gpu
@pytest.mark.parametrize("shape,kw", [((4400, 4000), dict(extend_cost=True)),
                                      ((2300, 2100), dict(extend_cost=True, cost_limit=4.0)),
                                      ((4200, 4200), {})])
def test_lapjv_global_state_vs_oracle(torch_cuda, shape, kw):
    """bx_lapjv past the LDS (n > 4096: the solver state in HBM, its column-ownership atomics read
    back through an invalidated L1) on tie-heavy integer costs with a planted cheap matching."""
    rng = np.random.default_rng(7)
    nr, nc = shape
    c = rng.integers(5, 9, (nr, nc)).astype(np.float64)
    k = min(nr, nc)
    c[np.arange(k), rng.permutation(nc)[:k]] = rng.integers(0, 3, k)
    ox, oy = po.lapjv(c, **kw)
    gx, gy = gpu_lapjv(torch_cuda, c, **kw)
    np.testing.assert_array_equal(gx, ox)
    np.testing.assert_array_equal(gy, oy)


@pytest.mark.gpu
def test_lapjv_errors(torch_cuda):
    with pytest.raises(ValueError, match="Square cost array expected"):
        gpu_lapjv(torch_cuda, np.zeros((2, 3)))
    x, y = gpu_lapjv(torch_cuda, np.zeros((0, 3)), extend_cost=True)
    assert x.size == 0 and list(y) == [-1, -1, -1]


def test_linear_assignment_empty(torch_cuda):
    for shape in [(0, 4), (4, 0)]:
        m, ua, ub = gpu_linear_assignment(torch_cuda, np.zeros(shape), 0.5)
        assert m.shape == (0, 2) and ua.size == shape[0] and ub.size == shape[1]


# --------------------------------------------------------------------------- tracker level
def make_dropin(kind, args):
    from boxmot_amd import BoostTrack, BotSort, ByteTrack, OcSort

    if kind == "bytetrack":
        ByteTrack.clear_count()
        return ByteTrack(**args)
    if kind == "ocsort":
        return OcSort(**args)
    if kind == "boosttrack":
        BoostTrack._id_count = 0  # fixtures were captured with the class counter reset
        return BoostTrack(reid_weights=None, device="cuda", half=False, **args)
    if kind == "strongsort":  # captured with GITHUB_ACTIONS=true (born Confirmed, App. A D8)
        import os

        from boxmot_amd import StrongSort

        os.environ["GITHUB_ACTIONS"] = "true"
        os.environ.pop("GITHUB_JOB", None)
        return StrongSort(reid_weights=None, device="cuda", half=False, **args)
    return BotSort(reid_weights=None, device="cuda", half=False, **args)


@pytest.mark.parametrize("path", TRK_FIXTURES, ids=fixture_id)
def test_tracker_fixture_parity(torch_cuda, path):
    """Every tracker fixture through the drop-in: bitwise vs the oracle each frame, and vs the
    reference capture (ids/det_ind/cls exact, boxes 1e-9).  Ids ending "parity-unpinned-ties<N>"
    are fixtures whose tie order comes from the restated lapjv (golden_util.fixture_id)."""
    fx = np.load(path)
    kind, args = fixture_tracker_args(fx)
    # C4 size ("large"): the drop-in starts at its default capacities and grows to 1024 objects
    # (CapacityGuard); no oracle replay
    large = "large" in fx.files
    tr = make_dropin(kind, args)
    orc = None if large else po.OracleTracker(
        kind, **(dict(args, born_confirmed=True) if kind == "strongsort" else args))
    cmc = None
    if "warps" in fx.files:
        from boxmot_amd.synth import SyntheticCMC

        cmc = SyntheticCMC(lambda t: fixture_warp(fx, t))
        tr.cmc = cmc
    img = np.zeros((1080, 1920, 3), np.uint8)
    rows = []
    ncol = 10 if kind == "strongsort" else 8
    for f, d, e in fixture_frames(fx):
        if cmc is not None:
            cmc.t = f
        o = tr.update(d, img, e) if e is not None else tr.update(d, img)
        o = np.asarray(o, np.float64).reshape(-1, ncol)
        if orc is not None:
            oo = orc.update(d, e, fixture_warp(fx, f)).reshape(-1, ncol)
            np.testing.assert_array_equal(o, oo, err_msg=f"frame {f}: GPU != oracle")
        rows.append(np.concatenate([np.full((o.shape[0], 1), f), o], 1))
    crash = fixture_crash(fx)
    if crash is not None:  # the reference raised TypeError here (occlusion handler, D7)
        with pytest.raises(TypeError, match="not iterable"):
            tr.update(crash[1], img, crash[2])
    got = np.concatenate(rows, 0) if rows else np.zeros((0, fx["outputs"].shape[1]))
    compare_outputs(got, fx["outputs"], box_atol=1e-9,
                    conf_atol=1e-9 if kind == "boosttrack" else None)


PER_CLASS_CASES = [
    ("bytetrack", dict(min_conf=0.1, track_thresh=0.6, match_thresh=0.9, track_buffer=30),
     dict(n_obj=60, seed=31, layout="crowded", conf_lo=0.05, classes=(0, 1, 1, 3, 79, 80))),
    ("botsort", dict(track_high_thresh=0.6, new_track_thresh=0.7, match_thresh=0.8),
     dict(n_obj=56, seed=32, layout="crowded", emb_dim=48, conf_lo=0.05, classes=(2, 0, 5))),
    ("ocsort", dict(det_thresh=0.6, max_age=30, min_hits=3, inertia=0.1),
     dict(n_obj=56, seed=33, layout="crowded", conf_lo=0.2, p_det=0.85, classes=(0, 7, 3))),
    ("boosttrack", dict(max_age=60, min_hits=3, det_thresh=0.6, use_rich_s=True, use_sb=True,
                        use_vt=True, with_reid=True),
     dict(n_obj=40, seed=34, layout="crowded", emb_dim=32, emb_dtype=np.float64, conf_lo=0.3,
          p_det=0.9, classes=(1, 0))),
]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,args,skw", PER_CLASS_CASES, ids=[c[0] for c in PER_CLASS_CASES])
def test_per_class_vs_oracle(torch_cuda, kind, args, skw):
    """per_class=True (basetracker.py:155-201) through the drop-ins' native per-class paths:
    every frame bitwise equal to the oracle's restated class loop (ByteTrack/BoT-SORT with the
    shared lost list, OCSort isolated per class with class-global ids, BoostTrack's D10 sharing);
    BoT-SORT also on CMC-warp frames."""
    from boxmot_amd.synth import SyntheticCMC, SyntheticScene, synth_warp

    args = dict(args, per_class=True)
    tr = make_dropin(kind, args)
    orc = po.OracleTracker(kind, **args)
    sc = SyntheticScene(**skw)
    warp = kind == "botsort"
    if warp:
        tr.cmc = SyntheticCMC(lambda t: synth_warp(32, t))
    img = np.zeros((1080, 1920, 3), np.uint8)
    rows = 0
    for t in range(1, 51):
        d, e, _ = sc.frame(t)
        if warp:
            tr.cmc.t = t
        o = tr.update(d, img, e) if e is not None else tr.update(d, img)
        oo = orc.update(d, e, synth_warp(32, t) if warp else None)
        np.testing.assert_array_equal(np.asarray(o, np.float64).reshape(-1, 8), oo,
                                      err_msg=f"{kind} frame {t}")
        rows += oo.shape[0]
    assert rows > 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["botsort", "boosttrack"])
def test_per_class_stateful_cmc_vs_oracle(torch_cuda, kind):
    """under per_class=True the reference calls cmc.apply once per class call; an
    ECC-like CMC (boxmot_amd.synth.StatefulCMC) returns the frame's warp to class 0 and the
    identity to every later class call.  The drop-ins collect one warp per class call and the
    engine applies each to its own call: bitwise equal to the oracle fed the same warps."""
    from boxmot_amd.synth import StatefulCMC, SyntheticScene, synth_warp

    kind_, args, skw = next(c for c in PER_CLASS_CASES if c[0] == kind)
    args = dict(args, per_class=True)
    tr = make_dropin(kind, args)
    orc = po.OracleTracker(kind, **args)
    sc = SyntheticScene(**skw)
    tr.cmc = StatefulCMC(lambda t: synth_warp(36, t))
    img = np.zeros((1080, 1920, 3), np.uint8)
    for t in range(1, 41):
        d, e, _ = sc.frame(t)
        tr.cmc.t = t
        o = tr.update(d, img, e) if e is not None else tr.update(d, img)
        w = np.broadcast_to(np.eye(2, 3), (po.NR_CLASSES, 2, 3)).copy()
        w[0] = synth_warp(36, t)
        oo = orc.update(d, e, w)
        np.testing.assert_array_equal(np.asarray(o, np.float64).reshape(-1, 8), oo,
                                      err_msg=f"{kind} frame {t}")


def run_batched(torch, kind, scenes, n_frames, args, emb_dim=0, seq_frames=None, warps=None,
                overlap=False):
    """Drive an Engine with len(scenes) sequences in one launch per frame (``warps(s, t)``: the
    2x3 CMC warp of sequence s at frame t, BoT-SORT's multi_gmc).  ``overlap``: the engine leaves
    each step's feature EMA unjoined (bx_engine_set_overlap), so a step's input tensors are kept
    alive until the next step is enqueued."""
    from boxmot_amd.engine import Engine, EngineParams

    S = len(scenes)
    eng = Engine(kind, n_seq=S, track_cap=1024, det_cap=384, emb_dim=emb_dim,
                 params=EngineParams(**args))
    if overlap:
        eng.set_overlap(True)
    keep = None
    outs = [[] for _ in range(S)]
    for t in range(1, n_frames + 1):
        frames = [sc.frame(t) for sc in scenes]
        off = np.zeros(S + 1, np.int32)
        off[1:] = np.cumsum([f[0].shape[0] for f in frames])
        dets = np.concatenate([f[0] for f in frames], 0).astype(np.float32)
        dd = dev(torch, dets)
        do = dev(torch, off)
        de = dev(torch, np.concatenate([f[1] for f in frames], 0)) if emb_dim else None
        out = torch.empty((max(int(off[-1]), 1), 8), dtype=torch.float64, device="cuda")
        cnt = torch.empty(S, dtype=torch.int32, device="cuda")
        w = None if warps is None else dev(torch, np.stack([warps(s, t).reshape(6)
                                                            for s in range(S)]))
        eng.step(dd, do, de, w, out, cnt)
        keep = (dd, do, de, w)  # the previous step's inputs are released only now
        o, c = host(out), host(cnt)
        for s in range(S):
            outs[s].append(o[off[s]: off[s] + c[s]])
    assert eng.status() == 0
    del keep
    run_batched.engine = eng  # the last run's engine (Kalman-state checks)
    return outs


def assert_kalman_state_equal(eng, s, orc):
    """Track lists and Kalman state (covariances with their pending predicts applied) bitwise."""
    g, r = eng.tracks(s), orc.tracks()
    np.testing.assert_array_equal(g["id"], r["id"])
    np.testing.assert_array_equal(g["state"], r["state"])
    np.testing.assert_array_equal(g["mean"], r["mean"])
    np.testing.assert_array_equal(g["covariance"], r["covariance"])


@pytest.mark.parametrize("kind", ["bytetrack", "botsort"])
def test_batched_sequences_vs_oracle(torch_cuda, kind):
    from boxmot_amd.synth import SyntheticScene

    emb = 64 if kind == "botsort" else 0
    scenes = [SyntheticScene(n_obj=30 + 7 * s, seed=100 + s, emb_dim=emb,
                             layout="crowded" if s % 2 else "grid",
                             conf_lo=0.05 if s % 3 == 0 else 0.65) for s in range(6)]
    args = dict(min_conf=0.1, track_thresh=0.6, match_thresh=0.9, track_buffer=30) \
        if kind == "bytetrack" else dict(track_high_thresh=0.6, new_track_thresh=0.7,
                                         match_thresh=0.8)
    outs = run_batched(torch_cuda, kind, scenes, 60, args, emb)
    eng = run_batched.engine
    for s, sc in enumerate(scenes):
        orc = po.OracleTracker(kind, **args)
        for t in range(1, 61):
            d, e, _ = sc.frame(t)
            np.testing.assert_array_equal(outs[s][t - 1], orc.update(d, e),
                                          err_msg=f"seq {s} frame {t}")
        assert_kalman_state_equal(eng, s, orc)


def test_botsort_batched_warps_vs_oracle(torch_cuda):
    """multi_gmc (botsort_track.py:91-104) on per-sequence non-identity warps, several sequences
    per launch, against the oracle (itself pinned by the trk_botsort_warp_* fixtures)."""
    from boxmot_amd.synth import SyntheticScene, synth_warp

    scenes = [SyntheticScene(n_obj=24 + 9 * s, seed=140 + s, emb_dim=64,
                             layout="crowded" if s % 2 else "grid") for s in range(4)]
    args = dict(track_high_thresh=0.6, new_track_thresh=0.7, match_thresh=0.8)
    warps = lambda s, t: synth_warp(140 + s, t, rot=0.004 * (s + 1))  # noqa: E731
    outs = run_batched(torch_cuda, "botsort", scenes, 50, args, 64, warps=warps)
    eng = run_batched.engine
    for s, sc in enumerate(scenes):
        orc = po.OracleTracker("botsort", **args)
        for t in range(1, 51):
            d, e, _ = sc.frame(t)
            np.testing.assert_array_equal(outs[s][t - 1], orc.update(d, e, warps(s, t)),
                                          err_msg=f"seq {s} frame {t}")
        assert_kalman_state_equal(eng, s, orc)


@pytest.mark.parametrize("warped", [False, True])
def test_botsort_overlap_mode_vs_oracle(torch_cuda, warped):
    """bx_engine_set_overlap: each step returns with its feature EMA (K5) still on the side
    stream; the next step's K1 queues behind it and its cosine pass joins it.  Outputs (whose
    appearance costs read the previous frame's smooth_feat) and Kalman state bitwise vs the
    oracle, with and without warp frames; state reads settle the side stream first."""
    from boxmot_amd.synth import SyntheticScene, synth_warp

    scenes = [SyntheticScene(n_obj=40 + 11 * s, seed=170 + s, emb_dim=128,
                             layout="crowded" if s % 2 else "grid") for s in range(5)]
    args = dict(track_high_thresh=0.6, new_track_thresh=0.7, match_thresh=0.8)
    warps = (lambda s, t: synth_warp(170 + s, t)) if warped else None  # noqa: E731
    outs = run_batched(torch_cuda, "botsort", scenes, 40, args, 128, warps=warps, overlap=True)
    eng = run_batched.engine
    for s, sc in enumerate(scenes):
        orc = po.OracleTracker("botsort", **args)
        for t in range(1, 41):
            d, e, _ = sc.frame(t)
            np.testing.assert_array_equal(outs[s][t - 1],
                                          orc.update(d, e, warps(s, t) if warped else None),
                                          err_msg=f"seq {s} frame {t}")
        assert_kalman_state_equal(eng, s, orc)


def test_pending_covariance_predicts_mixed_warps(torch_cuda):
    """Lost tracks keep covariance predicts pending across identity-CMC frames (no per-frame
    covariance pass); warp frames and state reads apply them.  Warps on some frames only, Kalman
    state read mid-sequence and at the end — all bitwise against the oracle."""
    from boxmot_amd.synth import SyntheticScene, synth_warp

    scenes = [SyntheticScene(n_obj=30 + 10 * s, seed=150 + s, emb_dim=64, p_det=0.35,
                             layout="crowded" if s else "grid") for s in range(3)]
    args = dict(track_high_thresh=0.6, new_track_thresh=0.7, match_thresh=0.8)
    warps = lambda s, t: synth_warp(150 + s, t) if t % 7 == 0 else None  # noqa: E731
    from boxmot_amd.engine import Engine, EngineParams

    eng = Engine("botsort", n_seq=3, track_cap=512, det_cap=256, emb_dim=64,
                 params=EngineParams(**args))
    orcs = [po.OracleTracker("botsort", **args) for _ in scenes]
    for t in range(1, 46):
        fr = [sc.frame(t) for sc in scenes]
        off = np.zeros(4, np.int32)
        off[1:] = np.cumsum([f[0].shape[0] for f in fr])
        w = [warps(s, t) for s in range(3)]
        wd = None if w[0] is None else dev(torch_cuda, np.stack([x.reshape(6) for x in w]))
        out = torch_cuda.empty((max(int(off[-1]), 1), 8), dtype=torch_cuda.float64, device="cuda")
        cnt = torch_cuda.empty(3, dtype=torch_cuda.int32, device="cuda")
        eng.step(dev(torch_cuda, np.concatenate([f[0] for f in fr]).astype(np.float32)),
                 dev(torch_cuda, off), dev(torch_cuda, np.concatenate([f[1] for f in fr])), wd,
                 out, cnt)
        o, c = host(out), host(cnt)
        for s in range(3):
            np.testing.assert_array_equal(o[off[s]: off[s] + c[s]],
                                          orcs[s].update(fr[s][0], fr[s][1], w[s]),
                                          err_msg=f"seq {s} frame {t}")
            if t in (12, 30, 45):
                assert_kalman_state_equal(eng, s, orcs[s])
    assert eng.status() == 0


def test_botsort_c3_scale_vs_oracle(torch_cuda):
    """BASELINE config C3 geometry (256 objects, ~128 dets, 512-d) against the oracle."""
    from boxmot_amd.synth import SyntheticScene

    sc = SyntheticScene(n_obj=256, seed=11, emb_dim=512)
    args = dict(track_high_thresh=0.6, new_track_thresh=0.7, match_thresh=0.8)
    outs = run_batched(torch_cuda, "botsort", [sc], 45, args, 512)
    orc = po.OracleTracker("botsort", **args)
    for t in range(1, 46):
        d, e, _ = sc.frame(t)
        np.testing.assert_array_equal(outs[0][t - 1], orc.update(d, e), err_msg=f"frame {t}")


def test_float64_embeddings(torch_cuda):
    from boxmot_amd import BotSort
    from boxmot_amd.synth import SyntheticScene

    sc = SyntheticScene(n_obj=40, seed=5, emb_dim=32, emb_dtype=np.float64, layout="crowded")
    tr = BotSort(track_high_thresh=0.6, new_track_thresh=0.7)
    orc = po.OracleTracker("botsort", track_high_thresh=0.6, new_track_thresh=0.7)
    img = np.zeros((1080, 1920, 3), np.uint8)
    for t in range(1, 40):
        d, e, _ = sc.frame(t)
        o = np.asarray(tr.update(d, img, e), np.float64).reshape(-1, 8)
        np.testing.assert_array_equal(o, orc.update(d, e))


# ------------------------------------------------------ reference semantic tests, re-expressed
@pytest.mark.parametrize("name", ["bytetrack", "botsort"])
def test_reference_semantics(torch_cuda, name):
    """tests/unit/test_trackers.py of the reference: shape, empty input, assertions, ID stability."""
    from boxmot_amd import create_tracker, get_tracker_config

    def mk():
        return create_tracker(name, get_tracker_config(name), None, "cuda", False, False)

    rgb = np.random.randint(255, size=(640, 640, 3), dtype=np.uint8)
    det = np.array([[144, 212, 400, 480, 0.82, 0], [425, 281, 576, 472, 0.72, 65]])
    embs = np.random.random((2, 512))
    tr = mk()
    out = tr.update(det, rgb, embs) if name == "botsort" else tr.update(det, rgb)
    assert out.shape == (2, 8)

    for dets in (None, np.array([])):
        tr = mk()
        out = tr.update(dets, rgb, np.random.random((0, 512)))
        assert out.size == 0

    tr = mk()
    with pytest.raises(AssertionError):
        tr.update(np.random.rand(2, 5), rgb, np.random.rand(2, 512))
    if name == "botsort":
        with pytest.raises(AssertionError):
            mk().update(np.array([[10, 10, 20, 20, 0.7, 0]]), rgb, np.random.rand(2, 512))

    tr = mk()
    det = np.array([[50, 50, 100, 100, 0.95, 3]])
    e1 = np.random.rand(1, 512)
    o1 = tr.update(det, rgb, e1) if name == "botsort" else tr.update(det, rgb)
    o2 = tr.update(det, rgb, e1) if name == "botsort" else tr.update(det, rgb)
    assert o1.shape == o2.shape == (1, 8)
    assert o1[0, 4] == o2[0, 4]


def test_bytetrack_global_id_counter(torch_cuda):
    """ByteTrack ids continue across instances like the reference's process-global counter."""
    from boxmot_amd import ByteTrack

    ByteTrack.clear_count()
    rgb = np.zeros((640, 640, 3), np.uint8)
    det = np.array([[50, 50, 100, 100, 0.95, 0]])
    a = ByteTrack(track_thresh=0.6)
    assert a.update(det, rgb)[0, 4] == 1
    b = ByteTrack(track_thresh=0.6)
    assert b.update(det, rgb)[0, 4] == 2


def test_capacity_errors(torch_cuda):
    from boxmot_amd.engine import Engine

    eng = Engine("bytetrack", n_seq=1, track_cap=8, det_cap=4)
    with pytest.raises(ValueError):
        eng.update_host(0, np.zeros((5, 6)))
    dets = np.array([[10 * i, 0, 10 * i + 5, 5, 0.9, 0] for i in range(4)], np.float64)
    eng.update_host(0, dets)  # 4 tracks
    eng.update_host(0, dets + np.array([200, 200, 200, 200, 0, 0]))  # 4 new → 8 live
    with pytest.raises(RuntimeError):
        eng.update_host(0, dets + np.array([400, 400, 400, 400, 0, 0]))  # would need 12 slots


# ------------------------------------------------------------------------------------- OCSort
def run_ocsort_batched(torch, scenes, n_frames, args, track_cap=256, det_cap=256):
    from boxmot_amd.engine import OcsortEngine, OcsortParams

    S = len(scenes)
    eng = OcsortEngine(n_seq=S, track_cap=track_cap, det_cap=det_cap,
                       params=OcsortParams(**args))
    orcs = [po.OracleTracker("ocsort", **args) for _ in range(S)]
    for t in range(1, n_frames + 1):
        frames = [sc.frame(t)[0] for sc in scenes]
        off = np.zeros(S + 1, np.int32)
        off[1:] = np.cumsum([f.shape[0] for f in frames])
        dets = np.concatenate(frames, 0).astype(np.float32)
        out = torch.empty((max(int(off[-1]), 1), 8), dtype=torch.float64, device="cuda")
        cnt = torch.empty(S, dtype=torch.int32, device="cuda")
        eng.step(dev(torch, dets), dev(torch, off), out, cnt)
        o, c = host(out), host(cnt)
        for s in range(S):
            np.testing.assert_array_equal(o[off[s]: off[s] + c[s]], orcs[s].update(frames[s]),
                                          err_msg=f"seq {s} frame {t}")
    assert eng.status() == 0
    # Kalman state: bitwise the oracle's (and so within 1e-5 rel of the reference)
    for s in range(S):
        g, r = eng.tracks(s), orcs[s].ocsort_tracks()
        np.testing.assert_array_equal(g["id"], r["id"])
        np.testing.assert_array_equal(g["x"], r["x"])
        np.testing.assert_array_equal(g["P"], r["P"])


OCS_ARGS = dict(min_conf=0.1, det_thresh=0.6, max_age=30, min_hits=3, asso_threshold=0.3,
                delta_t=3, inertia=0.1, use_byte=False, Q_xy_scaling=0.01, Q_s_scaling=0.0001)


@pytest.mark.parametrize("variant", ["default", "byte", "short_age", "giou", "diou_byte", "ciou",
                                     "hmiou", "centroid"])
def test_ocsort_batched_vs_oracle(torch_cuda, variant):
    """Several sequences per launch (grid / crowded layouts, low-confidence detections, missed
    detections -> ORU re-updates, deaths) against the oracle, outputs and KF state bitwise."""
    from boxmot_amd.synth import SyntheticScene

    args = dict(OCS_ARGS)
    if variant == "byte":
        args.update(use_byte=True, det_thresh=0.5)
    if variant == "short_age":
        args.update(max_age=5, min_hits=1, delta_t=1, inertia=0.3)
    if variant in ("giou", "ciou", "hmiou"):
        args.update(asso_func=variant)
    if variant == "diou_byte":
        args.update(asso_func="diou", use_byte=True, det_thresh=0.5)
    if variant == "centroid":  # 1 - distance / frame diagonal: a threshold near 1
        args.update(asso_func="centroid", asso_threshold=0.95, frame_w=1280, frame_h=720)
    scenes = [SyntheticScene(n_obj=12 + 9 * s, seed=300 + s,
                             layout="crowded" if s % 2 else "grid", p_det=0.35 + 0.1 * (s % 3),
                             conf_lo=0.2 if s % 3 == 0 else 0.55) for s in range(6)]
    run_ocsort_batched(torch_cuda, scenes, 60, args)


def test_ocsort_large_scene_vs_oracle(torch_cuda):
    """A crowded 160-object sequence: assignment problems past the LDS cost budget (HBM path)."""
    from boxmot_amd.synth import SyntheticScene

    sc = SyntheticScene(n_obj=160, seed=17, layout="crowded", p_det=0.3, conf_lo=0.4)
    run_ocsort_batched(torch_cuda, [sc], 30, dict(OCS_ARGS, use_byte=True, det_thresh=0.5))


def test_ocsort_empty_frames_and_global_ids(torch_cuda):
    from boxmot_amd import OcSort

    img = np.zeros((720, 1280, 3), np.uint8)
    a = OcSort(**OCS_ARGS)
    orc = po.OracleTracker("ocsort", **OCS_ARGS)
    d = np.array([[10, 10, 60, 120, 0.9, 0], [200, 50, 260, 170, 0.8, 2]], np.float32)
    for t in range(6):
        dd = d if t not in (2, 3) else np.empty((0, 6), np.float32)
        o = np.asarray(a.update(dd, img), np.float64).reshape(-1, 8)
        np.testing.assert_array_equal(o, orc.update(dd))
    # the id counter is class-global: a second instance resets it, the first continues from it
    b = OcSort(**OCS_ARGS)
    ob = b.update(d, img)
    assert ob.shape == (2, 8) and sorted(ob[:, 4]) == [1.0, 2.0]
    assert OcSort._id_count == 2


# ------------------------------------------------------------- StrongSort appearance metric
def gpu_nn_cosine(torch, samples, off, feats, normalized=False):
    from boxmot_amd import _native as N

    L = N.load()
    s = dev(torch, np.asarray(samples, np.float64).reshape(-1, feats.shape[1]))
    o = dev(torch, np.asarray(off, np.int32))
    f = dev(torch, np.asarray(feats, np.float64))
    T, D, F = len(off) - 1, feats.shape[0], feats.shape[1]
    out = torch.full((T, D), -7.0, dtype=torch.float64, device="cuda")
    N.check(L.bx_nn_cosine_distance(s.data_ptr(), int(off[-1]), o.data_ptr(), T, f.data_ptr(), D,
                                    F, 1 if normalized else 0, out.data_ptr(), None),
            "bx_nn_cosine_distance")
    return host(out)


@pytest.mark.parametrize("case", ["small", "reid512", "reid2048"])
def test_nn_cosine_distance_fixture(torch_cuda, case):
    """Reference NearestNeighborDistanceMetric.distance (after partial_fit rounds): the fp64 MFMA
    op equals the oracle bitwise and the reference within 1e-13 (np.dot's BLAS order)."""
    fx = np.load(GOLDEN / "strongsort_ops.npz")
    s, off, f, ref = (fx[f"{case}_{k}"] for k in ("samples", "off", "feats", "dist"))
    got = gpu_nn_cosine(torch_cuda, s, off, f)
    np.testing.assert_array_equal(got, po.nn_cosine_distance(s, off, f))
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-13)


@pytest.mark.parametrize("F,T,D,smax", [(100, 37, 300, 9), (2048, 9, 513, 40), (16, 300, 5, 3),
                                        (512, 70, 129, 150), (64, 240, 300, 160)])
def test_nn_cosine_distance_random_vs_oracle(torch_cuda, F, T, D, smax):
    """Ragged galleries (empty targets, tiles spanning several targets, F not a multiple of the
    16-wide K chunk, D past one 256-wide column block; the last case is large enough for the
    128 x 256 tile, the others run the 64 x 64 one): bitwise vs the oracle."""
    rng = np.random.default_rng(F * 7 + T)
    cnt = rng.integers(0, smax + 1, T)
    cnt[0] = 0
    off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
    base = rng.normal(size=(T, F))
    s = np.repeat(base, cnt, 0) + 0.5 * rng.normal(size=(int(off[-1]), F))
    s *= rng.uniform(0.2, 3.0, (s.shape[0], 1))
    f = base[rng.integers(0, T, D)] + 0.5 * rng.normal(size=(D, F))
    f[0] = s[0] if s.shape[0] else f[0]  # an exact match: distance 0 (clip at 1)
    got = gpu_nn_cosine(torch_cuda, s, off, f)
    np.testing.assert_array_equal(got, po.nn_cosine_distance(s, off, f))
    # a gallery kept normalised (BX_NN_SAMPLES_NORMALIZED): samples used as given
    sh = s / (np.linalg.norm(s, axis=1, keepdims=True) + 1e-8)
    fh = f / (np.linalg.norm(f, axis=1, keepdims=True) + 1e-8)
    got_n = gpu_nn_cosine(torch_cuda, sh, off, f, normalized=True)
    for t in range(T):
        if cnt[t] == 0:
            assert np.all(got_n[t] == 1e5)
        else:
            ref = (1 - np.clip(sh[off[t]:off[t + 1]] @ fh.T, -1, 1)).min(0)
            np.testing.assert_allclose(got_n[t], ref, rtol=0, atol=1e-13)


# ----------------------------------------------------------------------------------- BoostTrack
BOOST_ARGS = dict(max_age=60, min_hits=3, det_thresh=0.6, iou_threshold=0.3, use_ecc=True,
                  min_box_area=10, aspect_ratio_thresh=1.6, lambda_iou=0.5, lambda_mhd=0.25,
                  lambda_shape=0.25, use_dlo_boost=True, use_duo_boost=True, dlo_boost_coef=0.65,
                  s_sim_corr=False, use_rich_s=True, use_sb=True, use_vt=True, with_reid=True)


def run_boost_batched(torch, scenes, n_frames, args, emb_dim, track_cap=256, det_cap=256,
                      warps=None):
    """BoostEngine with len(scenes) sequences per launch vs one oracle per sequence: outputs and
    the track state (ids, Kalman mean/covariance, embeddings) bitwise."""
    from boxmot_amd.engine import BoostEngine, BoostParams

    S = len(scenes)
    eng = BoostEngine(n_seq=S, track_cap=track_cap, det_cap=det_cap, emb_dim=emb_dim,
                      params=BoostParams(**args))
    orcs = [po.OracleTracker("boosttrack", **args) for _ in range(S)]
    reid = args["with_reid"]
    for t in range(1, n_frames + 1):
        frames = [sc.frame(t) for sc in scenes]
        off = np.zeros(S + 1, np.int32)
        off[1:] = np.cumsum([f[0].shape[0] for f in frames])
        dets = np.concatenate([f[0] for f in frames], 0).astype(np.float32)
        de = None
        if reid:
            de = dev(torch, np.concatenate([f[1] for f in frames], 0).astype(np.float64))
        w = None if warps is None else dev(torch, np.stack([warps(s, t) for s in range(S)]))
        out = torch.empty((max(int(off[-1]), 1), 8), dtype=torch.float64, device="cuda")
        cnt = torch.empty(S, dtype=torch.int32, device="cuda")
        eng.step(dev(torch, dets), dev(torch, off), de, w, out, cnt)
        o, c = host(out), host(cnt)
        for s in range(S):
            ref = orcs[s].update(frames[s][0], frames[s][1] if reid else None,
                                 None if warps is None else warps(s, t))
            np.testing.assert_array_equal(o[off[s]: off[s] + c[s]], ref,
                                          err_msg=f"seq {s} frame {t}")
    assert eng.status() == 0
    for s in range(S):
        g = eng.tracks(s)
        L = po.lib()
        n = L.bxo_boost_tracks(orcs[s].h, 0, None, None, None)
        ids = np.zeros(max(n, 1), np.int32)
        x = np.zeros((max(n, 1), 8))
        P = np.zeros((max(n, 1), 8, 8))
        L.bxo_boost_tracks(orcs[s].h, n, ids.ctypes.data, x.ctypes.data, P.ctypes.data)
        np.testing.assert_array_equal(g["id"], ids[:n])
        np.testing.assert_array_equal(g["x"], x[:n])
        np.testing.assert_array_equal(g["P"], P[:n])
    return eng


@pytest.mark.parametrize("variant", ["plusplus", "plain", "v2_sb", "vt_noreid"])
def test_boosttrack_batched_vs_oracle(torch_cuda, variant):
    """Several sequences per launch (grid / crowded layouts, low-confidence detections for the
    DLO/DUO boosts, misses, deaths) against the oracle, outputs and Kalman state bitwise."""
    from boxmot_amd.synth import SyntheticScene

    args = dict(BOOST_ARGS)
    emb = 64
    if variant == "plain":
        args.update(use_rich_s=False, use_sb=False, use_vt=False, with_reid=False)
    if variant == "v2_sb":
        args.update(s_sim_corr=True, use_vt=False, det_thresh=0.5, max_age=8, min_hits=1)
    if variant == "vt_noreid":
        args.update(use_sb=False, with_reid=False, use_ecc=False)
    if not args["with_reid"]:
        emb = 0
    scenes = [SyntheticScene(n_obj=12 + 9 * s, seed=500 + s, emb_dim=emb or 0,
                             emb_dtype=np.float64, layout="crowded" if s % 2 else "grid",
                             p_det=0.4 + 0.1 * (s % 3), conf_lo=0.2 if s % 3 == 0 else 0.4)
              for s in range(6)]
    run_boost_batched(torch_cuda, scenes, 60, args, emb)


class _EmptyScene:
    def __init__(self, emb_dim):
        self.emb_dim = emb_dim

    def frame(self, t):
        return np.zeros((0, 6)), np.zeros((0, self.emb_dim))


@pytest.mark.parametrize("n_seq", [384, 600, 1024])
def test_boosttrack_wide_launch_vs_oracle(torch_cuda, n_seq):
    """Launch widths with fewer threads per sequence (three and two waves: `frame_threads`):
    three busy sequences (first, middle, last) among empty ones, bitwise against the oracle."""
    from boxmot_amd.synth import SyntheticScene

    busy = {0: 0, n_seq // 2: 1, n_seq - 1: 2}
    scenes = [SyntheticScene(n_obj=30 + 12 * busy[s], seed=900 + s, emb_dim=32,
                             emb_dtype=np.float64, layout="crowded" if busy[s] != 1 else "grid",
                             p_det=0.5, conf_lo=0.3)
              if s in busy else _EmptyScene(32) for s in range(n_seq)]
    run_boost_batched(torch_cuda, scenes, 30, dict(BOOST_ARGS), 32, track_cap=128, det_cap=64)


def test_boosttrack_engines_of_different_lds_sizes(torch_cuda):
    """The frame kernel's dynamic-LDS limit is shared by every engine: a later engine with a
    smaller LDS footprint (more sequences: less LDS per workgroup) must not shrink the limit an
    earlier one launches with.  Steps the small-launch engine after creating the large one and
    checks it against the oracle."""
    from boxmot_amd.engine import BoostEngine, BoostParams
    from boxmot_amd.synth import SyntheticScene

    args = dict(BOOST_ARGS)
    big = BoostEngine(n_seq=2, track_cap=128, det_cap=64, emb_dim=32, params=BoostParams(**args))
    BoostEngine(n_seq=1024, track_cap=128, det_cap=64, emb_dim=32, params=BoostParams(**args))
    sc = SyntheticScene(n_obj=30, seed=31, emb_dim=32, emb_dtype=np.float64, layout="crowded",
                        p_det=0.5, conf_lo=0.3)
    orc = po.OracleTracker("boosttrack", **args)
    for t in range(1, 16):
        d, e = sc.frame(t)[:2]
        np.testing.assert_array_equal(big.update_host(0, d, e), orc.update(d, e),
                                      err_msg=f"frame {t}")
    assert big.status() == 0


class _DupScene:
    """A scene whose detections are each listed twice (same box, score and embedding): every
    association with both copies in play has a tied optimum, so the frame kernel's
    shortest-augmenting-path solve must hand it to lapjv (lapx's own order decides)."""

    def __init__(self, sc, every=1):
        self.sc, self.every, self.emb_dim = sc, every, sc.emb_dim

    def frame(self, t):
        d, e = self.sc.frame(t)[:2]
        k = np.arange(0, d.shape[0], self.every)
        dd = np.concatenate([d, d[k]], 0)
        ee = np.concatenate([e, e[k]], 0) if e is not None and e.size else e
        return dd, ee


@pytest.mark.parametrize("variant", ["reid", "noreid"])
def test_boosttrack_tied_assignments_vs_oracle(torch_cuda, variant):
    """Tied LAP optima (duplicated detections; without ReID also exactly-zero costs of
    non-overlapping pairs, tied with lapjv's zero padding): the tie test must send them to lapjv,
    outputs and Kalman state bitwise against the oracle (lapjv_restated order)."""
    from boxmot_amd.synth import SyntheticScene

    args = dict(BOOST_ARGS)
    emb = 48
    if variant == "noreid":
        args.update(with_reid=False, use_sb=False, use_vt=False, use_rich_s=False)
        emb = 0
    scenes = [_DupScene(SyntheticScene(n_obj=10 + 6 * s, seed=1300 + s, emb_dim=emb,
                                       emb_dtype=np.float64, layout="crowded" if s % 2 else "grid",
                                       p_det=0.6, conf_lo=0.3), every=1 + s)
              for s in range(4)]
    run_boost_batched(torch_cuda, scenes, 30, args, emb)


def test_boosttrack_large_scene_vs_oracle(torch_cuda):
    """A crowded 160-object sequence with 512-d ReID: cost matrices past the LDS budget (HBM
    path), several MFMA output tiles per sequence, LAP solves."""
    from boxmot_amd.synth import SyntheticScene

    sc = SyntheticScene(n_obj=160, seed=23, layout="crowded", p_det=0.5, conf_lo=0.3,
                        emb_dim=512, emb_dtype=np.float64)
    run_boost_batched(torch_cuda, [sc], 25, dict(BOOST_ARGS), 512)


def test_boosttrack_warp_and_embeddings(torch_cuda):
    """Non-identity camera warps per sequence (camera_update) and the embedding EMA state."""
    from boxmot_amd.synth import SyntheticScene

    scenes = [SyntheticScene(n_obj=20 + 5 * s, seed=700 + s, emb_dim=96, emb_dtype=np.float64,
                             conf_lo=0.3) for s in range(3)]

    def warp(s, t):
        a = 0.002 * np.sin(0.3 * t + s)
        return np.array([[1.0 + a, -a, 1.5 * s - 0.5], [a, 1.0 - a, 0.25 * t % 2.0]])

    eng = run_boost_batched(torch_cuda, scenes, 40, dict(BOOST_ARGS), 96, warps=warp)
    snap = eng.tracks(0)
    norms = np.linalg.norm(snap["emb"], axis=1)
    assert snap["emb"].shape[1] == 96 and np.all(norms > 0)


def test_boosttrack_dropin_empty_frames_and_global_ids(torch_cuda):
    from boxmot_amd import BoostTrack, create_tracker

    img = np.zeros((720, 1280, 3), np.uint8)
    BoostTrack._id_count = 0
    args = dict(BOOST_ARGS, with_reid=False)
    a = BoostTrack(**args)
    orc = po.OracleTracker("boosttrack", **args)
    d = np.array([[10, 10, 60, 120, 0.9, 0], [200, 50, 260, 170, 0.8, 2]], np.float32)
    for t in range(6):
        dd = d if t not in (2, 3) else np.empty((0, 6), np.float32)
        o = a.update(dd, img)
        assert o.shape[1] == 8
        np.testing.assert_array_equal(o, orc.update(dd))
    # the id counter is class-global and never reset: a second instance continues it
    b = BoostTrack(**args)
    ob = b.update(d, img)
    assert ob.shape == (2, 8) and sorted(ob[:, 4]) == [3.0, 4.0]
    # the plugin path (YAML defaults = BoostTrack++ with ReID) takes embeddings
    t = create_tracker("boosttrack")
    e = np.random.default_rng(0).standard_normal((2, 32))
    assert t.update(d, img, e).shape[1] == 8
    with pytest.raises(AssertionError):
        t.update(d, img, e[:1])


# ----------------------------------------------------------------------------------- StrongSort
SS_ARGS = dict(min_conf=0.1, max_cos_dist=0.15, max_iou_dist=0.7, max_age=50, n_init=2,
               nn_budget=150, mc_lambda=0.995, ema_alpha=0.9, conf_thresh_high=0.7,
               conf_thresh_low=0.3, id_preservation_weight=0.1, crowd_detection=True,
               born_confirmed=True)


def run_ss_batched(torch, scenes, n_frames, args, emb_dim, track_cap=256, det_cap=256,
                   warps=None, vec_cap=32, lsap_fast=True):
    """SsEngine with len(scenes) sequences per launch vs one oracle per sequence: outputs and
    Kalman state bitwise."""
    from boxmot_amd.engine import SsEngine, SsParams

    S = len(scenes)
    eng = SsEngine(n_seq=S, track_cap=track_cap, det_cap=det_cap, emb_dim=emb_dim,
                   vec_cap=vec_cap, params=SsParams(**args))
    if not lsap_fast:
        eng.set_lsap_mode(False)
    orcs = [po.OracleTracker("strongsort", **args) for _ in range(S)]
    for t in range(1, n_frames + 1):
        frames = [sc.frame(t) for sc in scenes]
        off = np.zeros(S + 1, np.int32)
        off[1:] = np.cumsum([f[0].shape[0] for f in frames])
        dets = np.concatenate([f[0] for f in frames], 0).astype(np.float64)
        de = dev(torch, np.concatenate([f[1] for f in frames], 0).astype(np.float64))
        w = None if warps is None else dev(torch, np.stack([warps(s, t) for s in range(S)]))
        out = torch.empty((max(int(off[-1]), 1), 10), dtype=torch.float64, device="cuda")
        cnt = torch.empty(S, dtype=torch.int32, device="cuda")
        eng.step(dev(torch, dets), dev(torch, off), de, w, out, cnt)
        o, c = host(out), host(cnt)
        for s in range(S):
            ref = orcs[s].update(frames[s][0], frames[s][1],
                                 None if warps is None else warps(s, t))
            np.testing.assert_array_equal(o[off[s]: off[s] + c[s]], ref,
                                          err_msg=f"seq {s} frame {t}")
    assert eng.status() == 0
    L = po.lib()
    for s in range(S):
        g = eng.tracks(s)
        n = L.bxo_ss_tracks(orcs[s].h, 0, None, None, None, None)
        ids = np.zeros(max(n, 1), np.int32)
        st = np.zeros(max(n, 1), np.int32)
        mean = np.zeros((max(n, 1), 8))
        cov = np.zeros((max(n, 1), 8, 8))
        L.bxo_ss_tracks(orcs[s].h, n, ids.ctypes.data, st.ctypes.data, mean.ctypes.data,
                        cov.ctypes.data)
        np.testing.assert_array_equal(g["id"], ids[:n])
        np.testing.assert_array_equal(g["state"], st[:n])
        np.testing.assert_array_equal(g["mean"], mean[:n])
        np.testing.assert_array_equal(g["covariance"], cov[:n])
    return eng


@pytest.mark.parametrize("variant", ["default", "churn", "crowd", "tentative"])
def test_strongsort_batched_vs_oracle(torch_cuda, variant):
    """Several sequences per launch against the oracle: cascade levels, IoU stage, recovery from
    the lost buffer (churn), crowd mode, Tentative births; outputs and Kalman state bitwise."""
    from boxmot_amd.synth import SyntheticScene

    args = dict(SS_ARGS)
    kw = dict(emb_dim=48, emb_dtype=np.float64, conf_lo=0.15)
    if variant == "default":
        scenes = [SyntheticScene(n_obj=16 + 8 * s, seed=800 + s,
                                 layout="crowded" if s % 2 else "grid", **kw) for s in range(4)]
    elif variant == "churn":
        args.update(max_age=6, nn_budget=12)
        scenes = [SyntheticScene(n_obj=14 + 6 * s, seed=810 + s, p_det=0.3, **kw)
                  for s in range(4)]
    elif variant == "crowd":
        args.update(max_age=8, nn_budget=16)
        scenes = [SyntheticScene(n_obj=10 + 2 * s, seed=820 + s, layout="crowded", width=60.0,
                                 height=60.0, **kw) for s in range(3)]
    else:  # Tentative tracks are never matched nor deleted (App. A D8): they accumulate
        args.update(born_confirmed=False)
        scenes = [SyntheticScene(n_obj=12, seed=830 + s, **kw) for s in range(2)]
        run_ss_batched(torch_cuda, scenes, 30, args, 48, track_cap=512)
        return
    run_ss_batched(torch_cuda, scenes, 50, args, 48)


class DupScene:
    """A scene whose every `every`-th detection is repeated (same box, confidence, class and
    embedding) at the end of the frame: the cascade's LSAPs get exactly tied optima."""

    def __init__(self, sc, every):
        self.sc, self.every = sc, every

    def frame(self, t):
        d, e, x = self.sc.frame(t)
        k = np.arange(0, d.shape[0], self.every)
        return np.concatenate([d, d[k]], 0), np.concatenate([e, e[k]], 0), x


@pytest.mark.parametrize("lsap_fast", [True, False])
def test_strongsort_tied_lsaps_vs_oracle(torch_cuda, lsap_fast):
    """Duplicated detections make min_cost_matching's optimum tie between the copies: solve +
    certify must detect every such tie and re-solve it in scipy's order (or restart its cascade
    stage in scipy's order when an earlier level's unmatched order was only certified up to
    rejected pairs), and give the oracle's outputs and Kalman state bit for bit; scipy's order
    throughout (lsap_fast False) too."""
    from boxmot_amd.synth import SyntheticScene

    args = dict(SS_ARGS)
    args.update(max_age=8)
    scenes = [DupScene(SyntheticScene(n_obj=24 + 12 * s, seed=870 + s, emb_dim=48,
                                      emb_dtype=np.float64, conf_lo=0.15,
                                      layout="crowded" if s % 2 else "grid"), 2 + s)
              for s in range(4)]
    eng = run_ss_batched(torch_cuda, scenes, 40, args, 48, lsap_fast=lsap_fast)
    st = eng.lsap_stats()
    print(f"lsap_fast={lsap_fast}: {st}")
    if lsap_fast:
        assert st["ties"] > 0 and st["unique"] + st["unique_up_to_rejected"] > 0, st
    else:
        assert st["ties"] == 0 and st["unique"] == st["solves"], st


def test_strongsort_large_scene_vs_oracle(torch_cuda):
    """128 objects with 512-d ReID: several MFMA row/column tiles per track, large LSAPs."""
    from boxmot_amd.synth import SyntheticScene

    sc = SyntheticScene(n_obj=128, seed=31, emb_dim=512, emb_dtype=np.float64, conf_lo=0.15)
    run_ss_batched(torch_cuda, [sc], 20, dict(SS_ARGS), 512, track_cap=1024)


def test_strongsort_batched_warps_vs_oracle(torch_cuda):
    """Track.camera_update (sort/track.py:173-189) on per-sequence non-identity warps, against
    the oracle (pinned by the trk_strongsort_warp_* fixtures); outputs and Kalman state."""
    from boxmot_amd.synth import SyntheticScene, synth_warp

    scenes = [SyntheticScene(n_obj=20 + 8 * s, seed=860 + s, emb_dim=48, emb_dtype=np.float64,
                             conf_lo=0.15, layout="crowded" if s % 2 else "grid")
              for s in range(3)]
    run_ss_batched(torch_cuda, scenes, 40, dict(SS_ARGS), 48,
                   warps=lambda s, t: synth_warp(860 + s, t, rot=0.004 * (s + 1)).reshape(6))


def test_strongsort_c4_size_vs_oracle(torch_cuda):
    """configs[3] at its stated size: one sequence of 1024 objects (~512 detections a frame) with
    2048-d ReID and budget 150, at the bench's capacities (bench.py strongsort_c4) — the frames
    take the LDS-overflow paths of the match / pre kernels and the 4-track NN tiles; outputs
    every frame and the final Kalman state bitwise against the oracle (sort/tracker.py:183-281)."""
    from boxmot_amd.synth import SyntheticScene

    from boxmot_amd.workloads import CONFIGS, SS_C4_CAPS

    _, n_obj, F, params = CONFIGS["strongsort_c4"]
    caps = SS_C4_CAPS
    sc = SyntheticScene(n_obj=n_obj, seed=41, emb_dim=F, emb_dtype=np.float64, conf_lo=0.3)
    eng = run_ss_batched(torch_cuda, [sc], 16, dict(params), F, track_cap=caps["track_cap"],
                         det_cap=caps["det_cap"], vec_cap=caps["vec_cap"])
    st = eng.frame_stats()
    assert st["dets"] > 450 and st["tracks"] > 900, st  # the C4 geometry was really exercised


@pytest.mark.parametrize("emb_dim", [128, 1024, 2048, 640, 100, 37])
def test_strongsort_feature_widths_vs_oracle(torch_cuda, emb_dim):
    """Feature widths around the NN kernel's k-blocks and the pairwise norm's leaf tree: one
    leaf (128), 8 and 16 leaves (1024, 2048: the shuffle fold), 640 (the generic split tree);
    100 (whole 8-element MFMA-order blocks then a 4-element tail in order), 37 (odd: no 16-byte
    loads, every element in order)."""
    from boxmot_amd.synth import SyntheticScene

    scenes = [SyntheticScene(n_obj=20 + 10 * s, seed=900 + s, emb_dim=emb_dim,
                             emb_dtype=np.float64, conf_lo=0.15) for s in range(2)]
    run_ss_batched(torch_cuda, scenes, 15, dict(SS_ARGS), emb_dim)


def test_strongsort_dropin(torch_cuda, monkeypatch):
    from boxmot_amd import StrongSort, create_tracker

    monkeypatch.setenv("GITHUB_ACTIONS", "true")
    monkeypatch.delenv("GITHUB_JOB", raising=False)
    img = np.zeros((720, 1280, 3), np.uint8)
    t = StrongSort()  # the reference's defaults: handle_occlusions=True
    orc = po.OracleTracker("strongsort", **SS_ARGS, handle_occlusions=True)
    rng = np.random.default_rng(5)
    base = rng.standard_normal((3, 32))
    d = np.array([[10, 10, 60, 120, 0.9, 0], [200, 50, 260, 170, 0.8, 2],
                  [400, 300, 470, 460, 0.5, 0]], np.float64)
    for k in range(8):
        dd = d if k not in (3, 4) else d[:0]
        e = base[: len(dd)] + 0.01 * rng.standard_normal((len(dd), 32))
        o = np.asarray(t.update(dd, img, e), np.float64).reshape(-1, 10)
        np.testing.assert_array_equal(o, orc.update(dd, e).reshape(-1, 10))
    y = create_tracker("strongsort")
    assert not hasattr(y, "per_class") or y.per_class is False
    with pytest.raises(AssertionError):
        y.update(d, img, base[:2])


# ------------------------------------------------------------------- many-sequence runner
@pytest.mark.parametrize("kind", ["bytetrack", "botsort", "ocsort", "boosttrack", "strongsort"])
def test_run_sequences_matches_per_sequence_dropins(torch_cuda, tmp_path, kind):
    """motio.run_sequences (one batched engine for all sequences, val.py:357-405's process pool
    replaced) writes the same MOT files as one fresh drop-in tracker per sequence fed by
    MOT17.py's np.loadtxt + mask selection (val.py:337-353); inputs in val.py's text format."""
    import os

    from boxmot_amd import BoostTrack, ByteTrack, motio
    from boxmot_amd.synth import SyntheticScene
    from boxmot_amd.tracker_zoo import create_tracker

    os.environ["GITHUB_ACTIONS"] = "true"  # StrongSort born Confirmed, like its fixtures
    os.environ.pop("GITHUB_JOB", None)
    rng = np.random.default_rng(9)
    F = 32
    rows = {}
    fx = np.load(GOLDEN / "trk_bytetrack_MOT17-02-FRCNN.npz")
    rows["MOT17-02-FRCNN"] = fx["dets"][fx["dets"][:, 0] <= 60]
    for s in (1, 2):
        sc = SyntheticScene(n_obj=20 + 10 * s, seed=40 + s, layout="crowded" if s == 2 else "grid")
        fr = []
        for t in range(1, 50):
            if t % 11 == 5:  # a frame without detections
                continue
            d = sc.frame(t)[0]
            fr.append(np.concatenate([np.full((d.shape[0], 1), t), d], 1))
        rows[f"SYN-{s}"] = np.concatenate(fr)
    packed, frame_ids = {}, {}
    for nm, r in rows.items():
        e = rng.standard_normal((r.shape[0], F))
        e /= np.linalg.norm(e, axis=1, keepdims=True)
        dp, ep = tmp_path / f"{nm}.dets.txt", tmp_path / f"{nm}.embs.txt"
        np.savetxt(dp, r, fmt="%f", header=nm)
        np.savetxt(ep, e, fmt="%f")
        packed[nm] = motio.pack_sequence(dp, ep, tmp_path / f"{nm}.bxmot")
        frame_ids[nm] = list(range(1, int(r[:, 0].max()) + 2))  # image frames, some empty
    # StrongSort: MOT17-02 has mutually occluding tracks at the top-left corner, where the
    # default handle_occlusions=True raises (D7) in the runner and the drop-in alike
    kw = dict(handle_occlusions=False) if kind == "strongsort" else {}
    if kind == "strongsort":
        with pytest.raises(TypeError, match="not iterable"):
            motio.run_sequences(kind, packed, tmp_path / "crash", frame_ids=frame_ids)
    motio.run_sequences(kind, packed, tmp_path / "batched", frame_ids=frame_ids,
                        tracker_kwargs=kw)
    img = np.zeros((1080, 1920, 3), np.uint8)
    for nm in rows:
        ByteTrack.clear_count()
        BoostTrack._id_count = 0
        tr = create_tracker(kind, evolve_param_dict=kw) if kw else create_tracker(kind)
        dets = np.loadtxt(tmp_path / f"{nm}.dets.txt", comments="#")
        embs = np.loadtxt(tmp_path / f"{nm}.embs.txt", comments="#")
        out = []
        for fid in frame_ids[nm]:
            mask = dets[:, 0].astype(int) == fid
            d, e = dets[mask, 1:], embs[mask]
            if d.size and e.size:
                tracks = np.asarray(tr.update(d, img, e))
                if tracks.size:
                    out.append(motio.convert_to_mot_format(tracks, fid))
        motio.write_mot_results(tmp_path / "single" / f"{nm}.txt",
                                np.vstack(out) if out else np.empty((0, 0)))
        a = (tmp_path / "batched" / f"{nm}.txt").read_bytes()
        b = (tmp_path / "single" / f"{nm}.txt").read_bytes()
        assert a == b, f"{kind} {nm}: batched run differs from the per-sequence drop-in"
        assert len(a) > 0


# ------------------------------------------------------------------ host state write-back
@pytest.mark.parametrize("kind", ["bytetrack", "botsort", "ocsort", "boosttrack", "strongsort"])
def test_state_set_vs_oracle(torch_cuda, kind):
    """bx_*_state_set_host: host code edits the Kalman mean / covariance of some live tracks
    between frames (what the reference's occlusion handler does to Track.mean / .covariance,
    utils/occlusion_handler.py:380-398); the same edit on the oracle, outputs bitwise after."""
    from boxmot_amd.synth import SyntheticScene

    emb = {"botsort": 32, "boosttrack": 32, "strongsort": 32}.get(kind, 0)
    args = {"bytetrack": dict(min_conf=0.1, track_thresh=0.6, match_thresh=0.9, track_buffer=30),
            "botsort": dict(track_high_thresh=0.6, new_track_thresh=0.7, match_thresh=0.8),
            "ocsort": dict(OCS_ARGS), "boosttrack": dict(BOOST_ARGS),
            "strongsort": dict(SS_ARGS)}[kind]
    tr = make_dropin(kind, {k: v for k, v in args.items() if k != "born_confirmed"})
    orc = po.OracleTracker(kind, **args)
    sc = SyntheticScene(n_obj=36, seed=77, emb_dim=emb, layout="crowded",
                        emb_dtype=np.float64 if kind in ("boosttrack", "strongsort") else np.float32,
                        conf_lo=0.3 if kind in ("ocsort", "boosttrack", "strongsort") else 0.65)
    img = np.zeros((1080, 1920, 3), np.uint8)
    ncol = 10 if kind == "strongsort" else 8
    edits = 0
    for t in range(1, 36):
        d, e, _ = sc.frame(t)
        o = tr.update(d, img, e) if emb else tr.update(d, img)
        o = np.asarray(o, np.float64).reshape(-1, ncol)
        np.testing.assert_array_equal(o, orc.update(d, e).reshape(-1, ncol), err_msg=f"frame {t}")
        if t in (10, 18, 25):
            g = tr.engine.tracks(0)
            a, b = (g["x"], g["P"]) if kind in ("ocsort", "boosttrack") else (g["mean"],
                                                                                g["covariance"])
            sel = np.arange(0, len(g["id"]), 3)
            ids, a, b = g["id"][sel], a[sel].copy(), b[sel].copy()
            a[:, 0] += 3.25
            a[:, 1] -= 1.5
            b[:, :4, :4] *= 1.5
            if t == 18:  # mean only: the covariance (and its pending predicts) stay
                b = None
            tr.engine.state_set(0, ids, a, b)
            orc.state_set(ids, a, b)
            edits += len(ids)
    assert edits > 0
    with pytest.raises(ValueError):
        tr.engine.state_set(0, [10 ** 6], np.zeros((1, 7 if kind == "ocsort" else 8)))


def gpu_legacy_lap_pair(torch, cost):
    from boxmot_amd import _native as N

    nr, nc = cost.shape
    c = dev(torch, np.ascontiguousarray(cost, np.float64))
    k = max(min(nr, nc), 1)
    a = torch.full((2 * k,), -7, dtype=torch.int32, device="cuda")
    b = torch.full((2 * k,), -7, dtype=torch.int32, device="cuda")
    info = torch.zeros(3, dtype=torch.int32, device="cuda")
    N.check(N.load().bx_legacy_lap_pair(c.data_ptr(), nr, nc, a.data_ptr(), b.data_ptr(),
                                        info.data_ptr(), None), "bx_legacy_lap_pair")
    torch.cuda.synchronize()
    na, nb, ran = (int(v) for v in host(info))
    return host(a)[: 2 * na].reshape(-1, 2), host(b)[: 2 * nb].reshape(-1, 2), bool(ran)


@pytest.mark.gpu
def test_legacy_lap_ssp_equals_lapjv_op_level(torch_cuda):
    """legacy_lap_ssp (scipy-order SSP + the tight-graph uniqueness certificate, lapjv only on a
    tie; bx_jv.h lsap_unique64) against legacy_lap (lapx's lapjv order) on the same matrices, and
    both against the oracle's lapx restatement (association.py:109's extend_cost lapjv):
    random, exact duplicate rows / columns, duplicates 1e-12 apart (inside the certificate's
    1e-9 tolerance), nr != nc both ways, +inf and NaN entries.  Random problems with nr <= nc
    must mostly certify (no lapjv; with nr > nc the real rows left on the zero padding form
    dummy-column cycles, which the certificate conservatively counts as ties), exact duplicates
    must fall back."""
    rng = np.random.default_rng(61)
    certified = eligible = fell_back = 0
    for t in range(240):
        nr, nc = int(rng.integers(1, 65)), int(rng.integers(1, 65))
        c = rng.uniform(-1.0, 1.0, (nr, nc))
        kind = t % 8
        if kind == 1 and nr > 1:
            c[1] = c[0]                      # exact duplicate row
        elif kind == 2 and nc > 1:
            c[:, -1] = c[:, 0]               # exact duplicate column
        elif kind == 3 and nr > 1:
            c[-1] = c[0] + 1e-12             # near-duplicate row
        elif kind == 4:
            c = np.round(c, 1)               # coarse grid: many ties
        elif kind == 5:
            c[rng.random((nr, nc)) < 0.1] = np.inf
        elif kind == 6:
            c[rng.random((nr, nc)) < 0.05] = np.nan
        a, b, ran = gpu_legacy_lap_pair(torch_cuda, c)
        np.testing.assert_array_equal(b, a, err_msg=f"t={t} kind={kind} {nr}x{nc}")
        if kind in (0, 7) and nr <= nc:
            eligible += 1
            certified += not ran
        if kind in (1, 2) and min(nr, nc) > 1:
            fell_back += ran
        if kind not in (5, 6):
            ox, _ = po.lapjv(c, extend_cost=True)
            ref = np.array([[i, j] for i, j in enumerate(ox[:nr]) if 0 <= j < nc],
                           np.int64).reshape(-1, 2)
            np.testing.assert_array_equal(a, ref, err_msg=f"oracle t={t} kind={kind}")
    print(f"certified {certified}/{eligible}, duplicates fell back {fell_back}")
    assert certified >= 0.8 * eligible and eligible >= 10, (certified, eligible)
    assert fell_back >= 1, fell_back


def gpu_ss_lsap(torch, cost, max_d, fast):
    from boxmot_amd import _native as N

    R, CC = cost.shape
    c = dev(torch, np.ascontiguousarray(cost, np.float64))
    rows = torch.full((R,), -7, dtype=torch.int32, device="cuda")
    cols = torch.full((R,), -7, dtype=torch.int32, device="cuda")
    info = torch.zeros(2, dtype=torch.int32, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    N.check(N.load().bx_ss_lsap_op(c.data_ptr(), R, CC, float(max_d), int(fast), rows.data_ptr(),
                                   cols.data_ptr(), info.data_ptr(), st.data_ptr(), None),
            "bx_ss_lsap_op")
    torch.cuda.synchronize()
    assert int(host(st)[0]) == 0
    np_, fs = (int(v) for v in host(info))
    if np_ < 0:
        return None, fs
    return np.stack([host(rows)[:np_], host(cols)[:np_]], 1), fs


@pytest.mark.gpu
def test_strongsort_lsap_solve_certify_vs_scipy(torch_cuda):
    """The match kernel's LSAP op-level (bx_ss_lsap_op) on min_cost_matching-shaped costs
    (linear_assignment.py:62-70: entries above max_distance clamped to max_distance + 1e-5,
    then linear_sum_assignment): scipy's row order (fast = 0) returns the oracle's pairs
    (scipy restated, pinned by test_oracle) bit for bit on every matrix, ties included.  Solve +
    certify (fast = 1) must either return the same pairs (stat 0: unique), the same pairs where
    the cost is <= max_distance (stat 1: other optima differ in rejected pairs only), or report a
    tie (-1) — never a different accepted match.  Random, sparse-real (most entries clamped:
    the cascade's shape), duplicated rows and coarse-grid (tie-heavy) matrices, R <= CC up to
    1024 columns."""
    rng = np.random.default_rng(2024)
    stats = {0: 0, 1: 0, 2: 0}
    for t in range(150):
        R = int(rng.integers(1, 200))
        CC = int(min(1024, R + rng.integers(0, 300)))
        if t % 25 == 0:
            R, CC = int(rng.integers(300, 700)), 1024
        max_d = 0.2 + 0.3 * rng.random()
        kind = t % 5
        c = rng.uniform(0.0, 1.0, (R, CC))
        if kind == 1:  # sparse real entries: a few candidates per row
            c = np.full((R, CC), 5.0)
            for r in range(R):
                k = int(rng.integers(0, 4))
                c[r, rng.choice(CC, k, replace=False)] = rng.uniform(0, max_d, k)
        elif kind == 2 and R > 1:
            c[R // 2] = c[0]
        elif kind == 3:
            c = np.round(c * 4) / 4
        c = np.where(c > max_d, max_d + 1e-5, c)
        rr, kk = po.lsap(c)
        ref = np.stack([rr, kk], 1).astype(np.int64)
        ex, fs0 = gpu_ss_lsap(torch_cuda, c, max_d, False)
        np.testing.assert_array_equal(ex, ref, err_msg=f"exact t={t} kind={kind} {R}x{CC}")
        assert fs0 == 0
        got, fs = gpu_ss_lsap(torch_cuda, c, max_d, True)
        stats[fs] += 1
        if fs == 2:
            assert got is None
            continue
        if fs == 0:
            np.testing.assert_array_equal(got, ref, err_msg=f"fast t={t} kind={kind}")
        real = lambda p: p[c[p[:, 0], p[:, 1]] <= max_d]  # noqa: E731
        np.testing.assert_array_equal(real(got), real(ref), err_msg=f"fast real t={t} k={kind}")
    print(f"solve + certify outcomes: {stats}")
    assert stats[0] + stats[1] >= 75 and stats[2] >= 3, stats
