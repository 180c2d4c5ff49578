import os, sys, time
import numpy as np
sys.path.insert(0, os.getcwd())
import torch
from boxmot_amd.synth import SyntheticScene
from boxmot_amd.tracker_zoo import create_tracker
from boxmot_amd.engine import Engine, EngineParams
import bench
kind, n_obj, F, params = bench.CONFIGS["botsort"]
sc = SyntheticScene(n_obj=n_obj, seed=777, emb_dim=F)
frames = [sc.frame(t) for t in range(1, 261)]
img = np.zeros((1080, 1920, 3), np.uint8)
tr = create_tracker("botsort", evolve_param_dict=params)
for d, e, _ in frames[:30]: tr.update(d, img, e)
t0 = time.perf_counter()
for d, e, _ in frames[30:]: tr.update(d, img, e)
print("tracker.update ms", (time.perf_counter() - t0) / 230 * 1e3)
eng = Engine("botsort", n_seq=1, track_cap=1024, det_cap=384, emb_dim=F, params=EngineParams(**params))
for d, e, _ in frames[:30]: eng.update_host(0, d, e)
t0 = time.perf_counter()
for d, e, _ in frames[30:]: eng.update_host(0, d, e)
print("engine.update_host ms", (time.perf_counter() - t0) / 230 * 1e3)
eng2 = Engine("botsort", n_seq=1, track_cap=1024, det_cap=384, emb_dim=F, params=EngineParams(**params))
dev = [(torch.from_numpy(d.astype(np.float32)).cuda(), torch.tensor([0, d.shape[0]], dtype=torch.int32).cuda(), torch.from_numpy(e).cuda()) for d, e, _ in frames]
out = torch.empty((400, 8), dtype=torch.float64, device="cuda"); cnt = torch.empty(1, dtype=torch.int32, device="cuda")
for d, o, e in dev[:30]: eng2.step(d, o, e, None, out, cnt)
torch.cuda.synchronize()
t0 = time.perf_counter()
for d, o, e in dev[30:]:
    eng2.step(d, o, e, None, out, cnt); torch.cuda.synchronize()
print("engine.step+sync ms", (time.perf_counter() - t0) / 230 * 1e3)
t0 = time.perf_counter()
for d, o, e in dev[30:]:
    eng2.step(d, o, e, None, out, cnt)
torch.cuda.synchronize()
print("engine.step pipelined ms", (time.perf_counter() - t0) / 230 * 1e3)
import cProfile, pstats
pr = cProfile.Profile(); pr.enable()
for d, e, _ in frames[30:130]: tr.update(d, img, e)
pr.disable(); pstats.Stats(pr).sort_stats("tottime").print_stats(12)
