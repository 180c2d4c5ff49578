"""dev: print ms/step and stage probes of gpurun_out/<cfg>_<variant>.json lines"""
import json, sys
cfg = sys.argv[1]
for v in sys.argv[2:]:
    try:
        d = json.loads(open(f"gpurun_out/{cfg}_{v}.json").read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(v, "missing", e); continue
    r = d["roofline"]
    print(f"{v:12s} {d['value']:>12} {d['ms_per_step']:.4f} ms", {k: round(x, 3) for k, x in r["stage_ms_probe"].items()})
