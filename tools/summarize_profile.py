#!/usr/bin/env python
"""Summarise tools/trace_only.sh + tools/pmc_passes.sh runs into profiles/<tag>_<config>.md and
profiles/pmc_<config>.json (read by bench.py for roofline.traffic, per pipeline stage).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KiB
(bytes = value * 1024), collected in separate passes; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced streaming read, so the corrected read side is 2 x FETCH_SIZE.  Both
the raw and the corrected sums are recorded.
"""
import collections
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
STAGE_OF = {"det_feature_kernel": "det_features", "predict_kernel": "predict",
            "gate_kernel": "gate", "cosine_kernel": "cosine", "cosine_kernel_any": "cosine",
            "assoc_kernel": "assoc", "update_kernel": "update",
            "cov_predict_kernel": "cov_predict", "cov_predict_gmc_kernel": "cov_predict",
            "feature_kernel": "features", "finish_kernel": "finish",
            "ocsort_frame_kernel": "ocsort_frame", "boost_embcost_kernel": "embcost",
            "boost_frame_kernel": "frame", "boost_feature_kernel": "feature",
            "ss_prep_kernel": "prep", "ss_nn_kernel": "nn", "ss_rec_kernel": "recovery",
            "ss_pre_kernel": "pre", "ss_sort_kernel": "sort", "ss_cost_kernel": "cost", "ss_match_kernel": "match",
            "ss_update_kernel": "update", "ss_post_kernel": "post", "ss_fit_kernel": "fit"}


def kname(full):
    if "anonymous namespace)::" not in full or "at::" in full:
        return None
    k = full.split("::")[1].split("(")[0]
    return k.split("<")[0]


def main(tag, config, dest=None, timed_n=50):
    tr = ROOT / "gpurun_out" / f"trace_{tag}_{config}"
    pm = ROOT / "gpurun_out" / f"pmc_{tag}_{config}"
    stats = list(csv.DictReader(open(tr / "run_kernel_stats.csv")))
    # per-kernel durations of the TIMED launches (the last `timed` of each kernel), as bench.py
    # averages them
    durs = collections.defaultdict(list)
    for r in csv.DictReader(open(tr / "run_kernel_trace.csv")):
        k = kname(r["Kernel_Name"])
        if k:
            durs[STAGE_OF.get(k, k)].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in pm.glob("*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k:
                pmc[STAGE_OF.get(k, k)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    bench = None
    for ln in (tr / "bench.log").read_text().splitlines():
        if ln.startswith("{"):
            bench = json.loads(ln)
    out = {"tag": tag, "config": config, "stages": {}}
    md = [f"# rocprofv3 summary — {tag} / {config}", "",
          f"Commands: `bash tools/trace_only.sh {tag} {config}` (rocprofv3 --kernel-trace "
          f"--stats, bench.py --steps 50 --warmup 10) and `bash tools/pmc_passes.sh {tag} "
          f"{config}` (separate --pmc passes: SQ group, FETCH_SIZE, WRITE_SIZE, misc).", "",
          "## Engine kernels (rocprofv3 --stats)", "",
          "| stage | kernel | calls | avg us (all) | avg us (timed 50) | FETCH x2 + WRITE "
          "(MB/launch) | VALU instrs (M) | active-inst frac |", "|---|---|---|---|---|---|---|---|"]
    tot = 0.0
    for r in stats:
        k = kname(r["Name"])
        if not k:
            continue
        st = STAGE_OF.get(k, k)
        us = float(r["AverageNs"]) / 1e3
        tot += us
        c = {n: sum(v) / len(v) for n, v in pmc.get(st, {}).items()}
        fetch, write = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
        corr = (2 * fetch + write) * 1024 if fetch is not None and write is not None else None
        raw = (fetch + write) * 1024 if fetch is not None and write is not None else None
        busy = (c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"]) if c.get("SQ_WAVE_CYCLES") else None
        timed = durs.get(st, [])[-timed_n:]
        tus = sum(timed) / len(timed) if timed else None
        out["stages"][st] = {"kernel": r["Name"].split("::", 1)[1].split("((")[0],
            "avg_us": us, "avg_us_timed": tus,
            "calls": int(r["Calls"]),
            "hbm_bytes_per_launch_raw": raw, "hbm_bytes_per_launch_corrected": corr,
            "valu_instrs": c.get("SQ_INSTS_VALU"), "active_inst_frac_of_wave_cycles": busy}
        md.append(f"| {st} | `{out['stages'][st]['kernel'][:48]}` | {r['Calls']} | {us:.1f} | "
                  f"{tus if tus else float('nan'):.1f} | "
                  f"{corr / 1e6 if corr else float('nan'):.1f} | "
                  f"{(c.get('SQ_INSTS_VALU') or 0) / 1e6:.1f} | "
                  f"{busy if busy is not None else float('nan'):.2f} |")
    md += ["", f"Sum of engine kernels per step: {tot:.1f} us", ""]
    if bench:
        out["bench_traced"] = {k: bench[k] for k in ("value", "ms_per_step")}
        out["bench_traced"]["roofline"] = bench["roofline"]
        md += ["## bench line of the traced run", "", "```", json.dumps(bench), "```", ""]
    dst = Path(dest) if dest else ROOT / "profiles"
    dst.mkdir(parents=True, exist_ok=True)
    (dst / f"pmc_{config}.json").write_text(json.dumps(out, indent=1))
    (dst / f"{tag}_{config}.md").write_text("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
