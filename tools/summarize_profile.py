#!/usr/bin/env python
"""Summarise a tools/profile_round.sh run into profiles/<tag>_<config>.md and
profiles/pmc_<config>.json (read by bench.py for roofline.traffic).

HBM bytes per frame-kernel launch follow MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7:
FETCH_SIZE and WRITE_SIZE are KiB (bytes = value * 1024), collected in separate passes; on gfx950
FETCH_SIZE reads exactly half the bytes of a wide coalesced streaming read, so the corrected read
side is 2 x FETCH_SIZE.  The frame kernel mixes access widths (16-B feature rows, 8-B SoA state,
scattered LDS-miss reads), so both the raw and the corrected figures are recorded.
"""
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def rows(p):
    with open(p) as f:
        return list(csv.DictReader(f))


def main(tag, config, warmup=10):
    base = ROOT / "gpurun_out" / f"prof_{tag}_{config}"
    trace = [r for r in rows(base / "trace" / "run_kernel_trace.csv")
             if "frame_kernel" in r["Kernel_Name"]]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in trace]
    timed = durs[warmup:]
    stats = rows(base / "trace" / "run_kernel_stats.csv")

    def pmc(kind, name):
        vals = [float(r["Counter_Value"]) for r in rows(base / kind / "run_counter_collection.csv")
                if "frame_kernel" in r["Kernel_Name"] and r["Counter_Name"] == name]
        vals = vals[warmup:]
        return sum(vals) / len(vals) if vals else None

    fetch_kb, write_kb = pmc("fetch", "FETCH_SIZE"), pmc("write", "WRITE_SIZE")
    bench_line = None
    for ln in (base / "bench_traced.log").read_text().splitlines():
        if ln.startswith("{"):
            bench_line = json.loads(ln)
    raw = (fetch_kb + write_kb) * 1024 if fetch_kb is not None else None
    corr = (2 * fetch_kb + write_kb) * 1024 if fetch_kb is not None else None
    summary = {
        "tag": tag, "config": config,
        "frame_kernel_launches": len(trace), "timed_launches": len(timed),
        "rocprof_avg_ms_timed": sum(timed) / len(timed),
        "bench_hip_event_kernel_ms_traced_run": bench_line["roofline"]["kernel_ms"] if bench_line else None,
        "fetch_size_kb_per_launch": fetch_kb, "write_size_kb_per_launch": write_kb,
        "hbm_bytes_per_launch_raw": raw, "hbm_bytes_per_launch_corrected": corr,
        "algorithmic_bytes_per_launch": bench_line["roofline"]["algorithmic_bytes_per_launch"] if bench_line else None,
        "vgpr": trace[0]["VGPR_Count"] if trace and "VGPR_Count" in trace[0] else None,
    }
    (ROOT / "profiles" / f"pmc_{config}.json").write_text(json.dumps(summary, indent=1))
    md = [f"# rocprofv3 summary — {tag} / {config}", "",
          "Command: `bash tools/profile_round.sh " + f"{tag} {config}` (bench.py --config {config} "
          f"--steps 30 --warmup 10, kernel trace + stats pass; FETCH_SIZE and WRITE_SIZE passes)", "",
          "## Kernel stats (rocprofv3 --stats, all dispatches of the traced run)", "",
          "| kernel | calls | avg ms | % |", "|---|---|---|---|"]
    for r in stats[:8]:
        md.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.4f} | "
                  f"{float(r['Percentage']):.1f} |")
    md += ["", "## Frame kernel", ""]
    for k, v in summary.items():
        md.append(f"- {k}: {v}")
    (ROOT / "profiles" / f"{tag}_{config}.md").write_text("\n".join(md) + "\n")
    print("\n".join(md))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
