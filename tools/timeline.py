#!/usr/bin/env python
"""Per-step kernel timeline of a rocprofv3 --kernel-trace CSV (engine kernels only): for the last
`n` frames, each kernel's start offset from the frame's first kernel and its duration (us), then
the average over those frames — shows which kernels overlap (fork-join) and the critical path.

Usage: python tools/timeline.py <trace dir> [first kernel name of a frame] [n]"""
import collections
import csv
import glob
import sys


def main(d, first="det_feature_kernel", n=10):
    rows = []
    for f in glob.glob(f"{d}/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "anonymous namespace)::" not in k or "at::" in k:
                continue
            name = k.split("::")[1].split("(")[0].split("<")[0]
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2] == first]
    frames = []
    for a, b in zip(starts, starts[1:] + [len(rows)]):
        frames.append(rows[a:b])
    frames = frames[-n - 1:-1]  # complete frames only
    acc = collections.defaultdict(lambda: [0.0, 0.0, 0.0, 0])
    spans = []
    for fr in frames:
        t0 = fr[0][0]
        spans.append((max(r[1] for r in fr) - t0) / 1e3)
        for s, e, name in fr:
            a = acc[name]
            a[0] += (s - t0) / 1e3
            a[1] += (e - t0) / 1e3
            a[2] += (e - s) / 1e3
            a[3] += 1
    print(f"{d}: {len(frames)} frames, kernel span per frame {sum(spans) / len(spans):.1f} us")
    for name, (s, e, dur, c) in sorted(acc.items(), key=lambda kv: kv[1][0]):
        print(f"  {name:28s} start {s / c:8.1f}  end {e / c:8.1f}  dur {dur / c:8.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []), *(int(x) for x in sys.argv[3:4]))
