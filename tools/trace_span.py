"""Union span of concurrent kernel launches per bench step, from a rocprofv3 kernel trace.

bench.py runs the three environment segments as concurrent launches (carmpc_solve_segments
forks them onto side streams); each launch then lasts the whole step, so rocprof's per-launch
average is not the step time.  This groups the dominant kernel's launches by start time
(launches of one step start within `--gap-ms` of each other) and reports each group's union
span [min start, max end], to compare with bench.py's roofline.kernel_ms_per_step.

    python tools/trace_span.py gpurun_out/prof/run_kernel_trace.csv --match ipm_riccati
"""
import argparse
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--match", default="ipm_riccati_kernel")
ap.add_argument("--gap-ms", type=float, default=1.0)
ap.add_argument("--skip", type=int, default=3, help="leading groups to drop (warm-up steps)")
ap.add_argument("--out", default=None)
args = ap.parse_args()

rows = [r for r in csv.DictReader(open(args.trace)) if args.match in r["Kernel_Name"]]
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
groups, cur = [], []
for s, e in ev:
    if cur and (s - cur[0][0]) > args.gap_ms * 1e6:
        groups.append(cur)
        cur = []
    cur.append((s, e))
if cur:
    groups.append(cur)
# steps are the groups with the full launch count (drops e.g. single launches outside the loop)
full = max(len(g) for g in groups)
groups = [g for g in groups if len(g) == full]
spans = [(max(e for _, e in g) - min(s for s, _ in g)) / 1e6 for g in groups]
per_launch = [[(e - s) / 1e6 for s, e in g] for g in groups]
timed = spans[args.skip:]
out = {"kernel": args.match, "launches_per_step": [len(g) for g in groups], "span_ms": [round(x, 4) for x in spans],
       "per_launch_ms": [[round(x, 4) for x in g] for g in per_launch],
       "timed_steps": len(timed), "mean_span_ms_timed": round(sum(timed) / max(len(timed), 1), 4)}
print(json.dumps(out, indent=1))
if args.out:
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
