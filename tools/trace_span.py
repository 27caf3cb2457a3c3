"""Union span of concurrent kernel launches per bench step, from a rocprofv3 kernel trace.

bench.py runs the three environment segments as concurrent launches (carmpc_solve_segments
forks them onto side streams); each launch then lasts the whole step, so rocprof's per-launch
average is not the step time.  This groups the dominant kernel's launches by dispatch order
(`--per-step` launches per step) and reports each step's union span [min start, max end], to
compare with bench.py's roofline.kernel_ms_per_step.

    python tools/trace_span.py gpurun_out/prof/run_kernel_trace.csv --skip 3 --steps 5
"""
import argparse
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--match", default="ipm_riccati_kernel")
ap.add_argument("--per-step", type=int, default=3, help="launches per bench step (environment segments)")
ap.add_argument("--steps", type=int, default=None, help="timed steps after --skip (default: all but the last group)")
ap.add_argument("--skip", type=int, default=3, help="leading groups to drop (warm-up steps)")
ap.add_argument("--out", default=None)
args = ap.parse_args()

rows = [r for r in csv.DictReader(open(args.trace)) if args.match in r["Kernel_Name"]]
# steps in dispatch order: bench.py issues `per_step` launches per step (one per environment
# segment), --skip warm-up steps first, then the timed steps, then the end-to-end step
rows.sort(key=lambda r: int(r["Dispatch_Id"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
groups = [ev[i:i + args.per_step] for i in range(0, len(ev) - args.per_step + 1, args.per_step)]
spans = [(max(e for _, e in g) - min(s for s, _ in g)) / 1e6 for g in groups]
per_launch = [[(e - s) / 1e6 for s, e in g] for g in groups]
stop = args.skip + args.steps if args.steps is not None else len(spans) - 1
timed = spans[args.skip:stop]
timed_launches = [x for g in per_launch[args.skip:stop] for x in g]
out = {"kernel": args.match, "launches_per_step": [len(g) for g in groups], "span_ms": [round(x, 4) for x in spans],
       "mean_launch_ms_timed": round(sum(timed_launches) / max(len(timed_launches), 1), 4),
       "per_launch_ms": [[round(x, 4) for x in g] for g in per_launch],
       "timed_steps": len(timed), "mean_span_ms_timed": round(sum(timed) / max(len(timed), 1), 4)}
print(json.dumps(out, indent=1))
if args.out:
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
