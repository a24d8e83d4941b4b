"""Steady-state kernel times from a rocprofv3 --kernel-trace of bench.py, beside the bench's own
HIP-event stage times from the same lease ("Reproducing the roofline").

rocprofv3 --stats averages EVERY launch of a kernel: the warm-up steps, and the end-to-end steps the
bench runs after its timed ones.  This summary cuts the trace into steps instead: every step of the
C3 sort starts with exactly one launch of the L0 count kernel (msd0_count_kernel), so step i spans
from the i-th such launch to the next one.  The timed steps are W .. W + K - 1 (W warm-up steps
first); each kernel's launches inside them give its mean duration and its time per step.  The bench's
device stage times (HIP events on the engine's stream) are printed beside them.  The transfers' own
kernels (unpack_chunk_kernel, runtime copy kernels) are left out.

Usage: python tools/trace_summary.py KERNEL_TRACE.csv BENCH_LINE.json OUT.json [--warmup W --steps K]
"""

import argparse
import csv
import json
from bisect import bisect_right
from collections import defaultdict

MARK = "msd0_count_kernel"
SKIP = ("unpack_chunk_kernel", "__amd_rocclr")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("out")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"].replace("void ", "").split("(")[0].strip()
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    marks = [s for s, _, n in rows if MARK in n]
    W, K = a.warmup, a.steps
    if len(marks) < W + K:
        raise SystemExit(f"{len(marks)} step markers ({MARK}) for {W} + {K} steps")
    lo = marks[W]
    hi = marks[W + K] if len(marks) > W + K else float("inf")
    per = defaultdict(list)
    for s, e, n in rows:
        if lo <= s < hi and not any(x in n for x in SKIP):
            per[n].append((e - s) / 1e6)
    step_of = lambda s: bisect_right(marks, s) - 1  # noqa: E731
    kern = {}
    for n, d in per.items():
        kern[n] = {"launches_in_window": len(d), "per_step": round(len(d) / K, 2), "avg_ms": sum(d) / len(d),
                   "ms_per_step": sum(d) / K, "min_ms": min(d), "max_ms": max(d)}
    with open(a.bench) as fh:
        line = json.loads(fh.read().strip().splitlines()[-1])
    stages = line["roofline"].get("stages", {})
    # the timed steps run back to back: the marker period over them (the last step's end is not marked)
    period_ms = (marks[W + K - 1] - marks[W]) / 1e6 / max(K - 1, 1)
    out = {"_bench": {"ms_per_step": line["ms_per_step"], "roofline_kernel": line["roofline"]["kernel"],
                      "roofline_avg_launch_ms": line["roofline"]["avg_launch_ms"], "frac": line["roofline"]["frac"],
                      "stages_ms_per_launch": {k: v["ms_per_launch"] for k, v in stages.items()}},
           "_trace_window": {"steps": K, "first_step": W, "step_period_ms": round(period_ms, 3),
                             "first_marker_step": step_of(lo)},
           "_method": __doc__.split("\n\n")[1].replace("\n", " "),
           "kernels": dict(sorted(kern.items(), key=lambda kv: -kv[1]["ms_per_step"]))}
    top = next(iter(out["kernels"]), None)
    out["_dominant_by_trace"] = top
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"bench (unprofiled): {line['ms_per_step']} ms/step; roofline kernel "
          f"{line['roofline']['kernel'][:70]} avg {line['roofline']['avg_launch_ms']} ms")
    print(f"trace (profiled): steps {W}..{W + K - 1}: one step every {period_ms:.3f} ms (L0-count markers)")
    for k, v in list(out["kernels"].items())[:12]:
        print(f"  {v['ms_per_step']:8.3f} ms/step  x{v['per_step']:<5} avg {v['avg_ms']:8.3f}  {k[:90]}")


if __name__ == "__main__":
    main()
