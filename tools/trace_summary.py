"""Steady-state kernel times from a rocprofv3 --kernel-trace of bench.py, beside the bench's own
HIP-event stage times from the same lease ("Reproducing the roofline").

rocprofv3 --stats averages EVERY launch of a kernel, the warm-up steps included; the first step
touches freshly allocated buffers and runs slower.  This summary also averages the launches of the
timed window only: a kernel launched c times per step has (W + K + E) * c launches in the trace
(W warm-up steps, K timed steps, E = 6 end-to-end steps after them), and the first W * c are
dropped.

Usage: python tools/trace_summary.py KERNEL_TRACE.csv BENCH_LINE.json OUT.json [--warmup W --steps K --extra E]
"""

import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("out")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--extra", type=int, default=6)
    a = ap.parse_args()
    runs = defaultdict(list)
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"].replace("void ", "").split("(")[0].strip()
            runs[name].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    per_step = a.warmup + a.steps + a.extra
    rows = {}
    for name, v in runs.items():
        v.sort()
        d = [(e - s) / 1e6 for s, e in v]
        c = len(d) / per_step
        rec = {"launches": len(d), "avg_all_ms": sum(d) / len(d), "min_ms": min(d), "max_ms": max(d)}
        if c >= 1 and abs(c - round(c)) < 1e-9:
            c = int(round(c))
            w = d[a.warmup * c:]
            rec.update({"per_step": c, "avg_steady_ms": sum(w) / len(w), "first_ms": d[0],
                        "ms_per_step_steady": sum(w) / len(w) * c})
        rows[name] = rec
    with open(a.bench) as fh:
        line = json.loads(fh.read().strip().splitlines()[-1])
    stages = line["roofline"].get("stages", {})
    out = {"_bench": {"ms_per_step": line["ms_per_step"], "roofline_kernel": line["roofline"]["kernel"],
                      "roofline_avg_launch_ms": line["roofline"]["avg_launch_ms"], "frac": line["roofline"]["frac"],
                      "stages_ms_per_launch": {k: v["ms_per_launch"] for k, v in stages.items()}},
           "_method": __doc__.split("\n\n")[1].replace("\n", " "),
           "kernels": dict(sorted(rows.items(), key=lambda kv: -kv[1].get("ms_per_step_steady", 0)))}
    top = [k for k, v in out["kernels"].items() if "ms_per_step_steady" in v][:1]
    out["_dominant_by_trace"] = top[0] if top else None
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"bench: {line['ms_per_step']} ms/step; roofline kernel {line['roofline']['kernel'][:60]} "
          f"avg {line['roofline']['avg_launch_ms']} ms")
    for k, v in list(out["kernels"].items())[:12]:
        if "ms_per_step_steady" in v:
            print(f"  {v['ms_per_step_steady']:8.3f} ms/step  x{v['per_step']}  steady {v['avg_steady_ms']:8.3f}  "
                  f"all {v['avg_all_ms']:8.3f}  first {v['first_ms']:8.3f}  {k[:90]}")


if __name__ == "__main__":
    main()
