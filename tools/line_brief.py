"""One-line summary of a bench.py JSON line (the last line of FILE): step time, value, the roofline
kernel and fraction, end to end, and the stages above 1 ms.  Usage: line_brief.py FILE [--label X]"""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
label = sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--label" else ""
r = d.get("roofline") or {}
st = (d.get("config") or {}).get("stages_ms_per_step") or {}
print(label, d.get("ms_per_step"), f"{d.get('value', 0):.4g}", "e2e", d.get("e2e_ms"),
      "|", (r.get("kernel") or "")[:48], r.get("avg_launch_ms"), r.get("frac"),
      {k: st[k] for k in sorted(st) if st[k] > 1})
