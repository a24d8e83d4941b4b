"""One line per world size of a tools/range_emulate.py output (other stdout lines, e.g. RCCL's banner, skipped)."""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "world" not in d:
        print(f"scheme {d['scheme']} config {d['config']} single {d['single_gpu_ms']} ms")
        continue
    st = d.get("slowest_rank_stages_ms") or {}
    print(d["world"], d["max_rank_ms"], f"{d['speedup_vs_single']}x", json.dumps(st))
