"""Stage times of the C3 step (or a prefix) for timing experiments: no self-check, so library
variants with wrong output (GKM_EXP_* switches) can be timed.  Usage:
  python tools/exp_stages.py [--config c3|c4|c5] [--genome-len L] [--steps S] [--label X]
(env selects the variant; c4 / c5: the GRCh38 surrogate, c5 canonical k = 63)"""

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))

from genome_kmers import _native, synthetic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", choices=("c3", "c4", "c5"), default="c3")
ap.add_argument("--genome-len", type=int, default=3_100_000_000)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--k", type=int, default=None)
ap.add_argument("--label", default="")
a = ap.parse_args()
sba, seg = synthetic.c3_genome(a.genome_len, 42) if a.config == "c3" else synthetic.grch38_surrogate(2)
k = a.k or (63 if a.config == "c5" else 31)
canonical = a.config == "c5"
eng = _native.Engine()
eng.set_sequence(sba, seg)
eng.sync()


def step():
    eng.enumerate(k)
    eng.sort(k, canonical=canonical)
    eng.materialize_keys()
    return eng.unique_count_only()


step()
eng.sync()
eng.profile_enable(True)
t0 = time.perf_counter()
for _ in range(a.steps):
    step()
eng.sync()
dt = (time.perf_counter() - t0) / a.steps
rep = eng.profile_report()
stages = {k: round(v["total_ms"] / a.steps, 3) for k, v in rep.items() if v["total_ms"] / a.steps > 0.3}
print(json.dumps({"label": a.label, "ms_per_step": round(dt * 1e3, 2), "stages": stages}), flush=True)
