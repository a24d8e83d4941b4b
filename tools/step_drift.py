"""Per-step wall time of the C3 step over many steps (does the first timed step run slower than
later ones, e.g. while clocks settle?).  Tuning only: python tools/step_drift.py [steps]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))


def main():
    from genome_kmers import _native, synthetic

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    sba, seg = synthetic.c3_genome(3_100_000_000, 42)
    e = _native.Engine(0)
    e.set_sequence(sba, seg)
    e.sync()
    out = []
    for i in range(steps):
        e.sync()
        t0 = time.perf_counter()
        e.enumerate(31)
        e.sort(31)
        e.materialize_keys()
        e.unique_count_only()
        e.sync()
        out.append((time.perf_counter() - t0) * 1e3)
        print(f"step {i}: {out[-1]:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
