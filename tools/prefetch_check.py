"""Debug aid: the sort of a single-contig random genome with and without the sort hint (prefetched
L0), compared start by start.  Usage: python tools/prefetch_check.py L [L ...]"""

import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genome-kmers_amd"))


def main():
    from genome_kmers import _native, synthetic

    k = 31
    for L in [int(x) for x in sys.argv[1:]]:
        sba, seg = synthetic.c3_genome(L, 42)
        outs = []
        for hint in (0, k):
            eng = _native.Engine(0)
            eng.sort_hint(hint)
            eng.profile_enable(True)
            t0 = time.perf_counter()
            eng.set_sequence(sba, seg)
            n = eng.enumerate(k)
            eng.sort(k)
            eng.sync()
            dt = time.perf_counter() - t0
            rep = eng.profile_report()
            outs.append(eng.copy_starts(np.empty(n, dtype=np.uint32)))
            print(f"L={L:,} hint={hint} n={n:,} {dt * 1e3:.1f} ms prefetch_l0={'prefetch_l0' in rep} "
                  f"max={int(outs[-1].max()):,}", flush=True)
            del eng
        a, b = outs
        bad = np.flatnonzero(a != b)
        print(f"L={L:,}: {len(bad):,} differing positions" +
              (f", first at {bad[0]:,} (plain {a[bad[0]]}, hint {b[bad[0]]}), last {bad[-1]:,}" if len(bad) else ""),
              flush=True)


if __name__ == "__main__":
    main()
