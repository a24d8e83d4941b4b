"""Per-kernel summary of a rocprofv3 --pmc counter CSV (averages per launch; SQ cycle counters
are quad-cycles on gfx950, reported here as fractions of SQ_WAVE_CYCLES)."""
import csv
import sys
from collections import defaultdict


def main(path):
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for k, d in acc.items():
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        rows.append((avg.get("SQ_WAVE_CYCLES", 0), k, avg, len(next(iter(d.values())))))
    for wc, k, avg, n in sorted(rows, reverse=True)[:14]:
        fr = {c.replace("SQ_", "").lower(): (v / wc if ("CYCLES" in c or "WAIT" in c or "ACTIVE" in c) and not c.startswith("SQ_LDS") else v)
              for c, v in avg.items() if c != "SQ_WAVE_CYCLES" and wc}
        txt = "  ".join(f"{c}={v:.3g}" for c, v in sorted(fr.items()))
        print(f"{k[:48]:48s} n={n:<3d} wave_cycles={wc:.3g}  {txt}")


if __name__ == "__main__":
    main(sys.argv[1])
