"""Per-kernel mean of every counter in a rocprofv3 --pmc counter_collection.csv (the 10 kernels
with the most of the first counter), one line each."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
names = []
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
    c = r["Counter_Name"]
    if c not in names:
        names.append(c)
    acc[k][c].append(float(r["Counter_Value"]))
first = names[0] if names else None
rows = sorted(acc.items(), key=lambda kv: -(sum(kv[1].get(first, [0])) / max(1, len(kv[1].get(first, [0])))))
print("kernel (per launch): " + ", ".join(names))
for k, d in rows[:10]:
    print(f"{k[:64]:64s} " + "  ".join(f"{n}={sum(d.get(n, [0])) / max(1, len(d.get(n, [0]))):.4g}" for n in names))
