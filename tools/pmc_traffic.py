"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs into per-launch HBM bytes per kernel.

Usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv OUT.json [--label TEXT]

Counter convention (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts exactly half the bytes of a wide coalesced streaming read, so the read
side is doubled.  Calibration in this repo: alphabet_kernel streams the 3.1 GB sequence byte array
with 16-B loads and reports FETCH_SIZE x 1024 x 2 = 3.1 GB (profiles/r1/README.md).
"""

import csv
import json
import sys
from collections import defaultdict


def per_kernel(path):
    acc = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            acc[name].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch, write, out = sys.argv[1:4]
    label = sys.argv[5] if len(sys.argv) > 5 and sys.argv[4] == "--label" else ""
    f, w = per_kernel(fetch), per_kernel(write)
    res = {"_label": label, "_convention": "bytes = FETCH_SIZE*1024*2 + WRITE_SIZE*1024, averaged per launch"}
    for k in sorted(set(f) | set(w)):
        fl, wl = f.get(k, [0]), w.get(k, [0])
        fk = sum(fl) / max(len(fl), 1)
        wk = sum(wl) / max(len(wl), 1)
        # the largest launch (launches pair up in order: same command, same dispatch sequence)
        per = [a * 1024 * 2 + b * 1024 for a, b in zip(fl, wl)]
        rec = {"kernel": k, "launches": max(len(fl), len(wl)),
               "fetch_bytes_per_launch": fk * 1024 * 2, "write_bytes_per_launch": wk * 1024,
               "hbm_bytes_per_launch": fk * 1024 * 2 + wk * 1024,
               "hbm_bytes_max_launch": max(per) if per else None}
        # keyed by the instantiation (template arguments, no spaces) and, for the first one of a
        # name, by the bare name
        res[k.split("::")[-1].replace(" ", "")] = rec
        res.setdefault(k.split("::")[-1].split("<")[0], rec)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, v in res.items():
        if not k.startswith("_") and "<" not in k:
            print(f"{k:28s} x{v['launches']:3d}  read {v['fetch_bytes_per_launch'] / 1e9:8.2f} GB  "
                  f"write {v['write_bytes_per_launch'] / 1e9:8.2f} GB")


if __name__ == "__main__":
    main()
