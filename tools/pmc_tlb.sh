# Address-translation counters per kernel (round 5: are the box-to-box differences of the scattered
# passes translation misses?): one unprofiled C3 bench line to place the box, then one --pmc pass
# of the UTCL1 hit / miss / request counts and UTCL2 busy over a 2-step bench.
#   bash tools/pmc_tlb.sh TAG  -> gpurun_out/tlb_TAG/
set -o pipefail
O=gpurun_out/tlb_${1:-box}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-boundary \
  > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 tools/line_brief.py $O/bench.json
timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum \
  GRBM_UTCL2_BUSY -d $O/pmc -o run --output-format csv -- python3 bench.py --config c3 --steps 2 --warmup 1 \
  --no-cpu-baseline --no-boundary > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 - "$(find $O/pmc -name '*counter_collection.csv' | head -1)" > $O/pmc_summary.txt <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"].split("(")[0].replace("void ", "").strip()][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = sorted(((sum(d.get("TCP_UTCL1_REQUEST_sum", [0])) / max(1, len(d.get("TCP_UTCL1_REQUEST_sum", [0]))), k, d)
               for k, d in acc.items()), key=lambda t: -t[0])
print("kernel, per launch: UTCL1 requests, hits, misses, miss rate, UTCL2 busy")
for req, k, d in rows[:12]:
    av = {c: sum(v) / len(v) for c, v in d.items()}
    hit, miss = av.get("TCP_UTCL1_TRANSLATION_HIT_sum", 0), av.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0)
    print(f"{k[:60]:60s} req {req:.4g}  hit {hit:.4g}  miss {miss:.4g}  rate {miss / max(hit + miss, 1):.4f}  "
          f"utcl2_busy {av.get('GRBM_UTCL2_BUSY', 0):.4g}")
PY
rm -rf $O/pmc
head -30 $O/pmc_summary.txt
