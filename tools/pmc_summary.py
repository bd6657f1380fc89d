"""Average PMC counter values per kernel (regex on the kernel name) over rocprofv3 csv files.
  python tools/pmc_summary.py 'mha_bwd' gpurun_out/pmcm1/pmcm1_counter_collection.csv ..."""
import collections
import csv
import re
import sys

pat = re.compile(sys.argv[1])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[2:]:
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        m = pat.search(k)
        if not m:
            continue
        name = re.sub(r"\(.*", "", k.replace("(anonymous namespace)::", ""))[:60]
        agg[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("   %-28s %14.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))
