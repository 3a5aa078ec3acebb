"""Sum rocprofv3 --pmc counter_collection.csv files per kernel: python tools/sum_counters.py <dir>..."""
import csv
import glob
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]
            tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", kv[1].get("SQ_BUSY_CYCLES", 0))):
    wc = c.get("SQ_WAVE_CYCLES", 0)
    print(k)
    for n, v in sorted(c.items()):
        extra = f"  ({v / wc:.3f} of wave cycles)" if wc and n.startswith("SQ_WAIT") or n == "SQ_ACTIVE_INST_ANY" and wc else ""
        print(f"   {n:28s} {v:16.4g}{extra}")
