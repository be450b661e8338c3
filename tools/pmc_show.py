"""Mean counter values per kernel from rocprofv3 --pmc CSV output: python tools/pmc_show.py DIR [substr]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if sub in k:
        acc[(k.split("(")[0][:50], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print("%-50s %-28s n=%3d mean=%.4g" % (k, c, len(v), sum(v) / len(v)))
