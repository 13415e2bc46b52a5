"""Summarise tools/pmc.sh output: mean counter value per dispatch of the fused kernel."""
import csv
import glob
import sys

d = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "informer_forward"
vals = {}
for f in sorted(glob.glob(f"{d}/p*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in vals.items():
    print(f"{k:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")
