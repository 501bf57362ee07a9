"""Per-dispatch averages of SQ counters collected by tools/pmc_sq.sh (engine kernels only)."""
import csv
import glob
import sys
from collections import defaultdict

out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "")
            if "mpcqp" not in k:
                continue
            name = next((t for t, key in (("k64", "kernel_64"), ("k96", "kernel_96"), ("k128", "kernel_128"),
                                          ("kipm", "kernel_ipm"), ("order", "order_kernel")) if key in k), k[:40])
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, d in acc.items():
    print(name)
    for c in sorted(d):
        v = d[c]
        print(f"  {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")
