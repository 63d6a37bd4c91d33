"""Average PMC counters per dispatch for each kernel in rocprofv3 counter_collection CSVs."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta[k] = (r["Grid_Size"], r["Workgroup_Size"], r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"])
for k, cs in acc.items():
    print("%s grid=%s wg=%s vgpr=%s sgpr=%s lds=%s" % ((k,) + meta[k]))
    for c, v in sorted(cs.items()):
        print("   %-24s %16.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))
