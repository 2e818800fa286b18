"""SQ counters per launch of each kernel (rocprofv3 --pmc passes under a directory) as the JSON
bench.py's valu_roofline reads: {"limbs": L, "<counter>": {"<kernel>": mean per dispatch}}.
Usage: sq_json.py <pmc_dir> <limbs> <out.json>"""
import collections
import csv
import glob
import json
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("void ", "").split("(")[0].split("<")[0]
        acc[r["Counter_Name"]][name].append(float(r["Counter_Value"]))
out = {"limbs": int(sys.argv[2]), "source": "rocprofv3 --pmc, mean per dispatch (scripts/gpu_pmc.sh)"}
for c, ks in sorted(acc.items()):
    out[c] = {k: round(sum(v) / len(v), 1) for k, v in sorted(ks.items())}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
