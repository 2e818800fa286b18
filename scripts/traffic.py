"""Per-HMult HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads exactly half the bytes of a
wide coalesced read -- calibrated here on k_ks_mac (known 2970 MiB read per launch) -- so
bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024.  Usage: traffic.py <pmc_dir> <hmults_in_run | auto> [out.json]
"""
import collections
import csv
import glob
import json
import sys

pmc_dir = sys.argv[1]
if sys.argv[2] == "auto":
    # one k_ks_row_mac dispatch per HMult
    ids = set()
    for f in glob.glob(f"{pmc_dir}/FETCH_SIZE/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_ks_row_mac" in r["Kernel_Name"]:
                ids.add(r.get("Dispatch_Id", len(ids)))
    hmults = max(1, len(ids))
else:
    hmults = int(sys.argv[2])
# one-time setup kernels of the bench process (key preparation), not part of any HMult
SETUP = ("k_key_pack",)
setup = collections.defaultdict(float)
tot = collections.defaultdict(float)
per_kernel = collections.defaultdict(lambda: collections.defaultdict(float))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{pmc_dir}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != c:
                continue
            v = float(r["Counter_Value"]) * 1024 * (2 if c == "FETCH_SIZE" else 1)
            if any(k in r["Kernel_Name"] for k in SETUP):
                setup[c] += v
                continue
            tot[c] += v
            per_kernel[r["Kernel_Name"].replace("void ", "").split("(")[0]][c] += v
hbm = (tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) / hmults
res = {
    "hbm_bytes_per_hmult": hbm,
    "read_bytes_per_hmult": tot["FETCH_SIZE"] / hmults,
    "write_bytes_per_hmult": tot["WRITE_SIZE"] / hmults,
    "correction": "FETCH_SIZE x2 (gfx950 wide-load undercount), WRITE_SIZE x1",
    "setup_kernels_excluded": {k: None for k in SETUP} | {"bytes_total": setup["FETCH_SIZE"] + setup["WRITE_SIZE"]},
    "per_kernel_GB_per_hmult": {k: round((v["FETCH_SIZE"] + v["WRITE_SIZE"]) / hmults / 1e9, 4)
                                for k, v in sorted(per_kernel.items(), key=lambda kv: -sum(kv[1].values()))},
}
print(json.dumps(res, indent=1))
if len(sys.argv) > 3:
    json.dump(res, open(sys.argv[3], "w"), indent=1)
