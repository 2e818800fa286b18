"""Summarise a rocprofv3 --stats kernel CSV: share, calls, average per call.

kstats.py STATS.csv            one run
kstats.py diff A.csv B.csv     B - A per kernel (e.g. a 2-image minus a 1-image run = one image)
"""
import csv
import sys


def load(path):
    return {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(path))}


if sys.argv[1] == "diff":
    a, b = load(sys.argv[2]), load(sys.argv[3])
    d = {k: (b[k][0] - a.get(k, (0, 0))[0], b[k][1] - a.get(k, (0, 0))[1]) for k in b}
    # a kernel whose time difference is negative ran slower in the shorter run (e.g. a rare
    # sequential PRNG redraw during key generation): listed apart, not netted into the total
    neg = {k: v for k, v in d.items() if v[1] < 0}
    tot_ns = sum(v[1] for v in d.values() if v[1] >= 0)
    tot_calls = sum(v[0] for v in d.values())
    print(f"difference: {tot_calls} launches, {tot_ns / 1e6:.1f} ms of kernel time"
          + (f" (excluding {len(neg)} kernel(s) slower in the shorter run: "
             + ", ".join(f"{k.replace('void ', '')[:60]} {v[1] / 1e6:.1f} ms" for k, v in neg.items()) + ")" if neg else ""))
    for k, (c, ns) in sorted(d.items(), key=lambda kv: -kv[1][1]):
        if c <= 0 or ns < 0:
            continue
        print(f"{100 * ns / tot_ns:6.2f}%  calls={c:>6}  total={ns / 1e6:8.1f} ms  avg={ns / c / 1e3:7.1f} us  "
              f"{k.replace('void ', '')[:90]}")
else:
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Name"].replace("void ", "")[:100]
        print(f"{float(r['Percentage']):6.2f}%  calls={r['Calls']:>5}  avg={float(r['AverageNs']) / 1e3:9.1f} us  {name}")
