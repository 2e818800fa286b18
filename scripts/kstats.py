"""Summarise a rocprofv3 --stats kernel CSV: share, calls, average per call."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    name = r["Name"].replace("void ", "")[:100]
    print(f"{float(r['Percentage']):6.2f}%  calls={r['Calls']:>5}  avg={float(r['AverageNs']) / 1e3:9.1f} us  {name}")
