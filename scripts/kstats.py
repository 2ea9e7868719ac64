"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, avg/min/max us."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5} avg {float(r['AverageNs'])/1e3:9.2f} us  min {float(r['MinNs'])/1e3:9.2f}  max {float(r['MaxNs'])/1e3:9.2f}")
