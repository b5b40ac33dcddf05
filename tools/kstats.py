"""Print a rocprofv3 kernel_stats.csv as a table: name, calls, total ms, average us, percent."""
import csv
import sys

for r in list(csv.DictReader(open(sys.argv[1]))):
    print(f"{r['Name'][:72]:72s} {r['Calls']:>5s} {float(r['TotalDurationNs'])/1e6:9.2f}ms "
          f"{float(r['AverageNs'])/1e3:9.1f}us {float(r['Percentage']):6.2f}%")
