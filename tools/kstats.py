"""Print the top rows of a rocprofv3 kernel_stats.csv: python tools/kstats.py FILE [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 10]:
    print(f"{r['Name'][:56]:56s} calls={r['Calls']:>6s} total_ms={float(r['TotalDurationNs'])/1e6:9.2f} "
          f"avg_us={float(r['AverageNs'])/1e3:10.2f} pct={float(r['Percentage']):6.2f}")
