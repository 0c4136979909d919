"""Print the top kernels of a rocprofv3 kernel_stats.csv (usage: kstats.py file [n])"""
import csv
import sys
rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
for x in rows[:n]:
    print(f"{x['Name'][:48]:48s} {int(x['Calls']):7d} {float(x['TotalDurationNs']) / 1e6:10.2f} ms "
          f"{float(x['AverageNs']) / 1e3:10.1f} us avg {float(x['Percentage']):6.2f}%")
