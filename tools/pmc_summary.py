"""Average every PMC counter per kernel over the counter_collection CSVs under a directory."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r['Kernel_Name'].split('(')[0]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in sorted(agg.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print('   %-32s n=%-4d mean=%.6g' % (c, len(v), sum(v) / len(v)))
