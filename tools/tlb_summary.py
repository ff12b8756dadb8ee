"""Summarise rocprofv3 --pmc runs of tools/tlb_probe.py: per k_rollout dispatch its duration (the dispatch's own
Start/End timestamps) and counter values, grouped by allocation instance (a k_seed dispatch starts an instance);
per instance the medians over the timed launches (the last `timed` rollouts of the instance).

  python tools/tlb_summary.py DIR [timed]      (DIR: a rocprofv3 -d directory, searched for *counter_collection.csv)
"""
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
timed = int(sys.argv[2]) if len(sys.argv) > 2 else 6
files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
disp = {}
for f in files:
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = int(r['Dispatch_Id'])
            e = disp.setdefault(k, {'name': r['Kernel_Name'], 'ms': (int(r['End_Timestamp']) -
                                                                      int(r['Start_Timestamp'])) * 1e-6, 'c': {}})
            e['c'][r['Counter_Name']] = e['c'].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
inst, cur = [], None
for k in sorted(disp):
    e = disp[k]
    if 'k_seed' in e['name']:
        cur = []
        inst.append(cur)
    elif 'k_rollout' in e['name'] and cur is not None:
        cur.append(e)
names = sorted({c for e in disp.values() for c in e['c']})
print('instance  ms(median of last %d)  ' % timed + '  '.join(names))
for i, rows in enumerate(inst):
    t = rows[-timed:]
    if not t:
        continue
    med = statistics.median(e['ms'] for e in t)
    vals = ['%.4g' % statistics.median(e['c'].get(c, 0.0) for e in t) for c in names]
    print('%d  %.3f  ' % (i, med) + '  '.join(vals))
