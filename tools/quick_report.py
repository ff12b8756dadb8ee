#!/usr/bin/env python3
"""Summarise gpurun_out/quick (tools/gpu_quick.sh): test tail, bench ms / frac per game, WRITE_SIZE of the last 30
k_rollout dispatches."""
import csv
import glob
import json
import os

Q = 'gpurun_out/quick'
print(open(os.path.join(Q, 'tests.log')).read().strip().splitlines()[-1])
for f in sorted(glob.glob(os.path.join(Q, 'bench_*.log'))):
    lines = [l for l in open(f) if l.startswith('{')]
    if lines:
        d = json.loads(lines[-1])
        print(d['config']['game'], '%.4g env-steps/s  kernel %.3f ms  frac %.3f' % (
            d['value'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac']))
vals = []
for f in glob.glob(os.path.join(Q, 'write', '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_rollout' in r['Kernel_Name']:
            vals.append((int(r.get('Dispatch_Id') or 0), float(r['Counter_Value'])))
if vals:
    vals.sort()
    t = [v for _, v in vals[-30:]]
    print('WRITE_SIZE %.3f GB per launch (last %d)' % (sum(t) / len(t) * 1024 / 1e9, len(t)))
