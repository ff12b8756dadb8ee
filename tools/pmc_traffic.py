#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into per-kernel means and HBM bytes per k_rollout launch.

  python tools/pmc_traffic.py OUT_DIR KEY SOURCE PASS_DIR [PASS_DIR ...]

Each PASS_DIR is one `rocprofv3 --pmc <counters> -d PASS_DIR -- python bench.py ...` run (one counter group per run:
FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950). Writes OUT_DIR/pmc_summary.txt (mean counter value per
kernel) and merges profiles/traffic.json[KEY] (KEY = "game:envs:T", as bench.py looks it up) with
  bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE   (KiB -> bytes)
for the k_rollout kernel: /opt/skills/guides/MI355X_MICROARCH.md (HBM section) -- on gfx950 FETCH_SIZE reports half
the bytes of a wide coalesced read; WRITE_SIZE is exact for 16-B streaming stores.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split('(')[0]


def read_pass(d):
    vals = collections.defaultdict(list)   # (kernel, counter) -> [value per dispatch]
    for path in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                vals[(short(row['Kernel_Name']), row['Counter_Name'])].append(float(row['Counter_Value']))
    return vals


def main():
    out_dir, key, source = sys.argv[1], sys.argv[2], sys.argv[3]
    allv = collections.defaultdict(list)
    for d in sys.argv[4:]:
        for k, v in read_pass(d).items():
            allv[k].extend(v)
    if not allv:
        sys.exit('no counter_collection.csv under %s' % ' '.join(sys.argv[4:]))
    os.makedirs(out_dir, exist_ok=True)
    lines, by_kernel = [], collections.defaultdict(dict)
    for (kern, ctr), v in sorted(allv.items()):
        by_kernel[kern][ctr] = (len(v), sum(v) / len(v))
    for kern in sorted(by_kernel):
        lines.append(kern)
        for ctr, (n, m) in sorted(by_kernel[kern].items()):
            lines.append('   %-32s n=%-4d mean=%g' % (ctr, n, m))
    with open(os.path.join(out_dir, 'pmc_summary.txt'), 'w') as f:
        f.write('\n'.join(lines) + '\n')
    print('\n'.join(lines))
    roll = [k for k in by_kernel if 'k_rollout' in k]
    if len(roll) != 1 or not {'FETCH_SIZE', 'WRITE_SIZE'} <= set(by_kernel[roll[0]]):
        print('no single k_rollout kernel with FETCH_SIZE and WRITE_SIZE: traffic.json not updated')
        return
    r = by_kernel[roll[0]]
    fetch, write = r['FETCH_SIZE'][1], r['WRITE_SIZE'][1]
    tj = os.path.join(ROOT, 'profiles', 'traffic.json')
    try:
        with open(tj) as f:
            data = json.load(f)
    except (OSError, ValueError):
        data = {}
    data[key] = dict(bytes_per_launch=(2 * fetch + write) * 1024.0, fetch_size_kib=fetch, write_size_kib=write,
                     launches=min(r['FETCH_SIZE'][0], r['WRITE_SIZE'][0]), source=source)
    with open(tj, 'w') as f:
        json.dump(data, f, indent=1, sort_keys=True)
        f.write('\n')
    print('traffic.json[%s] = %.4g bytes per launch' % (key, data[key]['bytes_per_launch']))


if __name__ == '__main__':
    main()
