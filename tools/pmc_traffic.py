"""Record the HBM traffic of a bench configuration's k_rollout from a rocprofv3 PMC profile (tools/profile.sh) into
profiles/traffic.json, where bench.py reads it for roofline.traffic.

Per MI355X_MICROARCH.md (HBM): FETCH_SIZE / WRITE_SIZE come from separate --pmc passes, are in KiB, and on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads -> traffic = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes).
  python3 tools/pmc_traffic.py <profile dir> <game> <envs> <T> [source label]
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rollout_means(d):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'k_rollout' in r['Kernel_Name']:
                vals[r['Counter_Name']].append(float(r['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


if __name__ == '__main__':
    d, game, envs, T = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    label = sys.argv[5] if len(sys.argv) > 5 else os.path.relpath(d, ROOT)
    m, n = rollout_means(d)
    fetch, write = m['FETCH_SIZE'], m['WRITE_SIZE']
    path = os.path.join(ROOT, 'profiles', 'traffic.json')
    db = json.load(open(path)) if os.path.exists(path) else {}
    db['%s:%d:%d' % (game, envs, T)] = dict(
        bytes_per_launch=(2 * fetch + write) * 1024, fetch_size_kib=fetch, write_size_kib=write,
        launches=min(n.values()), source=label)
    json.dump(db, open(path, 'w'), indent=1, sort_keys=True)
    print(json.dumps(db['%s:%d:%d' % (game, envs, T)]))
