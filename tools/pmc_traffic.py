"""Record the HBM traffic and duration of a bench configuration's k_rollout from rocprofv3 runs of bench.py
(tools/gpu.sh profile:GAME: kernel trace + stats, then one --pmc pass each for FETCH_SIZE and WRITE_SIZE) into
profiles/traffic.json, where bench.py reads it for roofline.traffic.

Only the LAST `steps` k_rollout dispatches of each run are used -- bench.py's timed launches -- so the untimed
preconditioning / warm-up launches do not enter the averages.
Per MI355X_MICROARCH.md (HBM): FETCH_SIZE / WRITE_SIZE are in KiB, from separate --pmc passes; on gfx950 FETCH_SIZE
counts half the bytes of wide coalesced reads -> traffic = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes). The other
access shapes the rollout uses are calibrated by tools/calib.py (DESIGN's traffic account).
  python3 tools/pmc_traffic.py <profile dir> <game> <envs> <T> <steps> [source label]
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _did(r):
    for k in ('Dispatch_Id', 'Correlation_Id'):
        if r.get(k):
            return int(r[k])
    return 0


def counter_means(d, last):
    """counter -> mean over the last `last` k_rollout dispatches (each counter's own pass)."""
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'k_rollout' in r['Kernel_Name']:
                vals[r['Counter_Name']].append((_did(r), float(r['Counter_Value'])))
    out = {}
    for k, v in vals.items():
        v.sort()
        tail = [x for _, x in v[-last:]]
        out[k] = (sum(tail) / len(tail), len(tail), len(v))
    return out


def timed_durations(d, last):
    """(mean, min, max) ns of the last `last` k_rollout dispatches of the kernel trace, and the dispatch count."""
    v = []
    for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'k_rollout' in r['Kernel_Name']:
                v.append((int(r['Start_Timestamp']), int(r['End_Timestamp']) - int(r['Start_Timestamp'])))
    v.sort()
    tail = [x for _, x in v[-last:]]
    return (sum(tail) / len(tail), min(tail), max(tail)), len(v)


if __name__ == '__main__':
    d, game, envs, T, steps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    label = sys.argv[6] if len(sys.argv) > 6 else os.path.relpath(d, ROOT)
    m = counter_means(d, steps)
    fetch, write = m['FETCH_SIZE'][0], m['WRITE_SIZE'][0]
    entry = dict(bytes_per_launch=(2 * fetch + write) * 1024, fetch_size_kib=fetch, write_size_kib=write,
                 launches=min(m['FETCH_SIZE'][1], m['WRITE_SIZE'][1]), source=label)
    try:
        (mean, lo, hi), nd = timed_durations(d, steps)
        entry.update(kernel_ns_timed_mean=mean, kernel_ns_timed_min=lo, kernel_ns_timed_max=hi, dispatches=nd)
    except (ZeroDivisionError, ValueError):
        pass
    sys.path.insert(0, ROOT)
    from bench import kernel_source_digest      # bench.py reports the entry only for these kernel sources
    entry['src_sha16'] = kernel_source_digest()
    path = os.path.join(ROOT, 'profiles', 'traffic.json')
    db = json.load(open(path)) if os.path.exists(path) else {}
    key = '%s:%d:%d' % (game, envs, T)
    # one profile per HBM placement class: profiles of these kernel sources whose kernel times differ by
    # more than 5 % are kept side by side (bench.py cites the one nearest its own kernel time); older sources dropped
    old = db.get(key)
    old = [] if old is None else (old if isinstance(old, list) else [old])
    keep = [e for e in old if e.get('src_sha16') == entry['src_sha16'] and 'kernel_ns_timed_mean' in e and
            'kernel_ns_timed_mean' in entry and
            abs(e['kernel_ns_timed_mean'] - entry['kernel_ns_timed_mean']) > 0.05 * entry['kernel_ns_timed_mean']]
    db[key] = keep + [entry] if keep else entry
    json.dump(db, open(path, 'w'), indent=1, sort_keys=True)
    print(json.dumps(entry))
