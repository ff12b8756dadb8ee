"""bench.py's contract: the kernel-source digest that ties profiles/traffic.json to the built kernels (CPU), and one
short bench line on the GPU with the fields the driver and DESIGN 6 rely on (roofline, write_probe, placement)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_digest_ignores_comments_not_code():
    src = 'int a = 1; // one\n/* block\n comment */\n  int  b = 2;\n\n'
    assert bench._code_only(src) == bench._code_only('int a = 1;   // uno\nint b = 2; /* two */\n')
    assert bench._code_only(src) != bench._code_only('int a = 1;\nint b = 3;\n')
    d = bench.kernel_source_digest()
    assert len(d) == 16 and d == bench.kernel_source_digest()


def test_traffic_entries_carry_the_digest_and_kernel_time():
    db = json.load(open(os.path.join(ROOT, 'profiles', 'traffic.json')))
    for game, g in bench.GAMES.items():
        key = '%s:%d:%d' % (game, g['envs'], g['T'])
        es = db[key] if isinstance(db[key], list) else [db[key]]
        for e in es:   # (freshness against the built kernels is the bench line's own check: traffic_stale)
            assert len(e['src_sha16']) == 16 and int(e['src_sha16'], 16) >= 0, key
            assert e['kernel_ns_timed_mean'] > 0 and e['bytes_per_launch'] > 0


@pytest.mark.gpu
def test_bench_line_on_the_gpu():
    out = subprocess.run([sys.executable, 'bench.py', '--game', 'leduc-holdem', '--envs', '65536', '--T', '32',
                          '--steps', '5', '--warmup', '2', '--no-cpu-baseline', '--no-philox', '--no-device-state',
                          '--placement', '1'],
                         cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith('{')]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
              'vs_baseline', 'dtype', 'config', 'roofline'):
        assert k in d, k
    assert d['n_gpus'] == 1 and d['steps'] == 5 and d['value'] > 0
    r = d['roofline']
    assert r['bound'] == 'hbm' and 0 < r['frac'] < 1.5 and r['kernel_ms_per_launch'] > 0
    wp = r['write_probe']
    assert wp['ms'] > 0 and wp['bytes'] > 0 and wp['kernel_over_probe'] > 0
    sel = d['placement']['selection']   # the library's own choice (VecEnv.new_traj_out: probe cut, rollout-ranked)
    assert sel['by'] == 'rollout' and sel['library_default'] and sel['candidates'] == len(sel['probe_ms']) >= 2
    assert sel['select_ms'] > 0
    trial = sel['trial_ms']
    assert trial is None or (len(trial) == len(sel['probe_ms']) and any(t is not None and t > 0 for t in trial))
    assert len(d['placement']['kernel_ms_per_allocation']) == 2
