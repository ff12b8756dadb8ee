"""ASan + UBSan over the host-side C/C++: tools/san_driver.cpp exercises the CPU oracle (every game and
entry point, CFR, the evaluator, the DouDizhu legal-set hook), the C ABI's host paths that run without a GPU
(argument validation, error codes, cs_last_error, the no-device failure of cs_create) and the DouDizhu table
expansion, all compiled with -fsanitize=address,undefined -fno-sanitize-recover (any report fails the run)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which('g++') is None or not os.path.exists('/opt/rocm/bin/hipcc'),
                    reason='needs g++ and hipcc')
def test_host_code_under_asan_and_ubsan():
    tools = os.path.join(ROOT, 'tools')
    subprocess.check_call(['make', '-s', '-C', tools, 'san_driver'], timeout=900)
    env = dict(os.environ, ASAN_OPTIONS='abort_on_error=1', UBSAN_OPTIONS='print_stacktrace=1')
    r = subprocess.run([os.path.join(tools, 'san_driver')], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert 'san_driver: ok' in r.stdout
