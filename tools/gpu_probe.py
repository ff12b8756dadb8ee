"""GPU probe: seed / reset / rollout at several sizes in ONE process, synchronising after each call; stops at the
first error (a HIP fault is sticky). Prints one line per size.

  python tools/gpu_probe.py [--lib-first | --torch-first] GAME N...
--lib-first loads rlcard_amd/libcardsim.so before torch initialises HIP; --torch-first initialises torch's HIP
state (torch.cuda.current_device()) before the library is loaded.
"""
import sys
import time

sys.path.insert(0, '.')
args = sys.argv[1:]
order = 'default'
if args and args[0].startswith('--'):
    order = args.pop(0)[2:]
if order == 'lib-first':
    from rlcard_amd import _abi
    _abi.lib()
import torch  # noqa: E402
if order == 'torch-first':
    torch.cuda.current_device()
from rlcard_amd import VecEnv  # noqa: E402

game = args[0] if args else 'leduc-holdem'
sizes = [int(x) for x in args[1:]] or [1, 2, 64, 200, 4096, 65536, 1 << 20]
for n in sizes:
    t0 = time.time()
    v = VecEnv(game, n, seed=42, device=0)
    torch.cuda.synchronize()
    t1 = time.time()
    v.reset()
    torch.cuda.synchronize()
    tr = v.rollout(8, policy_seed=1)
    torch.cuda.synchronize()
    print('[%s] %s n=%d ok: seed %.2fs, reset+rollout %.3fs, done frac %.3f' % (
        order, game, n, t1 - t0, time.time() - t1, tr['done'].float().mean().item()), flush=True)
    del v, tr
