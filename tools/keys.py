"""print init_by_array keys 'k0 k1 len' for seeds base..base+n-1 (input for tools/abi_driver)"""
import sys
sys.path.insert(0, '.')
from rlcard_amd.seeding import seed_keys_range  # noqa: E402
k, l = seed_keys_range(int(sys.argv[1]), 0, int(sys.argv[2]))
sys.stdout.write(''.join('%d %d %d\n' % (a, b, c) for (a, b), c in zip(k.tolist(), l.tolist())))
