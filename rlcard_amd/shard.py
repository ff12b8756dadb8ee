"""Multi-GPU layout: one process per GPU, each owning a contiguous slice of the global env index space.

Envs are independent, so the data path has no collective: rank r runs envs [r*N, (r+1)*N) with the
seeds (seed + global index) and policy counters (global index) a single GPU would use for the same envs, so every
env's trajectory is bit-identical whatever the GPU count. The only exchange happens after a rollout, when the
consumer wants the trajectory shards in one place:

* gather_traj_to(..., dst=0): every shard to one rank (point-to-point sends into rank dst's [world, T, N, ...]
  buffers; RCCL over xGMI with the nccl backend). xGMI is point-to-point, so rank dst receives the 7 shards over its
  7 links at once, and no other rank holds world x the trajectory (gather to the consumer).
* gather_traj(...): all-gather into every rank (world x the trajectory per GPU; for consumers on every rank).

Timing across ranks (bench.py) goes through rank_max / whole_job_rate, so the aggregation is the one the gloo
world-size-2 test checks.
"""
import torch
import torch.distributed as dist

__all__ = ['shard_range', 'ShardedVecEnv', 'gather_traj', 'gather_traj_to', 'new_gathered', 'rank_max',
           'whole_job_rate', 'traj_bytes', 'time_exchange', 'shard_digest', 'verify_gathered']


def shard_range(envs_per_rank, rank):
    """-> (env_base, n): the global env ids [env_base, env_base + n) that `rank` owns (weak scaling)."""
    return rank * int(envs_per_rank), int(envs_per_rank)


def new_gathered(traj, world):
    """Receive buffers [world, *shape] for gather_traj / gather_traj_to (on the receiving rank only)."""
    return {k: torch.empty((world,) + tuple(v.shape), dtype=v.dtype, device=v.device) for k, v in traj.items()}


def traj_bytes(traj):
    return sum(v.numel() * v.element_size() for v in traj.values())


# dtypes RCCL (NCCL) moves natively; anything else (DouDizhu's int16 action rows) is moved as its bytes
_NCCL_DTYPES = {torch.uint8, torch.int8, torch.int32, torch.int64, torch.float16, torch.bfloat16, torch.float32,
                torch.float64}


def _wire(t, backend):
    """t itself, or a uint8 view of its bytes when the backend cannot move its dtype (same memory)."""
    if backend != 'gloo' and t.dtype not in _NCCL_DTYPES:
        return t.view(torch.uint8)
    return t


def gather_traj(traj, out, group=None):
    """All-gather every trajectory tensor [T, N, ...] of this rank into out[k] = [world, T, N, ...] (rank-major, so
    out[k][r] is rank r's shard = global envs [r*N, (r+1)*N))."""
    backend = dist.get_backend(group)
    for k, v in traj.items():
        if backend == 'gloo':      # gloo has no all_gather_into_tensor for every dtype: use the list form
            dist.all_gather(list(out[k].unbind(0)), v.contiguous(), group=group)
        else:
            dist.all_gather_into_tensor(_wire(out[k], backend), _wire(v.contiguous(), backend), group=group)
    return out


def gather_traj_to(traj, out, dst=0, group=None):
    """Every rank's trajectory shard into rank `dst`: out[k][r] = rank r's traj[k] on dst (out is ignored, and may be
    None, elsewhere). One batch of point-to-point operations for all tensors, so the transfers from the world - 1
    senders run concurrently. Returns out on dst, None elsewhere."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    ops = []
    if rank == dst:
        for k, v in traj.items():
            out[k][dst].copy_(v)
            for r in range(world):
                if r != dst:
                    ops.append(dist.P2POp(dist.irecv, _wire(out[k][r], backend), r, group))
    else:
        for k, v in traj.items():
            ops.append(dist.P2POp(dist.isend, _wire(v.contiguous(), backend), dst, group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return out if rank == dst else None


def shard_digest(traj):
    """A position-sensitive fingerprint of a trajectory shard, computed where it lives: per tensor (sorted keys), the
    wrapping int64 sums of its bytes in 4 KiB blocks (the last block zero-padded). Equal digests on sender and receiver
    mean the slice arrived intact and in its place."""
    parts = []
    for k in sorted(traj):
        v = traj[k].contiguous().view(-1).view(torch.uint8)
        main = v.numel() // 4096 * 4096
        if main:
            parts.append(v[:main].view(torch.int64).view(-1, 512).sum(dim=1))
        if v.numel() > main:
            tail = torch.zeros(4096, dtype=torch.uint8, device=v.device)
            tail[:v.numel() - main] = v[main:]
            parts.append(tail.view(torch.int64).sum().reshape(1))
    return torch.cat(parts)


def verify_gathered(traj, gathered, group=None):
    """After an exchange: every rank's digest of its own shard goes to every rank (a small all-gather), each rank
    holding gathered buffers checks every slice r against rank r's digest, and the verdict is the AND over ranks."""
    world = dist.get_world_size(group)
    mine = shard_digest(traj)
    digests = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(digests, mine, group=group)
    ok = True
    if gathered is not None:
        for r in range(world):
            got = shard_digest({k: v[r] for k, v in gathered.items()})
            ok = ok and bool(torch.equal(got, digests[r]))
    flag = torch.tensor([1 if ok else 0], dtype=torch.int64, device=mine.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(flag.item())


def rank_max(x, device=None, group=None):
    """max over ranks of a host float (a per-rank elapsed time); x itself with one rank."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def whole_job_rate(envs_per_rank, steps_per_launch, launches, elapsed_s, world):
    """env-steps/s of the whole job: every rank's env-steps over the slowest rank's time (weak scaling)."""
    return world * int(envs_per_rank) * int(steps_per_launch) * int(launches) / float(elapsed_s)


def time_exchange(produce, traj, mode, steps, envs_per_rank, steps_per_launch, sync=None, device=None):
    """bench.py's N > 1 exchange phase: `steps` x (produce() refills traj, then the exchange: mode 'rank0' =
    gather_traj_to rank 0, 'all' = gather_traj into every rank), bracketed by sync() + barrier, timed as the max
    over ranks. -> (info dict, gathered buffers on the ranks that hold them, else None)."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    gathered = new_gathered(traj, world) if (mode == 'all' or rank == 0) else None
    sync = sync or (lambda: None)
    sync()
    dist.barrier()
    import time
    t0 = time.perf_counter()
    for _ in range(steps):
        produce()
        if mode == 'all':
            gather_traj(traj, gathered)
        else:
            gather_traj_to(traj, gathered, dst=0)
    sync()
    dist.barrier()
    el = rank_max(time.perf_counter() - t0, device)
    info = dict(mode=mode, collective='RCCL %s over xGMI' % (
                    'all_gather_into_tensor' if mode == 'all' else 'send/recv into rank 0'),
                steps=steps, ms_per_step=1e3 * el / steps,
                value=whole_job_rate(envs_per_rank, steps_per_launch, steps, el, world),
                bytes_per_rank_per_step=traj_bytes(traj))
    # untimed: the last exchange's slices checked against their senders' digests (shard_digest)
    info['verified'] = verify_gathered(traj, gathered)
    return info, gathered


class ShardedVecEnv:
    """This rank's VecEnv: envs_per_rank envs starting at global id rank * envs_per_rank, seeded seed + global id."""

    def __init__(self, env_id, envs_per_rank, rank, seed=42, device=None, config=None):
        from .vec import VecEnv
        self.env_base, self.n = shard_range(envs_per_rank, rank)
        self.vec = VecEnv(env_id, self.n, seed=seed, env_base=self.env_base, device=device, config=config)

    def __getattr__(self, name):
        if name == 'vec':
            raise AttributeError(name)
        return getattr(self.vec, name)
