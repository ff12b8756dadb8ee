"""Multi-GPU layout: one process per GPU, each owning a contiguous slice of the global env index space.

Envs are independent, so the data path has no collective: rank r runs envs [r*N, (r+1)*N) with the
seeds (seed + global index) and policy counters (global index) a single GPU would use for the same envs, so every
env's trajectory is bit-identical whatever the GPU count. The only exchange happens after a rollout, when the
consumer wants the trajectory shards in one place:

* gather_traj_to(..., dst=0): every shard to one rank (point-to-point sends into rank dst's [world, T, N, ...]
  buffers; RCCL over xGMI with the nccl backend). xGMI is point-to-point, so rank dst receives the 7 shards over its
  7 links at once, and no other rank holds world x the trajectory (gather to the consumer).
* gather_traj(...): all-gather into every rank (world x the trajectory per GPU; for consumers on every rank).
* exchange_traj(...): either exchange in T-slices through receive buffers of a stated budget (default 32 GiB per
  GPU, checked before allocating), each slice handed to a consumer callback and optionally verified; this is what
  bench.py times (config 5's all-gather would otherwise need 8 x 12.9 GB of receive buffers on every GPU).

Timing across ranks (bench.py) goes through rank_max / whole_job_rate, so the aggregation is the one the gloo
world-size-2 test checks.
"""
import torch
import torch.distributed as dist

__all__ = ['shard_range', 'ShardedVecEnv', 'gather_traj', 'gather_traj_to', 'new_gathered', 'rank_max',
           'whole_job_rate', 'traj_bytes', 'time_exchange', 'shard_digest', 'verify_gathered', 'exchange_traj',
           'exchange_chunk_steps', 'RecvBuffers', 'DEFAULT_RECV_BUDGET']


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


_DIGEST_PIECE = 1 << 28   # bytes per aligned piece of shard_digest (a multiple of its 4 KiB blocks)


def _block_sums(v):
    """Wrapping int64 sums of a flat uint8 tensor's 4 KiB blocks (the last one zero-padded). Pieces that start off an
    8-byte boundary (a slice of a gathered buffer whose shard size is not a multiple of 8) or end mid-block are copied
    into an aligned zero-padded buffer first, so the int64 view is always legal."""
    out = []
    for s in range(0, v.numel(), _DIGEST_PIECE):
        seg = v[s:s + _DIGEST_PIECE]
        if seg.data_ptr() % 8 or seg.numel() % 4096:
            b = torch.zeros((seg.numel() + 4095) // 4096 * 4096, dtype=torch.uint8, device=seg.device)
            b[:seg.numel()] = seg
            seg = b
        out.append(seg.view(torch.int64).view(-1, 512).sum(dim=1))
    return out


def shard_digest(traj):
    """A position-sensitive fingerprint of a trajectory shard, computed where it lives: per tensor (sorted keys), the
    wrapping int64 sums of its bytes in 4 KiB blocks (the last block zero-padded). Equal digests on sender and receiver
    mean the slice arrived intact and in its place."""
    parts = []
    for k in sorted(traj):
        parts += _block_sums(traj[k].contiguous().view(-1).view(torch.uint8))
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


# -- bounded exchange: T-slices through fixed receive buffers ----------------------------------------------------------

DEFAULT_RECV_BUDGET = 32 << 30   # receive-buffer bytes per GPU (BASELINE config 5 all-gather: 8 x 12.9 GB otherwise)


def _steps(traj):
    T = {int(v.shape[0]) for v in traj.values()}
    if len(T) != 1:
        raise ValueError('trajectory tensors disagree on T: %s' % sorted(T))
    return T.pop()


def exchange_chunk_steps(traj, world, budget_bytes=DEFAULT_RECV_BUDGET):
    """T-rows per exchanged slice so that a receiver's buffers, world x rows x (bytes of one step of every tensor),
    stay within budget_bytes. Every rank computes the same value from its own shard (shards have equal shapes).
    Raises ValueError when not even one step fits."""
    T = _steps(traj)
    row = traj_bytes(traj) // max(T, 1)
    tc = min(T, int(budget_bytes) // max(1, world * row))
    if tc < 1:
        raise ValueError('receive budget %d B cannot hold one step of %d shards (%d B)' % (budget_bytes, world,
                                                                                          world * row))
    return tc


class RecvBuffers:
    """Receive buffers for chunk_steps T-rows of `world` shards: one flat allocation per tensor, viewed for a slice
    of n <= chunk_steps rows as a contiguous [world, n, ...] (what all_gather_into_tensor and the p2p receives
    need). The size is checked against the budget and, on a GPU, the free device memory before allocating."""

    def __init__(self, traj, world, chunk_steps, budget_bytes=DEFAULT_RECV_BUDGET):
        self.world, self.chunk_steps = int(world), int(chunk_steps)
        self.tail = {k: tuple(v.shape[1:]) for k, v in traj.items()}
        per = {k: self.world * self.chunk_steps * v[0].numel() for k, v in traj.items()}
        self.nbytes = sum(per[k] * traj[k].element_size() for k in traj)
        if self.nbytes > budget_bytes:
            raise ValueError('receive buffers of %d B exceed the budget of %d B' % (self.nbytes, budget_bytes))
        dev = next(iter(traj.values())).device
        if dev.type == 'cuda':
            free, _ = torch.cuda.mem_get_info(dev)
            if self.nbytes > free:
                raise MemoryError('receive buffers of %d B exceed the %d B free on %s' % (self.nbytes, free, dev))
        self.flat = {k: torch.empty(per[k], dtype=traj[k].dtype, device=dev) for k in traj}

    def view(self, n):
        """{key: [world, n, ...]} over the leading part of each flat buffer."""
        return {k: f[:self.world * n * _numel(self.tail[k])].view((self.world, n) + self.tail[k])
                for k, f in self.flat.items()}


def _numel(shape):
    m = 1
    for d in shape:
        m *= int(d)
    return m


def exchange_traj(traj, mode, recv=None, chunk_steps=None, dst=0, consume=None, verify=False, group=None,
                  budget_bytes=DEFAULT_RECV_BUDGET):
    """The trajectory exchange in T-slices of chunk_steps rows: for each slice [t0, t1) every shard's rows go to rank
    dst (mode 'rank0') or to every rank (mode 'all') into `recv` (RecvBuffers, reused for every slice; allocated here
    when None on a receiving rank), then consume(t0, t1, views) runs on the receiving ranks with views[k] =
    [world, t1 - t0, N, ...] (rank-major: views[k][r] = global envs [r*N, (r+1)*N) at steps t0..t1-1). With
    verify=True each slice is then checked against its senders' shard_digest (after consume, so whatever happened to
    the slice before it was consumed is covered). -> (verified: bool or None, recv)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    T = _steps(traj)
    if chunk_steps is None:
        chunk_steps = recv.chunk_steps if recv is not None else exchange_chunk_steps(traj, world, budget_bytes)
    receiving = mode == 'all' or rank == dst
    if receiving and recv is None:
        recv = RecvBuffers(traj, world, chunk_steps, budget_bytes)
    ok = True
    for t0 in range(0, T, chunk_steps):
        t1 = min(T, t0 + chunk_steps)
        piece = {k: v[t0:t1] for k, v in traj.items()}
        views = recv.view(t1 - t0) if receiving else None
        if mode == 'all':
            gather_traj(piece, views, group)
        else:
            gather_traj_to(piece, views, dst, group)
        if receiving and consume is not None:
            consume(t0, t1, views)
        if verify:
            ok = verify_gathered(piece, views, group) and ok
    return (ok if verify else None), recv


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


def time_exchange(produce, traj, mode, steps, envs_per_rank, steps_per_launch, sync=None, device=None,
                  budget_bytes=DEFAULT_RECV_BUDGET):
    """bench.py's N > 1 exchange phase: `steps` x (produce() refills traj, then the exchange: mode 'rank0' = every
    shard into rank 0, 'all' = into every rank; exchange_traj in T-slices whose receive buffers fit budget_bytes per
    GPU), bracketed by sync() + barrier, timed as the max over ranks. -> (info dict, the receive buffers' view of the
    last slice on the ranks that hold them, else None)."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    chunk = exchange_chunk_steps(traj, world, budget_bytes)
    recv = RecvBuffers(traj, world, chunk, budget_bytes) if (mode == 'all' or rank == 0) else None
    sync = sync or (lambda: None)
    sync()
    dist.barrier()
    import time
    t0 = time.perf_counter()
    for _ in range(steps):
        produce()
        exchange_traj(traj, mode, recv, chunk)
    sync()
    dist.barrier()
    el = rank_max(time.perf_counter() - t0, device)
    T = _steps(traj)
    info = dict(mode=mode, collective='RCCL %s over xGMI' % (
                    'all_gather_into_tensor' if mode == 'all' else 'send/recv into rank 0'),
                steps=steps, ms_per_step=1e3 * el / steps,
                value=whole_job_rate(envs_per_rank, steps_per_launch, steps, el, world),
                bytes_per_rank_per_step=traj_bytes(traj), chunk_steps=chunk, chunks=-(-T // chunk),
                recv_buffer_bytes=None if recv is None else recv.nbytes, recv_budget_bytes=int(budget_bytes))
    # untimed: one more exchange of the last trajectory, every slice checked against its senders' digests
    info['verified'], _ = exchange_traj(traj, mode, recv, chunk, verify=True)
    last = T - (T - 1) // chunk * chunk
    return info, (None if recv is None else recv.view(last))


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
