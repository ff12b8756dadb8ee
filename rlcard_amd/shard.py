"""Multi-GPU layout: one process per GPU, each owning a contiguous slice of the global env index space.

Envs are independent, so the data path has no collective: rank r runs envs [r*N, (r+1)*N) with the
seeds (seed + global index) and policy counters (global index) a single GPU would use for the same envs, so every
env's trajectory is bit-identical whatever the GPU count. The only exchange is optional and happens after a rollout:
gathering the trajectory shards (obs, legal, player, action, reward, done) to every rank with one all-gather per
tensor (RCCL over xGMI with the nccl backend; gloo in the CPU tests).
"""
import torch
import torch.distributed as dist

__all__ = ['shard_range', 'ShardedVecEnv', 'gather_traj', 'new_gathered']


def shard_range(envs_per_rank, rank):
    """-> (env_base, n): the global env ids [env_base, env_base + n) that `rank` owns (weak scaling)."""
    return rank * int(envs_per_rank), int(envs_per_rank)


def new_gathered(traj, world):
    """Receive buffers [world, *shape] for gather_traj."""
    return {k: torch.empty((world,) + tuple(v.shape), dtype=v.dtype, device=v.device) for k, v in traj.items()}


def gather_traj(traj, out, group=None):
    """All-gather every trajectory tensor [T, N, ...] of this rank into out[k] = [world, T, N, ...] (rank-major, so
    out[k][r] is rank r's shard = global envs [r*N, (r+1)*N))."""
    backend = dist.get_backend(group)
    for k, v in traj.items():
        if backend == 'gloo':      # gloo has no all_gather_into_tensor for every dtype: use the list form
            dist.all_gather(list(out[k].unbind(0)), v.contiguous(), group=group)
        else:
            dist.all_gather_into_tensor(out[k], v.contiguous(), group=group)
    return out


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
