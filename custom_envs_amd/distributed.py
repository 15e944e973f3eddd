"""Env-sharded multi-GPU path.

Envs never read each other's state, so the batch splits into contiguous
shards: rank r owns global envs [lo_r, hi_r) and seeds each with its global
index, which makes every env's trajectory independent of the rank count.
Stepping needs no communication.  When a consumer wants the whole batch on
every rank (the north star's centralised learner), ``ShardedEnvs.gather``
does ONE collective per step: the engine writes all its outputs into one
packed byte buffer (one aligned segment per field, no packing kernels) and
``all_gather_into_tensor`` concatenates the ranks' buffers -- RCCL over xGMI
under the ``nccl`` backend, gloo in the CPU tests.

The reference has no multi-GPU code; its scaling unit is one worker per env
(custom_envs/vectorize/concurrentvecenv.py:74-92).
"""
import torch

ALIGN = 256


def shard_range(num_envs, world, rank):
    """Contiguous [lo, hi) of ``num_envs`` for ``rank``; the first
    ``num_envs % world`` ranks get one env more."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError('bad rank/world')
    base, extra = divmod(num_envs, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class PackedLayout:
    """Fields of one shard's step outputs as aligned segments of a byte buffer.

    ``fields``: (name, torch dtype, rows per env, trailing shape).  Segments
    are sized for ``capacity`` envs (the largest shard) so every rank's
    buffer has the same length, as all_gather requires.
    """

    def __init__(self, fields, capacity):
        self.fields = [(n, d, int(r), tuple(t)) for n, d, r, t in fields]
        self.capacity = int(capacity)
        self.offsets = {}
        off = 0
        for name, dtype, rows, tail in self.fields:
            self.offsets[name] = off
            off += -(-self._nbytes(dtype, rows, tail, self.capacity) // ALIGN) * ALIGN
        self.nbytes = off

    @staticmethod
    def _nbytes(dtype, rows, tail, envs):
        n = envs * rows
        for t in tail:
            n *= t
        return n * torch.empty((), dtype=dtype).element_size()

    def views(self, buf, num_envs):
        """Typed views of the first ``num_envs`` envs of each segment."""
        out = {}
        for name, dtype, rows, tail in self.fields:
            off = self.offsets[name]
            size = self._nbytes(dtype, rows, tail, num_envs)
            out[name] = buf[off:off + size].view(dtype).view((num_envs * rows,) + tail)
        return out

    def unpack(self, gathered, counts):
        """Global outputs (rank-major) from the all-gathered buffers."""
        per_rank = gathered.view(len(counts), self.nbytes)
        parts = [self.views(per_rank[r], c) for r, c in enumerate(counts)]
        return {name: torch.cat([p[name] for p in parts]) for name, *_ in self.fields}


class ShardedEnvs:
    """One rank's shard of a global env batch, with the optional all-gather.

    ``engine`` is this rank's engine over ``hi - lo`` envs (``OptimizeEngine``
    or ``MultiOptEngine``); it must expose ``output_fields()``,
    ``reset_device(out)`` and ``step_device(actions, out)``.
    """

    def __init__(self, engine, num_envs, rank=0, world=1, group=None, device=None):
        self.engine, self.rank, self.world, self.group = engine, rank, world, group
        self.num_envs = int(num_envs)
        self.lo, self.hi = shard_range(self.num_envs, world, rank)
        if engine.num_envs != self.hi - self.lo:
            raise ValueError('engine has %d envs, shard %d owns %d'
                             % (engine.num_envs, rank, self.hi - self.lo))
        self.counts = [b - a for a, b in (shard_range(self.num_envs, world, r)
                                          for r in range(world))]
        self.layout = PackedLayout(engine.output_fields(), max(self.counts))
        device = device if device is not None else torch.device('cuda', torch.cuda.current_device())
        self.buffer = torch.zeros(self.layout.nbytes, dtype=torch.uint8, device=device)
        self.out = self.layout.views(self.buffer, engine.num_envs)
        self.gathered = (torch.empty(world * self.layout.nbytes, dtype=torch.uint8,
                                     device=device) if world > 1 else None)

    @property
    def global_indices(self):
        return list(range(self.lo, self.hi))

    def seed(self, base_seed=0):
        """Seed = base + global env index: shards reproduce a 1-GPU run."""
        return self.engine.seed([base_seed + g for g in self.global_indices])

    def reset(self):
        self.engine.reset_device(self.out)
        return self.out

    def step(self, actions):
        self.engine.step_device(actions, self.out)
        return self.out

    def gather(self):
        """Every rank gets the global outputs (rank-major = global env order)."""
        if self.world == 1:
            return self.out
        import torch.distributed as dist
        dist.all_gather_into_tensor(self.gathered, self.buffer, group=self.group)
        return self.layout.unpack(self.gathered, self.counts)
