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

The chunk schedule (``chunk`` = K > 1): the engine runs K steps in ONE
persistent launch (``rollout_device``) whose step t writes record t of a
[K]-record buffer, and ONE collective gathers all K records
(``gather_chunk``): the collective's fixed cost is paid once per K steps,
and with two buffers (``slots=2``) the gather of chunk c runs on RCCL's
stream while chunk c + 1's launch writes the other buffer.

The reference has no multi-GPU code; its scaling unit is one worker per env
(custom_envs/vectorize/concurrentvecenv.py:74-92).
"""
from collections.abc import Mapping

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

    def rank_views(self, gathered, world, rank_stride=None, offset=0):
        """Zero-copy views of an all-gathered buffer: field -> tensor of shape
        (world, capacity * rows, *tail), rank r's shard in row r (only its
        first counts[r] * rows entries are live).  ``rank_stride`` (bytes
        between ranks' records; default one record) and ``offset`` (bytes to
        this record in rank 0's part) address record t of a gathered chunk."""
        rank_stride = self.nbytes if rank_stride is None else rank_stride
        out = {}
        for name, dtype, rows, tail in self.fields:
            size = torch.empty((), dtype=dtype).element_size()
            flat = gathered.view(dtype)
            dims = (self.capacity * rows,) + tuple(tail)
            inner = [1] * len(dims)
            for i in range(len(dims) - 2, -1, -1):
                inner[i] = inner[i + 1] * dims[i + 1]
            out[name] = flat.as_strided((world,) + dims, (rank_stride // size,) + tuple(inner),
                                        flat.storage_offset() + (offset + self.offsets[name]) // size)
        return out

    def chunk_views(self, buf, num_envs, k):
        """Field -> (k, num_envs * rows, *tail) views of a [k]-record buffer
        (record t at t * nbytes): the output slab of a k-step rollout."""
        out = {}
        for name, dtype, rows, tail in self.fields:
            size = torch.empty((), dtype=dtype).element_size()
            flat = buf.view(dtype)
            dims = (num_envs * rows,) + tuple(tail)
            inner = [1] * len(dims)
            for i in range(len(dims) - 2, -1, -1):
                inner[i] = inner[i + 1] * dims[i + 1]
            out[name] = flat.as_strided((k,) + dims, (self.nbytes // size,) + tuple(inner),
                                        flat.storage_offset() + self.offsets[name] // size)
        return out

    def unpack(self, gathered, counts):
        """Global outputs (rank-major = global env order), one copy per field."""
        views = self.rank_views(gathered, len(counts))
        rows = {name: r for name, _, r, _ in self.fields}
        return {name: torch.cat([v[r, :c * rows[name]] for r, c in enumerate(counts)])
                for name, v in views.items()}


class GatheredOutputs(Mapping):
    """One step's all-gathered outputs.

    ``rank_major[name]`` is a zero-copy (world, capacity * rows, ...) view of
    the collective's buffer.  ``outputs[name]`` is the global array in env
    order, built on first access (one copy per field, only for fields a
    consumer reads; at world 1 a zero-copy view).  ``derived`` names fields
    the wire format leaves out (the compact form: full ``obs`` rows and
    ``done``) with the function that rebuilds each from the stored fields.

    Lifetime: the result reads the slot's gather buffer.  The next gather into
    the same slot overwrites it, so a field first read after that returns the
    newer step's data.  Read what you need before then, or call
    ``snapshot()``, which materialises every field as its own tensor.
    """

    def __init__(self, layout, gathered, counts, derived=None, rank_stride=None, offset=0):
        self.layout, self.counts = layout, counts
        self.rank_major = layout.rank_views(gathered, len(counts), rank_stride, offset)
        self._rows = {name: r for name, _, r, _ in layout.fields}
        self._derived = dict(derived or {})
        self._flat = {}

    def __getitem__(self, name):
        if name not in self._flat:
            if name in self._derived:
                self._flat[name] = self._derived[name](self)
            else:
                v, rows = self.rank_major[name], self._rows[name]
                if len(self.counts) == 1:
                    self._flat[name] = v[0, :self.counts[0] * rows]
                else:
                    self._flat[name] = torch.cat([v[r, :c * rows] for r, c in enumerate(self.counts)])
        return self._flat[name]

    def __iter__(self):
        names = list(self.rank_major)
        return iter(names + [n for n in self._derived if n not in names])

    def __len__(self):
        return len(set(self.rank_major) | set(self._derived))

    def snapshot(self):
        """Every field (stored and derived) as a tensor of its own: valid after
        later gathers into the same slot."""
        return {name: self[name].clone() for name in self}


class ShardedEnvs:
    """One rank's shard of a global env batch, with the optional all-gather.

    ``engine`` is this rank's engine over ``hi - lo`` envs (``OptimizeEngine``
    or ``MultiOptEngine``); it must expose ``output_fields()``,
    ``reset_device(out)`` and ``step_device(actions, out)``.  ``slots`` > 1
    keeps that many packed output buffers, so the collective of step t can
    run while step t+1 writes the other buffer (``step(actions, slot)``,
    ``gather(slot, async_op=True)``).
    """

    def __init__(self, engine, num_envs, rank=0, world=1, group=None, device=None, slots=1,
                 collective=None, compact=None, chunk=1):
        """``collective``: run the all-gather even at world 1 (tests the RCCL
        path on one GPU); default: only when world > 1.  ``compact``: have the
        engine write (and the collective move) the compact record -- obs
        without its identically-zero weight block, done folded into
        episode_len -- when the engine offers it (``set_compact_outputs``);
        default: whenever the collective runs.  ``gather`` rebuilds the full
        fields lazily.  ``chunk`` = K: every slot holds K step records
        (``rollout``, ``gather_chunk``)."""
        self.engine, self.rank, self.world, self.group = engine, rank, world, group
        self.collective = world > 1 if collective is None else bool(collective)
        self.num_envs = int(num_envs)
        self.lo, self.hi = shard_range(self.num_envs, world, rank)
        if engine.num_envs != self.hi - self.lo:
            raise ValueError('engine has %d envs, shard %d owns %d'
                             % (engine.num_envs, rank, self.hi - self.lo))
        self.counts = [b - a for a, b in (shard_range(self.num_envs, world, r)
                                          for r in range(world))]
        if compact is None:
            compact = self.collective
        self.compact = False
        if compact and hasattr(engine, 'set_compact_outputs'):
            from custom_envs_amd._native import NativeEngineError
            try:
                engine.set_compact_outputs(True)
                self.compact = True
            except NativeEngineError:       # this engine's kernel writes the full form only
                pass
        self.derived = engine.derived_fields() if hasattr(engine, 'derived_fields') else {}
        self.layout = PackedLayout(engine.output_fields(), max(self.counts))
        device = device if device is not None else torch.device('cuda', torch.cuda.current_device())
        # In place: the engine writes its outputs straight into this rank's
        # slot of the gathered buffer, so the all-gather moves only the other
        # ranks' records (NCCL/RCCL in-place form: send = recv + rank * count;
        # at world 1 it has nothing to move)
        self.chunk = int(chunk)
        if self.chunk < 1:
            raise ValueError('chunk must be >= 1')
        nb = self.layout.nbytes * self.chunk
        self.gathered = [torch.zeros(world * nb, dtype=torch.uint8, device=device)
                         if self.collective else None for _ in range(slots)]
        self.buffers = [g[rank * nb:(rank + 1) * nb] if g is not None
                        else torch.zeros(nb, dtype=torch.uint8, device=device)
                        for g in self.gathered]
        # record 0 of every slot: what the one-step calls write
        self.outs = [self.layout.views(b, engine.num_envs) for b in self.buffers]
        # every record of every slot: what a K-step rollout writes
        self.slabs = [self.layout.chunk_views(b, engine.num_envs, self.chunk) for b in self.buffers]
        self._partial = {}                 # receive buffers of shorter gathers, by (slot, k)

    @property
    def buffer(self):
        return self.buffers[0]

    @property
    def out(self):
        return self.outs[0]

    @property
    def global_indices(self):
        return list(range(self.lo, self.hi))

    def seed(self, base_seed=0):
        """Seed = base + global env index: shards reproduce a 1-GPU run."""
        return self.engine.seed([base_seed + g for g in self.global_indices])

    def reset(self, slot=0):
        self.engine.reset_device(self.outs[slot])
        return self.outs[slot]

    def step(self, actions, slot=0):
        self.engine.step_device(actions, self.outs[slot])
        return self.outs[slot]

    def rollout(self, actions, slot=0, k=None):
        """k (default: chunk) steps in one call of the engine's
        ``rollout_device``: step t reads actions[t] and writes record t of
        the slot."""
        k = self.chunk if k is None else int(k)
        if not 1 <= k <= self.chunk:
            raise ValueError('rollout of %d steps into a %d-record slot' % (k, self.chunk))
        self.engine.rollout_device(k, actions, self.slabs[slot], self.layout.nbytes)
        return self.slabs[slot]

    def rollout_runner(self, actions, slot=0, k=None):
        """``rollout`` bound once (the engine's pre-bound form when it has one)."""
        k = self.chunk if k is None else int(k)
        if hasattr(self.engine, 'rollout_runner'):
            return self.engine.rollout_runner(k, actions, self.slabs[slot], self.layout.nbytes)
        return lambda: self.rollout(actions, slot, k)

    def gather_chunk(self, slot=0, async_op=False, k=None):
        """ONE collective for the k (default: chunk) records of a slot: every
        rank gets every rank's k steps.  Returns a list of k
        ``GatheredOutputs`` (step t's global outputs; views of the gathered
        buffer, built lazily) and, with ``async_op``, the collective's work
        handle.  A k below the chunk gathers the first k records
        (out of place: the in-place form needs whole slots)."""
        k = self.chunk if k is None else int(k)
        nb = self.layout.nbytes
        world = len(self.counts)
        work = None
        if not self.collective:
            gathered, stride = self.buffers[slot], nb * self.chunk
        else:
            import torch.distributed as dist
            if k == self.chunk:
                gathered, stride = self.gathered[slot], nb * self.chunk
                work = dist.all_gather_into_tensor(gathered, self.buffers[slot], group=self.group,
                                                   async_op=async_op)
            else:
                # a persistent receive buffer per (slot, k): no allocation per
                # call (and none inside a captured graph)
                key = (slot, k)
                if key not in self._partial:
                    self._partial[key] = torch.empty(world * k * nb, dtype=torch.uint8,
                                                     device=self.buffers[slot].device)
                gathered, stride = self._partial[key], k * nb
                work = dist.all_gather_into_tensor(gathered, self.buffers[slot][:k * nb],
                                                   group=self.group, async_op=async_op)
        counts = self.counts if self.collective else [self.hi - self.lo]
        steps = [GatheredOutputs(self.layout, gathered, counts, self.derived, rank_stride=stride,
                                 offset=t * nb) for t in range(k)]
        return (steps, work) if async_op else steps

    def gather(self, slot=0, async_op=False):
        """Every rank gets the global outputs: ONE all_gather_into_tensor of the
        packed buffer.  Returns ``GatheredOutputs`` (at world 1 without the
        collective, views of this rank's own buffer); with ``async_op`` also the
        collective's work handle, whose ``wait()`` orders the caller's current
        stream after it."""
        if self.chunk > 1:                  # record 0 of a chunk slot
            steps, work = self.gather_chunk(slot, True, k=1)
            if work is not None and not async_op:
                work.wait()
            return (steps[0], work) if async_op else steps[0]
        if not self.collective:
            res = GatheredOutputs(self.layout, self.buffers[slot], [self.hi - self.lo],
                                  self.derived)
            return (res, None) if async_op else res
        import torch.distributed as dist
        work = dist.all_gather_into_tensor(self.gathered[slot], self.buffers[slot],
                                           group=self.group, async_op=async_op)
        res = GatheredOutputs(self.layout, self.gathered[slot], self.counts, self.derived)
        return (res, work) if async_op else res
