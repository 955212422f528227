"""Data-parallel training support for the Generator (BASELINE config 4).

One process per GPU.  Each rank runs the reference training step on its own shard of utterance
minibatches; the only exchange is the all-reduce (sum, then /world) of the flat 113.7 MB
gradient, after which every rank applies the same fused clip/Adam/EMA update, so the parameters
stay bit-identical across ranks.  The all-reduce is bucketed and overlapped with backward
(`GradBuckets`): contiguous ranges of the flat gradient, in reverse parameter order, are reduced
asynchronously as soon as backward has produced every gradient in them.  BatchNorm batch statistics stay per rank (no
SyncBN); the running buffers are broadcast from rank 0 before a checkpoint is written.
With the nccl backend torch.distributed is RCCL over xGMI on MI355X.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def average_gradients(flat_grad: torch.Tensor) -> torch.Tensor:
    """In-place mean of the flat gradient over all ranks (one collective)."""
    ws = world()
    if ws > 1:
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM)
        flat_grad.div_(ws)
    return flat_grad


class GradBuckets:
    """Bucketed all-reduce of a flat gradient, overlapped with backward.

    `params[i].grad` must be the view `flat_grad[off_i : off_i + n_i]` (AutoEncoder._ensure_flat),
    offsets increasing with i.  Buckets are runs of consecutive parameters of about
    `bucket_bytes`, formed from the LAST parameter backwards: backward produces the postnet's and
    decoder's gradients first and the encoder's last (the encoder is also the only block the
    loss runs twice, model.py:215-219, so its gradients are final only at the very end).  Each
    bucket is a contiguous slice of `flat_grad`, so it is reduced in place, without a copy.

    A parameter counts once per backward, when its gradient is complete: from a
    post-accumulate-grad hook (the autograd engine sums every use of a leaf before its one
    AccumulateGrad call), or -- with in-place gradients (ops.GradSink, train_step) -- from
    `param_ready`, which the layers' backward calls after the last use's gradient is written.  When a bucket is complete its
    all-reduce is issued with async_op=True, which orders it after the gradient kernels already
    on the stream and lets the rest of backward run beside it.  Buckets are issued strictly in
    index order, so every rank issues the same collectives in the same order.  `finish()` issues
    whatever is left (parameters that got no gradient this step), waits for all of them (a
    stream wait, not a host sync, with the nccl/RCCL backend) and divides by the world size.

    Outside `armed()` the hooks do nothing, so other backward passes (tests, user code) never
    start a collective.

    Co-residency rule.  The decoder LSTMs' backward runs as persistent launches that
    need every CU at once (lstm_persist.hip: bptt_persist_kernel); an RCCL kernel waiting for a
    lagging peer must never hold CUs while one dispatches, or the launch's resident workgroups
    spin until their bounded wait gives up.  So (ops._lstm_bwd calls the two hooks):
      * `before_recurrence`: the compute stream waits for every collective issued so far (a
        stream wait with RCCL; no host sync), so none is in flight when the persistent grid
        dispatches;
      * while a decoder LSTM's backward is still to come, complete buckets are held back; the ones
        whose gradients were final before a recurrence are issued right after it, on a side
        stream behind the event the library records after the persistent launch
        (avc_persist_notify), so they run beside that layer's dX/dW GEMMs and the rest of the
        backward -- never beside a dispatch;
      * after the last recurrence, buckets are issued as soon as they are complete.
    `all_reduce` / `world` replace dist.all_reduce / the process group's size (tests: a collective
    stand-in that holds CUs, world 1); `co_residency=False` turns the rule off (tests only)."""

    def __init__(self, params, flat_grad: torch.Tensor, bucket_bytes: int = 16 << 20, all_reduce=None,
                 world_size: int | None = None, co_residency: bool = True):
        params = list(params)
        self.flat = flat_grad
        self._all_reduce = all_reduce if all_reduce is not None else (
            lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True))
        self._world = world_size
        self.co_residency = co_residency
        self._side = None
        self._event = None
        base = flat_grad.data_ptr()
        spans = []
        for p in params:
            if p.grad is None:
                raise ValueError("GradBuckets needs every parameter's .grad to be a view of the flat gradient")
            off = (p.grad.data_ptr() - base) // flat_grad.element_size()
            spans.append((off, p.numel()))
        if any(spans[i][0] + spans[i][1] != spans[i + 1][0] for i in range(len(spans) - 1)):
            raise ValueError("parameter gradients are not consecutive slices of the flat gradient")
        per = max(1, bucket_bytes // flat_grad.element_size())
        self.buckets = []           # (lo, hi) element ranges, in launch order
        self.bucket_of = [0] * len(params)
        members = []
        hi, size = None, 0
        for i in reversed(range(len(params))):
            off, n = spans[i]
            if hi is None:
                hi, size, cur = off + n, 0, []
            cur.append(i)
            size += n
            if size >= per or i == 0:
                self.buckets.append((off, hi))
                members.append(cur)
                hi = None
        for b, idx in enumerate(members):
            for i in idx:
                self.bucket_of[i] = b
        self.sizes = [len(m) for m in members]
        self._armed = False
        self._index = {id(p): i for i, p in enumerate(params)}
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i)) for i, p in enumerate(params)]
        self.reset()

    def reset(self, recurrences: int = 0):
        self.pending = list(self.sizes)
        self.next = 0
        self.handles = []
        self.fenced = 0             # handles the compute stream already waits for
        self.seen = set()
        self.launch_log = []        # (bucket, parameters still pending overall) per issue
        self.recurrences_left = recurrences if self.co_residency else 0
        self._behind = 0
        self._launches0 = 0

    def _ready(self, i):
        if not self._armed or i in self.seen:
            return
        self.seen.add(i)
        self.pending[self.bucket_of[i]] -= 1
        self._issue(ready_only=True)

    def _make_hook(self, i):
        def hook(_p):
            self._ready(i)
        return hook

    def param_ready(self, p):
        """A parameter's gradient is complete (in-place gradients, ops.GradSink: the layers write
        `p.grad` themselves, so autograd's accumulate hooks never run)."""
        i = self._index.get(id(p))
        if i is not None:
            self._ready(i)

    def _complete_run(self):
        """Complete buckets from `next` on, in issue order."""
        n = 0
        while self.next + n < len(self.buckets) and self.pending[self.next + n] <= 0:
            n += 1
        return n

    def _issue_n(self, n):
        for _ in range(n):
            lo, hi = self.buckets[self.next]
            self.launch_log.append((self.next, sum(max(0, c) for c in self.pending)))
            self.handles.append(self._all_reduce(self.flat[lo:hi]))
            self.next += 1

    def _issue(self, ready_only):
        if not ready_only:
            self._issue_n(len(self.buckets) - self.next)
        elif self.recurrences_left <= 0:  # held back while a persistent backward is still to come
            self._issue_n(self._complete_run())

    def before_recurrence(self):
        """A decoder LSTM backward (possibly a persistent launch) is about to be enqueued."""
        if not self._armed or not self.co_residency:
            return
        for h in self.handles[self.fenced:]:
            h.wait()
        self.fenced = len(self.handles)
        self._behind = self._complete_run()  # final before the recurrence starts
        dev = self.flat.device
        if dev.type == "cuda":
            from . import _lib
            if self._event is None:
                self._side = torch.cuda.Stream(device=dev)
                self._event = torch.cuda.Event()
                self._event.record(torch.cuda.current_stream(dev))  # creates the HIP event
            _lib.call("avc_persist_notify", _lib.context(dev), self._event.cuda_event)
            self._launches0 = _lib.persist_launches(dev)

    def after_recurrence(self, left: int):
        """The decoder LSTM backward is enqueued; `left` of them are still to come."""
        if not self._armed or not self.co_residency:
            return
        self.recurrences_left = left
        dev = self.flat.device
        fired = False
        if dev.type == "cuda":
            from . import _lib
            fired = _lib.persist_launches(dev) > self._launches0
            _lib.call("avc_persist_notify", _lib.context(dev), None)
        if self._behind and fired:
            # behind the persistent launch: beside the layer's dX / dW products, not its dispatch
            self._side.wait_event(self._event)
            with torch.cuda.stream(self._side):
                self._issue_n(self._behind)
        else:
            self._issue_n(self._behind)
        self._behind = 0
        self._issue(ready_only=True)

    def armed(self, recurrences: int = 0):
        """Context for one backward; `recurrences` = decoder LSTM backwards it will run."""
        outer = self

        class _Arm:
            def __enter__(self):
                outer.reset(recurrences)
                outer._armed = True
                return outer

            def __exit__(self, *exc):
                outer._armed = False
                if outer.flat.device.type == "cuda":
                    from . import _lib
                    _lib.call("avc_persist_notify", _lib.context(outer.flat.device), None)
                return False
        return _Arm()

    def finish(self) -> torch.Tensor:
        self._issue(ready_only=False)
        for h in self.handles:
            h.wait()
        self.handles = []
        self.flat.div_(self._world if self._world is not None else world())
        return self.flat

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


def broadcast_buffers(module: torch.nn.Module, src: int = 0) -> None:
    """Make every rank's BN running statistics equal to rank `src`'s (before saving)."""
    if world() > 1:
        for b in module.buffers():
            dist.broadcast(b, src)


def params_in_sync(flat_param: torch.Tensor) -> bool:
    """True when every rank holds bitwise the same parameters (max/min all-reduce of a checksum)."""
    if world() == 1:
        return True
    v = flat_param.detach().double()
    ck = torch.stack([v.sum(), (v * v).sum(), v.abs().max()]).to(collective_device())
    lo, hi = ck.clone(), ck.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return bool(torch.equal(lo, hi))


def collective_device() -> torch.device:
    """Where the default process group's tensors must live: the current GPU for nccl (RCCL has
    no CPU backend), the CPU for gloo."""
    if world() > 1 and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def broadcast_seed(src: int = 0) -> int:
    """A 63-bit seed drawn from rank `src`'s torch RNG, the same on every rank."""
    seed = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64)
    if world() > 1:
        seed = seed.to(collective_device())
        dist.broadcast(seed, src)
    return int(seed.item())


def shard_loader(loader, seed: int | None = None):
    """The caller's DataLoader (voice_converter.py:282-285 builds it: dataloader.py:123-144,
    batch_size utterances per batch, shuffle=True, zero-padding collate_fn) re-built over a
    DistributedSampler: rank r loads only its own 1/world of the utterances, in batches of the
    same batch_size (the per-GPU batch of BASELINE config 4), every rank runs the same number of
    steps (drop_last on the shard), and all ranks draw their shuffles from one seed broadcast from
    rank 0 (call set_epoch(epoch) on the returned loader's sampler each epoch, as learn() does).
    World 1: the loader itself."""
    from torch.utils.data import DataLoader, DistributedSampler, RandomSampler
    if world() == 1:
        return loader
    if not isinstance(loader, DataLoader) or loader.batch_size is None:
        raise TypeError("data-parallel learn() needs a torch DataLoader with a batch_size (dataloader.py:137)")
    seed = broadcast_seed() if seed is None else seed
    sampler = DistributedSampler(loader.dataset, num_replicas=world(), rank=rank(),
                                 shuffle=isinstance(loader.sampler, RandomSampler), seed=seed, drop_last=True)
    # everything but the sampler as the caller built it
    extra = dict(worker_init_fn=loader.worker_init_fn, generator=loader.generator, timeout=loader.timeout,
                 multiprocessing_context=loader.multiprocessing_context)
    if loader.num_workers > 0:
        extra.update(persistent_workers=loader.persistent_workers, prefetch_factor=loader.prefetch_factor)
    return DataLoader(loader.dataset, batch_size=loader.batch_size, sampler=sampler,
                      collate_fn=loader.collate_fn, num_workers=loader.num_workers,
                      pin_memory=loader.pin_memory, drop_last=loader.drop_last, **extra)


def set_epoch(loader, epoch: int) -> None:
    from torch.utils.data import DistributedSampler
    if isinstance(getattr(loader, "sampler", None), DistributedSampler):
        loader.sampler.set_epoch(epoch)


def shard_indices(n: int, r: int | None = None, ws: int | None = None) -> range:
    """Contiguous, equal-size shard of n utterance minibatches for rank r (drops the remainder
    so every rank runs the same number of steps, as the collective requires)."""
    r = rank() if r is None else r
    ws = world() if ws is None else ws
    per = n // ws
    return range(r * per, (r + 1) * per)
