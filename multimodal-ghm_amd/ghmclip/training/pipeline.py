"""Host sampler -> HBM pipeline: the native GHM sampler runs in a producer
thread one or more batches ahead, writing uint8 leaves into a ring of pinned
host buffers; the training stream copies a slot to the device with an async
H2D copy and records an event that releases the slot back to the producer.
(the sampler stays on the host, overlapped with compute.)
"""
import threading

import numpy as np
import torch


def _host_buffer(shape, dtype):
    """A page-locked host buffer for the async H2D copies (plain memory when no
    device is present: the producer side is tested on the CPU)."""
    t = torch.empty(*shape, dtype=dtype)
    return t.pin_memory() if torch.cuda.is_available() else t


def shard_rows(block_rows, n_blocks, rank, world):
    """Row indices rank `rank` of `world` keeps from a CLIP batch laid out as
    n_blocks blocks of block_rows rows: a contiguous slice of the within-block
    index i in every block (the loss is a mean over i, model.py:906-907, and
    each term only touches rows {b*B + i}), so shard losses / gradients average
    to the full-batch ones."""
    if block_rows % world:
        raise ValueError("block rows must divide by the world size")
    per = block_rows // world
    return np.concatenate([np.arange(k * block_rows + rank * per, k * block_rows + (rank + 1) * per)
                           for k in range(n_blocks)])


def shard_samples(batch_size, rank, world):
    """(start, stop) of the samples rank `rank` of `world` keeps from a CDM batch:
    a contiguous 1/world of the rows (the CDM loss is a mean over samples,
    model.py:998, so shard gradients average to the full-batch ones)."""
    if batch_size % world:
        raise ValueError("batch size must divide by the world size")
    per = batch_size // world
    return rank * per, (rank + 1) * per


class BatchPipeline:
    def __init__(self, native_sampler, batch_size, n_slots=3, row_slice=None):
        """native_sampler: data.NativeClipSampler whose MT state is already set.
        row_slice: optional (block_rows, rank, world): keep this rank's shard of
        every block (see shard_rows; data-parallel sharding)."""
        self.s = native_sampler
        self.B = batch_size
        self.slice = row_slice
        self._make_slots(n_slots)
        self.free = [threading.Event() for _ in range(n_slots)]
        self.ready = [threading.Event() for _ in range(n_slots)]
        self.copy_done = [None] * n_slots
        for f in self.free:
            f.set()
        self.n = n_slots
        self.stop = False
        self.err = None
        self.k_prod = 0
        self.k_cons = 0
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    # -- CLIP batches: text / image leaves [B(K+1), T] uint8 ------------------------
    def _make_slots(self, n_slots):
        rows = self.B * (self.s.K + 1)
        Tt, Ti = self.s.T_t, self.s.T_i  # text / image sequence lengths (trees may differ)
        self.full_rows, self.T = rows, self.s.T
        if self.slice is not None:  # this rank's shard only: (K+1) * B/world rows
            br, rank, world = self.slice
            if br != self.B or br % world:
                raise ValueError("row_slice must be (batch_size, rank, world) with world | batch_size")
            self.shard_lo, self.shard_n = rank * (br // world), br // world
            rows = (self.s.K + 1) * self.shard_n
        self.slots = [(_host_buffer((rows, Tt), torch.uint8), _host_buffer((rows, Ti), torch.uint8))
                      for _ in range(n_slots)]

    def _fill(self, i):
        """One draw of the global batch (the MT stream advances by all of it; only
        this rank's rows are expanded: ghm_sampler_next_shard == shard_rows of the
        full draw)."""
        t, im = self.slots[i]
        if self.slice is not None:
            self.s.next_shard_into(self.B, self.shard_lo, self.shard_n, t.numpy(), im.numpy())
        else:
            self.s.next_into(self.B, t.numpy(), im.numpy())

    def _stage(self, trainer, i):
        t, im = self.slots[i]
        trainer.set_tokens(t, im)

    def _run(self):
        try:
            while not self.stop:
                i = self.k_prod % self.n
                self.free[i].wait()
                if self.stop:
                    return
                ev = self.copy_done[i]
                if ev is not None:
                    ev.synchronize()  # the previous H2D copy out of this slot is done
                self.free[i].clear()
                self._fill(i)
                self.ready[i].set()
                self.k_prod += 1
        except Exception as e:  # surfaced on the consumer side
            self.err = e
            for r in self.ready:
                r.set()

    def next_into(self, trainer):
        """Wait for the next batch and enqueue its H2D copy on the current stream."""
        i = self.k_cons % self.n
        self.ready[i].wait()
        if self.err is not None:
            raise self.err
        self.ready[i].clear()
        self._stage(trainer, i)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self.copy_done[i] = ev
        self.free[i].set()
        self.k_cons += 1

    def close(self):
        self.stop = True
        for f in self.free:
            f.set()
        self.th.join(timeout=5)


class CdmBatchPipeline(BatchPipeline):
    """The same producer for ConditionalDenoiseSampler draws (text leaves, image
    leaves uint8 [B, T], noisy observations z float64 [B, T]).  row_slice:
    optional (rank, world) — keep a contiguous 1/world of the samples (the CDM
    loss is a mean over samples, model.py:998)."""

    def __init__(self, native_sampler, batch_size, sigma, n_slots=3, row_slice=None):
        self.sigma = float(sigma)
        super().__init__(native_sampler, batch_size, n_slots, row_slice)

    def _make_slots(self, n_slots):
        B, Tt, Ti = self.B, self.s.T_t, self.s.T_i
        self.T = self.s.T

        def slot():
            return (_host_buffer((B, Tt), torch.uint8), _host_buffer((B, Ti), torch.uint8),
                    _host_buffer((B, Ti), torch.float64))
        self.slots = [slot() for _ in range(n_slots)]
        if self.slice is not None:
            self.rows = shard_samples(B, *self.slice)

    def _fill(self, i):
        t, im, z = self.slots[i]
        self.s.next_cdm_into(self.B, self.sigma, t.numpy(), im.numpy(), z.numpy())

    def _stage(self, trainer, i):
        t, im, z = self.slots[i]
        if self.slice is not None:
            a, b = self.rows
            t, im, z = t[a:b], im[a:b], z[a:b]
        trainer.set_batch(t, im, z)


class NwpBatchPipeline(BatchPipeline):
    """The same producer for NextWordPredictSampler draws: text inputs / targets
    uint8 [B, T-1], the exact next-word posteriors float32 [B, T-1, V] (host BP,
    bp_nwp_posterior) and image leaves uint8 [B, T]; guide=True also the packed
    BP guide targets float32 [B, n] (vlm_guide_planes: train_NWP.py --guide=True;
    image_guide=False packs the text blocks only: train_sequential_NWP.py, whose
    image guides target the CLIP feature on the device).
    sampler: the NextWordPredictSampler (its native MT state already pulled from
    numpy).  row_slice: optional (rank, world) — a contiguous 1/world of the
    samples (the VLM loss is a mean over samples, model.py:1087-1098)."""

    def __init__(self, sampler, batch_size, n_slots=3, row_slice=None, guide=False, image_guide=True):
        self.sampler = sampler
        self.guide = guide
        self.image_guide = image_guide
        super().__init__(sampler.native, batch_size, n_slots, row_slice)

    def _make_slots(self, n_slots):
        B, T, Ti, V = self.B, self.s.T_t, self.s.T_i, self.sampler.variable_type
        self.T = T
        L = self.sampler.n_layers
        ng = (T - 1) * V * (3 * L[0] + 1) + (Ti * V * L[1] if self.image_guide else 0) if self.guide else 0

        def slot():
            return (_host_buffer((B, T - 1), torch.uint8), _host_buffer((B, T - 1), torch.uint8),
                    _host_buffer((B, T - 1, V), torch.float32), _host_buffer((B, Ti), torch.uint8),
                    _host_buffer((B, ng), torch.float32) if ng else None)
        self.slots = [slot() for _ in range(n_slots)]
        self.tl = np.empty((B, T), np.uint8)
        self.root = np.empty(B, np.uint8)
        if self.slice is not None:
            self.rows = shard_samples(B, *self.slice)

    def _fill(self, i):
        from ..data.data_random_GHM import vlm_guide_planes
        xt, yt, post, il, gt = self.slots[i]
        tl = self.tl
        self.s.next_cdm_into(self.B, 0.0, tl, il.numpy(), None, self.root)
        xt.numpy()[:] = tl[:, :-1]
        yt.numpy()[:] = tl[:, 1:]
        if self.guide:
            p, _, tg, ig = self.sampler.posterior(tl, il.numpy(), guide=True)
            post.numpy()[:] = p
            vlm_guide_planes(tg, ig if self.image_guide else [], self.sampler.variable_type, out=gt.numpy())
        else:
            post.numpy()[:] = self.sampler.posterior(tl, il.numpy())[0]

    def _stage(self, trainer, i):
        xt, yt, post, il, gt = self.slots[i]
        if self.slice is not None:
            a, b = self.rows
            xt, yt, post, il = xt[a:b], yt[a:b], post[a:b], il[a:b]
            gt = None if gt is None else gt[a:b]
        trainer.set_batch(xt, yt, post, il, *(() if gt is None else (gt,)))
