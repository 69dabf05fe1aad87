"""Fused CLIP training step on the HIP path — the hot loop of
src/ghmclip/training/train_CLIP.py:139-167 (zero_grad, sample, 2 encoder
forwards, GuidedClipLoss, backward, clip_grad_norm_, cosine LR, AdamW).

Design:
* both encoders' parameters live in ONE flat fp32 buffer (each nn.Parameter is a
  view into it), likewise gradients and the AdamW moments, so the clip and the
  optimizer are two launches over 1.84 M floats;
* every per-step scalar (lr_t, lr*wd) comes from a device table indexed by a
  device step counter, so the whole step is a static launch sequence that is
  captured once (one linear HIP graph per phase and tower) and replayed;
* the loss of every step is written on device into ``hist`` (no host sync per
  step; the host reads it at log intervals);
* data parallel (optional): each rank owns a shard of the within-block index i
  (the loss is a mean over i, model.py:906-907), grads are averaged by two
  bucketed RCCL all-reduces of the flat buffer (top layers while the lower
  layers' backward runs, then the rest) before the optimizer.
"""
import ctypes
import weakref
import os

import numpy as np
import torch

from .. import _native
from . import distributed
from ..data.data_random_GHM import DeviceTree
from ..models.gemm_encoder import make_encoder_plan
from ..models.hip_encoder import ENCODER_PRECISIONS, default_precision, require_hip
from ..models.optimizer import adam_consts, adam_lr_t


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _layer_of(name):
    """Encoder layer of a parameter name (_queries.3.weight, _mlps.3.0.bias,
    _lns_1.3.weight -> 3), None for the embeddings and readout."""
    parts = name.split(".")
    if parts[0] in ("_queries", "_keys", "_values", "_mlps", "_lns_1", "_lns_2") and len(parts) > 1:
        return int(parts[1])
    return None


def flat_layout(models, dp_top):
    """Offsets of every parameter of the towers in the flat buffers: [text
    tower][image tower], each in BACKWARD order (layer L-1's parameters first,
    ..., layer 0's, then the embeddings and the readout), so the gradients that
    are final once the backward of the top dp_top layers has run form one
    contiguous range per tower (data-parallel bucket A).  state_dict order is
    unchanged: the module parameters become views.
    Returns ([{name: (offset, numel)} per tower], [(start, end) of bucket A per
    tower], total numel)."""
    layout, bucket_a, off = [], [], 0
    for m in models:
        # each tower starts 16-byte aligned (the GEMM-path kernels read the embedding
        # tables and biases as float4; a tower's parameters are multiples of 4 floats
        # up to its readout, whose n_token + num_class + 1 floats may not be: n_token = 64
        # of the reference's default 3-layer, 4-child trees).  The gap stays zero.
        off = -(-off // 4) * 4
        top = min(dp_top, m.n_layer)  # a tower may have fewer layers than the text tower
        named = dict(m.named_parameters())
        order = [n for l in reversed(range(m.n_layer)) for n in named if _layer_of(n) == l]
        order += [n for n in named if _layer_of(n) is None]
        slots, start, a_end = {}, off, off
        for name in order:
            k = named[name].numel()
            slots[name] = (off, k)
            off += k
            ly = _layer_of(name)
            if ly is not None and ly >= m.n_layer - top:
                a_end = off
        layout.append(slots)
        bucket_a.append((start, a_end))
    return layout, bucket_a, off


def dp_bucket_ranges(bucket_a, n):
    """([bucket A ranges], [bucket B ranges]) of a flat gradient of n elements
    laid out by flat_layout: A = the top layers of each tower, B = the rest of
    each tower (the image tower starts where the text tower ends).  Together
    they cover [0, n) exactly once."""
    (ta, tb), (ia, ib) = bucket_a
    a = [(ta, tb), (ia, ib)]
    b = [(tb, ia), (ib, n)]
    return [r for r in a if r[1] > r[0]], [r for r in b if r[1] > r[0]]


def _destroy_events(evs):
    lib = _native.hip_lib()
    for ev in evs.values():
        lib.ghm_event_destroy(ev)
    evs.clear()


class ClipTrainer:
    def __init__(self, tmodel, imodel, K, batch_size, lr_schedule, max_norm=1.0, weight_decay=0.001,
                 betas=(0.9, 0.999), eps=1e-8, device="cuda", t_offset=0, process_group=None,
                 precision=None, penalty=1e-3, guide_trans=None):
        """lr_schedule: sequence of python-float learning rates, one per step
        (get_lr_cosine_schedule(i, ...) for i in range(total_iters+1)).
        precision: "f32" (exact-f32 MFMA), "x3" (split-bf16 MFMA) or "f32fwd" (the
        LN + projection and LN + MLP forwards exact f32, the rest split-bf16;
        n_embd = 128); None -> $GHM_PRECISION, else "x3" (unguided) / "f32fwd"
        (guided: the guided run amplifies the split products' 2^-17 rounding in
        the forward 20x past an f32 path's, which sits at the level of any one-ulp
        perturbation of the reference's own arithmetic, while split-bf16 gradients
        and attention stay inside the reference's spread).
        Guided CLIP (train_CLIP.py --clip_guide=True) is on when the encoders were
        built with guide=True: guide_trans = (text, image) transition templates
        [L][C][V][V] (ClipSampler.t_templ / i_templ) for the on-device BP guide
        targets, penalty = GuidedClipLoss's penalty."""
        self.device = torch.device(device)
        self.tm, self.im = tmodel, imodel
        self.K, self.B = K, batch_size
        self.max_norm = float(max_norm)
        self.pg = process_group
        self.models = [tmodel, imodel]
        params = [p for m in self.models for p in m.parameters()]
        for p in params:
            require_hip(p)
        L0 = max(m.n_layer for m in self.models)
        # layers in bucket A (clamped per tower in flat_layout / _bwd_a_gen)
        self.dp_top = int(os.environ.get("GHM_DP_BUCKET_LAYERS", str(L0 - L0 // 2)))
        self.dp_top = max(0, min(L0, self.dp_top))
        layout, self.bucket_a, n = flat_layout(self.models, self.dp_top)
        self.n_params = n  # (with the zero gap that aligns the image tower, if any)
        self.pflat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.gflat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.mflat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.vflat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.views = []  # per model: (param dict, grad dict, m dict, v dict)
        with torch.no_grad():
            for m, slots in zip(self.models, layout):
                named = dict(m.named_parameters())
                pd, gd, md, vd = {}, {}, {}, {}
                for name in named:  # views keyed in the module's own order (the plans look names up)
                    off, k = slots[name]
                    p = named[name]
                    self.pflat[off:off + k].copy_(p.data.reshape(-1))
                    p.data = self.pflat[off:off + k].view(p.shape)
                    p.grad = self.gflat[off:off + k].view(p.shape)
                    pd[name], gd[name] = p.data, p.grad
                    md[name] = self.mflat[off:off + k].view(p.shape)
                    vd[name] = self.vflat[off:off + k].view(p.shape)
                self.views.append((pd, gd, md, vd))
        T = tmodel.n_token
        n_seq = batch_size * (K + 1)
        if precision is None:
            precision = default_precision("f32fwd" if all(getattr(m, "guide", False) for m in self.models) else "x3",
                                          allowed=ENCODER_PRECISIONS)
        if any(m.n_embd != 128 for m in self.models) and all(getattr(m, "guide", False) for m in self.models):
            raise NotImplementedError("guided CLIP runs at n_embd = 128 (the guide kernels' row pitch)")
        # n_embd = 128: the fused token-parallel kernels; other widths (the reference
        # CLI's default 64): the GEMM path (models/gemm_encoder.py, split-bf16)
        self.plans = [make_encoder_plan(m.n_layer, m.n_token, n_seq, num_class=m.vocab_size, vocab=m.vocab_size,
                                        n_embd=m.n_embd, normalize_attn=m.normalize_attn, device=self.device,
                                        precision=precision, activation=getattr(m, "activation", "softmax"),
                                        defer_reduce=os.environ.get("GHM_DEFER_REDUCE", "1") != "0")
                      for m in self.models]
        self.precision = self.plans[0].precision
        self.T, self.n_seq = T, n_seq
        self.C = tmodel.vocab_size
        # optimizer constants and the per-step schedule table
        self.betas, self.wd = betas, weight_decay
        self.consts = adam_consts(betas, eps)
        self.t_offset = t_offset
        sched = np.zeros((len(lr_schedule), 2), dtype=np.float32)
        for s, lr in enumerate(lr_schedule):
            sched[s, 0] = adam_lr_t(lr, s + 1 + t_offset, betas)
            sched[s, 1] = lr * weight_decay
        self.lr_schedule = list(lr_schedule)
        self.sched = torch.from_numpy(sched.reshape(-1)).to(self.device)
        self.n_sched = len(lr_schedule)
        self.step_ctr = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.hyper = torch.zeros(4, dtype=torch.float32, device=self.device)
        self.work = torch.zeros(1024, dtype=torch.float32, device=self.device)
        self.hist = torch.zeros(max(1, len(lr_schedule)), dtype=torch.float32, device=self.device)
        self.graphs = None
        self.steps_done = 0
        self.side = torch.cuda.Stream(device=self.device)
        self.comm = torch.cuda.Stream(device=self.device)  # data-parallel bucket all-reduces
        # one process: reduce the top dp_top layers' partials on the (otherwise idle)
        # comm stream while the towers run their lower layers, instead of all of
        # them in the serial tail after the last layer (GHM_EARLY_REDUCE=0: tail
        # only).  Tail 163 -> 116 us (tl_r4ab6 / tl_r4ab7e), step unchanged (r4_ab7).
        self.early_reduce = os.environ.get("GHM_EARLY_REDUCE", "1") == "1"
        # cross-stream waits on native events without the system-scope fence
        # (ghm_event_create mode 2; 1 = device-scope release, 0 = torch's
        # Stream.wait_stream): a just-in-time wait costs 10.8 instead of 12.7 us of
        # idle queue, a satisfied one 5.7 (tools/xq_latency.py, profiles/r4_xq_report.txt)
        self.fast_events = int(os.environ.get("GHM_FAST_EVENTS", "2"))
        self._evs = {}
        self._ev_fin = None
        # data-parallel timing (bench.py): None, or a list that each step appends
        # (bucket A ms, bucket B ms, exposed ms) event triples to
        self.comm_timing = None
        self._bwd_it = [None, None]  # the towers' running backward launch generators
        self._pending = []  # started data-parallel collectives (distributed.allreduce_ranges_start)
        self._bucket_checked = [False, False]
        self._setup_guide(penalty, guide_trans)

    def _setup_guide(self, penalty, guide_trans):
        """Buffers of the guided objective (model.py:909-924): per-tower BP
        messages [N][n_nodes][V], per-(tower, guided layer) penalty partials, and
        the penalised loss history (train_CLIP.py ploss_history)."""
        flags = [getattr(m, "guide", False) for m in self.models]
        self.guide = all(flags)
        if any(flags) and not self.guide:
            raise ValueError("both encoders must be built with the same guide setting")
        self.loss_out = torch.zeros(3, dtype=torch.float32, device=self.device)
        self.phist = None
        if not self.guide:
            return
        if guide_trans is None:
            raise ValueError("guided CLIP needs guide_trans=(sampler.t_templ, sampler.i_templ)")
        self.penalty = float(penalty)
        self.glayers, self.gtrans, self.gmsgs, self.gtree = [], [], [], []
        for m, tr in zip(self.models, guide_trans):
            dt = DeviceTree.of(tr)  # templates, or per-edge tables (non-translation-invariant trees)
            tr, L, C, V = dt.trans, dt.L, dt.C, dt.V
            if C ** L != m.n_token or V != m.vocab_size:
                raise ValueError("guide transitions do not match the encoder's token count / vocabulary")
            layers = [l for l, f in enumerate(m.guided_layer_flag) if f]
            if len(layers) > L:
                raise ValueError("more guided layers than tree levels")
            n_total = (C ** L - 1) // (C - 1)
            self.glayers.append(layers)
            self.gtree.append((L, C, V, dt.per_edge))
            self.gtrans.append(torch.from_numpy(tr).to(self.device))
            self.gmsgs.append(torch.zeros(self.n_seq, n_total, V, dtype=torch.float32, device=self.device))
        self.n_gparts = sum(len(x) for x in self.glayers)
        self.gpart = torch.zeros(max(1, self.n_gparts), self.n_seq, dtype=torch.float32, device=self.device)
        self.phist = torch.zeros_like(self.hist)

    def _guide_fwd(self, tower, s):
        """BP guide targets from the staged tokens, then the penalty partials of
        the tower's guided layers (after its forward)."""
        L, C, V, per_edge = self.gtree[tower]
        plan = self.plans[tower]
        base = sum(len(x) for x in self.glayers[:tower])
        _native.call("ghm_bp_cls", _p(self.gtrans[tower]), _p(plan.tokens), _p(self.gmsgs[tower]), self.n_seq,
                     L, C, V, per_edge, s)
        for k, l in enumerate(self.glayers[tower]):
            _native.call("ghm_guide_fwd", _p(plan.H[l + 1]), _p(self.gmsgs[tower]), _p(self.gpart[base + k]),
                         self.n_seq, L, C, V, k, s)

    def _guide_hooks(self, tower):
        """{layer: fn(dH, stream)} adding d(penalty)/dH_{l+1} = 2 p (H - target) / N."""
        if not self.guide:
            return None
        L, C, V, _ = self.gtree[tower]
        plan = self.plans[tower]
        msgs = self.gmsgs[tower]
        scale = 2.0 * self.penalty / self.n_seq
        hooks = {}
        for k, l in enumerate(self.glayers[tower]):
            def fn(dH, s, l=l, k=k):
                _native.call("ghm_guide_bwd", _p(plan.H[l + 1]), _p(msgs), _p(dH), self.n_seq, L, C, V, k,
                             scale, s)
            hooks[l] = fn
        return hooks

    # -- the launch sequence -----------------------------------------------------
    # A step is a fixed sequence of phases; the two towers' phases run on two
    # streams (text: the current stream, image: a side stream), joined by stream
    # waits:
    #   fwd(text) || fwd(image) -> bwd(text) || bwd(image) -> loss value + optim
    # (each tower's readout backward recomputes its rows of the loss gradient from
    # both towers' embeddings, so no loss kernel sits between the phases; data
    # parallel: bwd splits into bwd_a || bwd_a -> bucket A all-reduce on the comm
    # stream -> bwd_b || bwd_b -> bucket B -> optim)
    # A tower's phase is a generator of pieces (the embedding, each encoder
    # layer, the readout), and the two towers' pieces are issued alternately.
    # Captured, every piece is its own small linear graph, replayed in the same
    # alternation.  Why pieces: a HIP graph launch submits its kernel nodes from
    # the host one by one (~7.5 us each), so the stream whose graph is launched
    # second starts that much later: with the whole step in one two-branch graph
    # (rounds 2-3) or one graph per tower and phase, the second tower started
    # 120-250 us after the first in the forward and in the backward and ran its
    # last layers alone (profiles/r3_v6, r3_ab3; tools/timeline.py).
    def _tower_streams(self):
        """(current stream, text tower's stream, image tower's stream);
        GHM_SERIAL_TOWERS=1 puts both towers on the current stream.  (Tried and
        slower: each tower on its own CU-masked stream, hipExtStreamCreateWithCUMask
        over halves / alternate CUs: 4.2 -> 4.95 / 4.5 ms per step, profiles/r3_ab8.)"""
        main = torch.cuda.current_stream()
        if os.environ.get("GHM_SERIAL_TOWERS") == "1":
            return main, main, main
        return main, main, self.side

    def _fwd_gen(self, tower):
        """Forward of one tower (+ its guide targets and penalty partials) as
        pieces: embedding, each layer, readout (+ guide)."""
        plan, p = self.plans[tower], self.views[tower][0]
        for _ in plan.forward_iter(p):
            yield
        if self.guide:
            self._guide_fwd(tower, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))

    def _loss(self):
        """The loss value of the step (and the penalised one) into the histories.
        Runs on the comm stream once both forwards are done, off the towers'
        paths: each tower's readout backward recomputes its rows of the loss
        gradient from both towers' embeddings (ghm_readout_bwd_clip), which stay
        untouched until the next forward."""
        pt, pi = self.plans
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _native.call("ghm_clip_loss", _p(pt.emb), _p(pi.emb), None, None, _p(self.loss_out),
                     _p(self.hist), _p(self.step_ctr), self.B, self.K, self.C, s)
        if self.guide:
            _native.call("ghm_guide_total", _p(self.gpart), self.n_gparts, self.n_seq, self.penalty,
                         _p(self.loss_out), _p(self.phist), _p(self.step_ctr), s)

    def _bwd_a_gen(self, tower, flush):
        """Backward of one tower's readout and top dp_top layers as pieces; flush:
        reduce their parameter-gradient partials at the end (the data-parallel
        bucket A of this tower is final after it)."""
        plan = self.plans[tower]
        p, g = self.views[tower][0], self.views[tower][1]
        clip = (self.plans[0].emb, self.plans[1].emb, tower, self.B, self.K)
        it = plan.backward_iter(p, g, layer_grad=self._guide_hooks(tower), clip=clip)
        self._bwd_it[tower] = it
        top = min(self.dp_top, plan.L)  # the towers' layer counts may differ (clip_{t,i}model_nlayer)
        for k in range(1 + top):
            next(it)
            if k < top:
                yield  # (the last piece ends with the generator: no empty piece)
        if not self._bucket_checked[tower]:
            self._check_bucket_a(tower)
        if flush:
            plan.flush_pending()

    def _check_bucket_a(self, tower):
        """Bucket A of this tower (all-reduced while the lower layers' backward
        runs) must hold only gradients whose partials are queued by now, i.e.
        final once flush_pending() has run: every gradient view inside the bucket's
        flat range is a destination of a pending reduction job.  Checked on the
        first step (host only)."""
        a0, a1 = self.bucket_a[tower]
        base, esz = self.gflat.data_ptr(), self.gflat.element_size()
        in_a = {t.data_ptr() for t in self.views[tower][1].values()
                if a0 <= (t.data_ptr() - base) // esz < a1}
        queued = self.plans[tower].queued_grad_ptrs()
        missing = in_a - queued
        if missing:
            raise RuntimeError(f"data-parallel bucket A of tower {tower} holds {len(missing)} gradients that are "
                               "not final after its top layers' backward")
        self._bucket_checked[tower] = True

    def _bwd_b_gen(self, tower):
        """The rest of one tower's backward as pieces (lower layers; the last
        piece also runs the embeddings and the final partial reductions)."""
        for _ in self._bwd_it[tower]:
            yield

    def _phase(self, genf, graphs=None, key=None, fork=True, join=True):
        """Run a two-tower phase: the pieces of genf(1) (image, side stream) and
        genf(0) (text, current stream) alternately, joined back into the current
        stream; graphs: replay the captured piece graphs[(key, tower)] instead.
        fork / join = False: the caller orders the streams itself (_cross_wait)."""
        main, s0, s1 = self._tower_streams()
        st = {1: s1, 0: s0}
        for x in (s0, s1):
            if x != main and fork:
                self._order(main, x, "fork")
        if graphs is None:
            live = {1: genf(1), 0: genf(0)}
            while live:
                for t in (1, 0):
                    if t in live:
                        with torch.cuda.stream(st[t]):
                            try:
                                next(live[t])
                            except StopIteration:
                                del live[t]
        else:
            pieces = {t: graphs[(key, t)] for t in (1, 0)}
            for i in range(max(len(v) for v in pieces.values())):
                for t in (1, 0):
                    if i < len(pieces[t]):
                        with torch.cuda.stream(st[t]):
                            pieces[t][i].replay()
        for x in (s0, s1):
            if x != main and join:
                self._order(x, main, "join")

    def _event(self, key):
        ev = self._evs.get(key)
        if ev is None:
            if self._ev_fin is None:  # destroy the native events with the trainer (or at close())
                self._ev_fin = weakref.finalize(self, _destroy_events, self._evs)
                self._ev_fin.atexit = False  # not from interpreter shutdown (the HIP runtime may be gone)
            ev = _native.hip_lib().ghm_event_create(self.fast_events)
            if not ev:
                _native.check(-1, "ghm_event_create")
            self._evs[key] = ev = ctypes.c_void_p(ev)
        return ev

    def close(self):
        """Release the native cross-stream events (also done when the trainer is
        garbage collected)."""
        if self._ev_fin is not None:
            self._ev_fin()

    def _order(self, producer, consumer, key):
        """consumer waits for the work enqueued on producer so far."""
        if producer == consumer:
            return
        if not self.fast_events:
            consumer.wait_stream(producer)
            return
        ev = self._event(key)
        _native.call("ghm_event_record", ev, ctypes.c_void_p(producer.cuda_stream))
        _native.call("ghm_stream_wait", ctypes.c_void_p(consumer.cuda_stream), ev)

    def _cross_wait(self):
        """Each tower's stream waits for the other's work so far (one hop each way,
        concurrently) -- between the forward and the backward, where each tower's
        readout backward needs both towers' embeddings; a join into the current
        stream and a fork back out would put two hops in series on the side stream."""
        _, s0, s1 = self._tower_streams()
        if s0 == s1:
            return
        if self.fast_events:
            e0, e1 = self._event("cross0"), self._event("cross1")
            _native.call("ghm_event_record", e0, ctypes.c_void_p(s0.cuda_stream))
            _native.call("ghm_event_record", e1, ctypes.c_void_p(s1.cuda_stream))
            _native.call("ghm_stream_wait", ctypes.c_void_p(s0.cuda_stream), e1)
            _native.call("ghm_stream_wait", ctypes.c_void_p(s1.cuda_stream), e0)
            return
        e0, e1 = torch.cuda.Event(), torch.cuda.Event()
        e0.record(s0)
        e1.record(s1)
        s0.wait_event(e1)
        s1.wait_event(e0)

    def _single(self, fn, graphs=None, key=None):
        if graphs is None:
            fn()
        else:
            graphs[key].replay()

    def _early(self):
        """Early reduce of the upper layers' partials (one process, two streams)."""
        _, s0, s1 = self._tower_streams()
        return self.early_reduce and s0 != s1 and self.dp_top > 0

    def _bwd_gen(self, tower):
        """The whole backward of one tower as pieces (one process: no bucket
        boundary, so no join of the two towers in the middle of the backward)."""
        yield from self._bwd_a_gen(tower, flush=False)
        yield
        yield from self._bwd_b_gen(tower)

    def _run(self, graphs=None):
        """One step (eager, or by replaying `graphs` from _capture_graphs)."""
        dp = self._dp()
        # collectives a failed earlier step started and never finished must not be
        # waited for (and scaled) again by this one
        self._pending = []
        self._phase(self._fwd_gen, graphs, "fwd", join=False)
        self._cross_wait()
        # the loss value on the comm stream, off both towers' backward paths (the
        # embeddings stay untouched until the next forward)
        main, s0, _ = self._tower_streams()
        self._order(s0, self.comm, "loss")
        with torch.cuda.stream(self.comm):
            self._single(self._loss, graphs, "loss")
        # the schedule the graphs were captured with (bench.py replays them with the
        # towers on one stream, where _early() would say no)
        early = self._early() if graphs is None else ("flush", 0) in graphs
        if early:  # the upper layers' partials reduced on the comm stream, off the towers' paths
            self._phase(lambda t: self._bwd_a_gen(t, flush=False), graphs, "bwd_a", fork=False, join=False)
            _, s0, s1 = self._tower_streams()
            for t, st in ((1, s1), (0, s0)):  # each tower's upper partials, after its bwd_a, on the comm stream
                self._order(st, self.comm, ("early", t))
                with torch.cuda.stream(self.comm):
                    self._single(self.plans[t].flush_pending, graphs, ("flush", t))
        if early and not dp:
            # one join on the main stream's path: the comm stream (its early
            # reductions long done) waits for the side tower, the main stream for
            # the comm stream -- instead of two waits in series on the main stream
            self._phase(self._bwd_b_gen, graphs, "bwd_b", fork=False, join=False)
            _, _, s1 = self._tower_streams()
            self._order(s1, self.comm, "side_join")
            self._order(self.comm, torch.cuda.current_stream(), "early_join")
        elif not dp:
            self._phase(self._bwd_gen, graphs, "bwd", fork=False)
            self._order(self.comm, main, "loss_join")
        else:
            # data parallel, the same schedule: bucket A (the top layers' gradients,
            # final once both towers' upper partials are reduced) is all-reduced on the
            # comm stream right behind those reductions while the towers run their
            # lower layers; bucket B after the backward; the collectives are started
            # asynchronously (the host goes on issuing the towers' launches, with gloo
            # too) and waited for before the optimizer
            ev = [] if self.comm_timing is not None else None
            bucket_a, bucket_b = self.dp_buckets()
            if early:
                self._allreduce_async(bucket_a, ev)  # the comm stream already follows both towers
            else:
                self._phase(lambda t: self._bwd_a_gen(t, flush=True), graphs, "bwd_a", fork=False, join=False)
                self._allreduce_async(bucket_a, ev, after=self._tower_streams()[1:])
            self._phase(self._bwd_b_gen, graphs, "bwd_b", fork=False)
            main = torch.cuda.current_stream()
            self._allreduce_async(bucket_b, ev, after=(main,))
            with torch.cuda.stream(self.comm):
                distributed.allreduce_finish(self._pending)
            self._pending = []
            if ev is not None:  # exposed: the main stream's wait for the collectives after its backward
                ev.append(torch.cuda.Event(enable_timing=True))
                ev[-1].record(main)
            main.wait_stream(self.comm)
            if ev is not None:
                ev.append(torch.cuda.Event(enable_timing=True))
                ev[-1].record(main)
                self.comm_timing.append(ev)
        self._single(self._optim, graphs, "optim")

    def _optim(self):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        b1, omb1, b2, omb2, eps = self.consts
        _native.call("ghm_clip_prepare", _p(self.gflat), self.n_params, self.max_norm, _p(self.sched),
                     self.n_sched, _p(self.step_ctr), _p(self.hyper), _p(self.work), s)
        _native.call("ghm_adamw", _p(self.pflat), _p(self.gflat), _p(self.mflat), _p(self.vflat),
                     self.n_params, _p(self.hyper), b1, omb1, b2, omb2, eps, s)

    def dp_buckets(self):
        """([(start, end) of bucket A per tower], [... bucket B]) of the flat
        gradient: A = the top dp_top layers' gradients (final after the bwd_a phase),
        B = the rest."""
        return dp_bucket_ranges(self.bucket_a, self.n_params)

    def _allreduce_async(self, ranges, ev=None, after=()):
        """Start the mean over ranks of gflat[a:b] for each range on the comm stream,
        after the work already queued on the streams in `after`; the pending
        collectives are finished (waited for, scaled) before the optimizer.  ev
        (bench.py's timing mode): a list to append the bucket's start / end events
        on the comm stream to -- the bucket is then finished right away, so the
        end event follows the collective (the towers' streams run on either way)."""
        comm = self.comm
        for st in after:
            if st != comm:
                comm.wait_stream(st)
        with torch.cuda.stream(comm):
            if ev is not None:
                ev.append(torch.cuda.Event(enable_timing=True))
                ev[-1].record(comm)
            pend = distributed.allreduce_ranges_start(self.gflat, ranges, group=self.pg)
            if ev is not None:
                distributed.allreduce_finish(pend)
                pend = []
                ev.append(torch.cuda.Event(enable_timing=True))
                ev[-1].record(comm)
        self._pending += pend

    def comm_stats(self):
        """Per-step averages (ms) of the recorded data-parallel timing: bucket A
        and bucket B all-reduce durations on the comm stream, and the exposed
        part (the main stream waiting for the collectives once its backward is
        done).  Host sync."""
        torch.cuda.synchronize()
        rows = [(a0.elapsed_time(a1), b0.elapsed_time(b1), w0.elapsed_time(w1))
                for a0, a1, b0, b1, w0, w1 in self.comm_timing]
        if not rows:
            return None
        a, b, w = (sum(r[k] for r in rows) / len(rows) for k in range(3))
        return {"bucket_a_ms": round(a, 4), "bucket_b_ms": round(b, 4), "exposed_ms": round(w, 4),
                "steps": len(rows)}

    def _dp(self):
        return self.pg is not None or distributed.is_on()

    def set_tokens(self, t_tokens, i_tokens, alias=False):
        """Stage one batch (uint8 [n_seq, T] host-pinned or device tensors) into
        the plans' token buffers, async on the current stream (the side stream
        is ordered after it by the fork of each phase); the caller may reuse its
        tensors as soon as this returns (stream-ordered copies).  alias=True (the
        bench's HBM ring): an eager step reads a contiguous uint8 device tensor of
        the right shape in place instead -- no copy kernel at the head of the step
        -- and the caller must then leave the tensor unmodified until the step
        has completed on the GPU.  Graph replays always read the plans' own
        buffers, whose addresses the graphs hold."""
        for plan, t in ((self.plans[0], t_tokens), (self.plans[1], i_tokens)):
            own = plan.token_buf
            if (alias and self.graphs is None and t.device == own.device and t.dtype == torch.uint8
                    and t.is_contiguous() and t.shape == own.shape):
                plan.tokens = t
            else:
                plan.tokens = own
                own.copy_(t, non_blocking=True)

    def step(self):
        """One training step on the staged tokens (async; no host sync).  Data
        parallel: the all-reduce of bucket A (the top layers' gradients) runs on
        the comm stream while the rest of the backward runs; bucket B follows."""
        if self.steps_done >= self.n_sched:
            raise RuntimeError("schedule exhausted")
        self._run(self.graphs)
        self.steps_done += 1

    def _capture_graphs(self):
        """{(phase, tower): [piece graphs] | phase: graph}: every piece of every
        phase captured as its own linear graph (see the launch-sequence notes)."""
        graphs = {}
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        dp = self._dp()

        def one(fn):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                fn()
            return g

        def pieces(gen):
            out, done = [], False
            while not done:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    try:
                        next(gen)
                    except StopIteration:
                        done = True
                out.append(g)
            return out
        for t in (0, 1):
            graphs[("fwd", t)] = pieces(self._fwd_gen(t))
        graphs["loss"] = one(self._loss)
        if self._early():  # one process or data parallel: the same early-reduce schedule
            for t in (0, 1):
                graphs[("bwd_a", t)] = pieces(self._bwd_a_gen(t, flush=False))
                graphs[("flush", t)] = one(self.plans[t].flush_pending)
            for t in (0, 1):
                graphs[("bwd_b", t)] = pieces(self._bwd_b_gen(t))
        elif not dp:
            for t in (0, 1):
                graphs[("bwd", t)] = pieces(self._bwd_gen(t))
        else:
            for t in (0, 1):
                graphs[("bwd_a", t)] = pieces(self._bwd_a_gen(t, flush=True))
            for t in (0, 1):
                graphs[("bwd_b", t)] = pieces(self._bwd_b_gen(t))
        graphs["optim"] = one(self._optim)
        torch.cuda.current_stream().wait_stream(s)
        return graphs

    def capture(self, graphs=None):
        """Switch the step to replaying HIP piece graphs (call after >= 1 eager step
        so all lazy initialisation has happened; replays reuse the staged tokens)
        -- if graphs is True, or if graphs is None and GHM_GRAPH=1.  The default
        keeps the step eager: the host issues each kernel far ahead of the GPU, and
        every piece-graph launch costs its stream ~9 us of idle queue at the piece
        boundary (eager 4.014 vs piece graphs 4.052 ms per step, r4_ab13)."""
        if graphs is None:
            graphs = os.environ.get("GHM_GRAPH", "0") == "1"
        if graphs:
            for plan in self.plans:  # the graphs bake the token addresses: the plans' own buffers
                if plan.tokens is not plan.token_buf:
                    plan.token_buf.copy_(plan.tokens, non_blocking=True)
                    plan.tokens = plan.token_buf
        self.graphs = self._capture_graphs() if graphs else None

    # -- host-side views -----------------------------------------------------------
    def loss_history(self, upto=None):
        """Plain CLIP loss per step (train_CLIP.py loss_history, from loss_nop)."""
        n = self.steps_done if upto is None else upto
        return self.hist[:n].double().cpu().numpy()

    def ploss_history(self, upto=None):
        """Loss including the guided penalty (train_CLIP.py ploss_history); equals
        loss_history without guidance."""
        if self.phist is None:
            return self.loss_history(upto)
        n = self.steps_done if upto is None else upto
        return self.phist[:n].double().cpu().numpy()

    def fill_optimizer_state(self, optimizer):
        """Expose the flat moments as the reference AdamW's per-parameter state
        ('t', 'm', 'v'), e.g. before optimizer.state_dict() for a checkpoint."""
        t = self.steps_done + self.t_offset
        for m, (_, _, md, vd) in zip(self.models, self.views):
            for name, p in m.named_parameters():
                optimizer.state[p] = {"t": t, "m": md[name], "v": vd[name]}

    def load_optimizer_state(self, optimizer):
        with torch.no_grad():
            for m, (_, _, md, vd) in zip(self.models, self.views):
                for name, p in m.named_parameters():
                    st = optimizer.state.get(p)
                    if st:
                        md[name].copy_(st["m"])
                        vd[name].copy_(st["v"])
