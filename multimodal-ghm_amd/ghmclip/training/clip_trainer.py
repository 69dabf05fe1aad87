"""Fused CLIP training step on the HIP path — the hot loop of
src/ghmclip/training/train_CLIP.py:139-167 (zero_grad, sample, 2 encoder
forwards, GuidedClipLoss, backward, clip_grad_norm_, cosine LR, AdamW).

Design:
* both encoders' parameters live in ONE flat fp32 buffer (each nn.Parameter is a
  view into it), likewise gradients and the AdamW moments, so the clip and the
  optimizer are two launches over 1.84 M floats;
* every per-step scalar (lr_t, lr*wd) comes from a device table indexed by a
  device step counter, so the whole step is a static launch sequence that is
  captured once into a HIP graph and replayed;
* the loss of every step is written on device into ``hist`` (no host sync per
  step; the host reads it at log intervals);
* data parallel (optional): each rank owns a shard of the within-block index i
  (the loss is a mean over i, model.py:906-907), grads are averaged with one
  RCCL all-reduce of the flat buffer between the backward graph and the
  optimizer graph.
"""
import ctypes
import os

import numpy as np
import torch

from .. import _native
from . import distributed
from ..models.hip_encoder import EncoderPlan, require_hip
from ..models.optimizer import adam_consts, adam_lr_t


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


class ClipTrainer:
    def __init__(self, tmodel, imodel, K, batch_size, lr_schedule, max_norm=1.0, weight_decay=0.001,
                 betas=(0.9, 0.999), eps=1e-8, device="cuda", t_offset=0, process_group=None,
                 precision=None, penalty=1e-3, guide_trans=None):
        """lr_schedule: sequence of python-float learning rates, one per step
        (get_lr_cosine_schedule(i, ...) for i in range(total_iters+1)).
        precision: "f32" (exact-f32 MFMA) or "x3" (split-bf16 MFMA); None ->
        $GHM_PRECISION or "x3".
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
        n = sum(p.numel() for p in params)
        self.n_params = n
        self.pflat = torch.empty(n, dtype=torch.float32, device=self.device)
        self.gflat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.mflat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.vflat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.views = []  # per model: (param dict, grad dict, m dict, v dict)
        off = 0
        with torch.no_grad():
            for m in self.models:
                pd, gd, md, vd = {}, {}, {}, {}
                for name, p in m.named_parameters():
                    k = p.numel()
                    self.pflat[off:off + k].copy_(p.data.reshape(-1))
                    p.data = self.pflat[off:off + k].view(p.shape)
                    p.grad = self.gflat[off:off + k].view(p.shape)
                    pd[name], gd[name] = p.data, p.grad
                    md[name] = self.mflat[off:off + k].view(p.shape)
                    vd[name] = self.vflat[off:off + k].view(p.shape)
                    off += k
                self.views.append((pd, gd, md, vd))
        T = tmodel.n_token
        n_seq = batch_size * (K + 1)
        self.plans = [EncoderPlan(m.n_layer, m.n_token, n_seq, num_class=m.vocab_size, vocab=m.vocab_size,
                                  n_embd=m.n_embd, normalize_attn=m.normalize_attn, device=self.device,
                                  precision=precision,
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
            tr = np.ascontiguousarray(tr, dtype=np.float64)
            L, C, V = tr.shape[0], tr.shape[1], tr.shape[2]
            if C ** L != m.n_token or V != m.vocab_size:
                raise ValueError("guide transitions do not match the encoder's token count / vocabulary")
            layers = [l for l, f in enumerate(m.guided_layer_flag) if f]
            if len(layers) > L:
                raise ValueError("more guided layers than tree levels")
            n_total = (C ** L - 1) // (C - 1)
            self.glayers.append(layers)
            self.gtree.append((L, C, V))
            self.gtrans.append(torch.from_numpy(tr).to(self.device))
            self.gmsgs.append(torch.zeros(self.n_seq, n_total, V, dtype=torch.float32, device=self.device))
        self.n_gparts = sum(len(x) for x in self.glayers)
        self.gpart = torch.zeros(max(1, self.n_gparts), self.n_seq, dtype=torch.float32, device=self.device)
        self.phist = torch.zeros_like(self.hist)

    def _guide_fwd(self, tower, s):
        """BP guide targets from the staged tokens, then the penalty partials of
        the tower's guided layers (after its forward)."""
        L, C, V = self.gtree[tower]
        plan = self.plans[tower]
        base = sum(len(x) for x in self.glayers[:tower])
        _native.call("ghm_bp_cls", _p(self.gtrans[tower]), _p(plan.tokens), _p(self.gmsgs[tower]), self.n_seq,
                     L, C, V, s)
        for k, l in enumerate(self.glayers[tower]):
            _native.call("ghm_guide_fwd", _p(plan.H[l + 1]), _p(self.gmsgs[tower]), _p(self.gpart[base + k]),
                         self.n_seq, L, C, V, k, s)

    def _guide_hooks(self, tower):
        """{layer: fn(dH, stream)} adding d(penalty)/dH_{l+1} = 2 p (H - target) / N."""
        if not self.guide:
            return None
        L, C, V = self.gtree[tower]
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
    @staticmethod
    def _interleave(jobs):
        """Advance launch generators [(generator, stream), ...] round-robin, each
        step issued under its own stream: the two towers' per-layer launches are
        issued (and, captured, become graph nodes) alternately instead of one
        tower's whole sequence first."""
        active = list(jobs)
        while active:
            for job in list(active):
                gen, st = job
                with torch.cuda.stream(st):
                    try:
                        next(gen)
                    except StopIteration:
                        active.remove(job)

    def _fwd_bwd(self):
        """Text tower on the current stream, image tower on a side stream (fork /
        join through stream waits, which graph capture records as edges), so the
        two towers' launches overlap and fill each other's tails.  The towers'
        launches are issued layer by layer alternately ($GHM_TOWER_ORDER =
        "interleave", default) or one tower after the other ("sequential")."""
        main = torch.cuda.current_stream()
        side = main if os.environ.get("GHM_SERIAL_TOWERS") == "1" else self.side
        inter = os.environ.get("GHM_TOWER_ORDER", "interleave") == "interleave"
        pt, pi = self.plans
        (tp, tg, _, _), (ip, ig, _, _) = self.views
        side.wait_stream(main)
        s = ctypes.c_void_p(main.cuda_stream)
        if inter:
            self._interleave([(pi.forward_iter(ip), side), (pt.forward_iter(tp), main)])
            if self.guide:
                with torch.cuda.stream(side):
                    self._guide_fwd(1, ctypes.c_void_p(side.cuda_stream))
                self._guide_fwd(0, s)
        else:
            with torch.cuda.stream(side):
                pi.forward(ip)
                if self.guide:
                    self._guide_fwd(1, ctypes.c_void_p(side.cuda_stream))
            pt.forward(tp)
            if self.guide:
                self._guide_fwd(0, s)
        main.wait_stream(side)
        _native.call("ghm_clip_loss", _p(pt.emb), _p(pi.emb), _p(pt.d_emb), _p(pi.d_emb), _p(self.loss_out),
                     _p(self.hist), _p(self.step_ctr), self.B, self.K, self.C, s)
        if self.guide:
            _native.call("ghm_guide_total", _p(self.gpart), self.n_gparts, self.n_seq, self.penalty,
                         _p(self.loss_out), _p(self.phist), _p(self.step_ctr), s)
        side.wait_stream(main)
        if inter:
            self._interleave([(pi.backward_iter(ip, ig, layer_grad=self._guide_hooks(1)), side),
                              (pt.backward_iter(tp, tg, layer_grad=self._guide_hooks(0)), main)])
        else:
            with torch.cuda.stream(side):
                pi.backward(ip, ig, layer_grad=self._guide_hooks(1))
            pt.backward(tp, tg, layer_grad=self._guide_hooks(0))
        main.wait_stream(side)

    def _optim(self):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        b1, omb1, b2, omb2, eps = self.consts
        _native.call("ghm_clip_prepare", _p(self.gflat), self.n_params, self.max_norm, _p(self.sched),
                     self.n_sched, _p(self.step_ctr), _p(self.hyper), _p(self.work), s)
        _native.call("ghm_adamw", _p(self.pflat), _p(self.gflat), _p(self.mflat), _p(self.vflat),
                     self.n_params, _p(self.hyper), b1, omb1, b2, omb2, eps, s)

    def _allreduce(self):
        distributed.allreduce_mean_(self.gflat, group=self.pg)

    def set_tokens(self, t_tokens, i_tokens):
        """Stage one batch (uint8 [n_seq, T] host-pinned or device tensors) into
        the plans' token buffers, async on the current stream (the side stream
        is ordered after it by the fork in _fwd_bwd)."""
        self.plans[0].tokens.copy_(t_tokens, non_blocking=True)
        self.plans[1].tokens.copy_(i_tokens, non_blocking=True)

    def step(self):
        """One training step on the staged tokens (async; no host sync)."""
        if self.steps_done >= self.n_sched:
            raise RuntimeError("schedule exhausted")
        if self.graphs is not None:
            self.graphs[0].replay()
            if len(self.graphs) > 1:
                self._allreduce()
                self.graphs[1].replay()
        else:
            self._fwd_bwd()
            if self.pg is not None or distributed.is_on():
                self._allreduce()
            self._optim()
        self.steps_done += 1

    def capture(self):
        """Capture the step into HIP graphs (call after >= 1 eager step so all
        lazy initialisation has happened).  Replays reuse the staged tokens.
        One process: fwd/bwd and the optimizer are one graph (one launch, no
        host gap between them).  Data parallel: two graphs with the gradient
        all-reduce between them."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        dp = self.pg is not None or distributed.is_on()
        with torch.cuda.stream(s):
            if dp:
                g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(g1, stream=s):
                    self._fwd_bwd()
                with torch.cuda.graph(g2, stream=s):
                    self._optim()
                graphs = (g1, g2)
            else:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    self._fwd_bwd()
                    self._optim()
                graphs = (g,)
        torch.cuda.current_stream().wait_stream(s)
        self.graphs = graphs

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
