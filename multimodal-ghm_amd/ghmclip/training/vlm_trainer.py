"""Sequential-VLM training step on the HIP path — the hot loop of
src/ghmclip/training/train_sequential_NWP.py:157-185 (zero_grad, sample, frozen CLIP
image encoder, next-word model forward, ConditionalGuidedCELoss, KLdiv "Compare",
backward, clip_grad_norm_, cosine LR, AdamW).

Per step (one captured graph + one optimizer graph): the frozen CLIP image
EncoderPlan forward -> [B, 10] prefix features, VlmPlan forward, ghm_ce_kl (loss,
Compare against the host BP posteriors, dlogits, histories), VlmPlan backward;
then ghm_clip_prepare + ghm_adamw over the flat buffer of the trained parameters
(i_embedding and _out get no gradient in the reference: skipped, optimizer.py:55-56).
Data parallel (optional): the loss is a mean over samples; ranks take equal
sample shards and average gradients with one RCCL all-reduce.
"""
import ctypes

import numpy as np
import torch

from .. import _native
from . import distributed
from ..models.gemm_encoder import make_encoder_plan
from ..models.hip_encoder import require_hip
from ..models.optimizer import adam_consts, adam_lr_t
from ..models.vlm import VlmPlan, vlm_guide_blocks, vlm_guide_plane_elems, vlm_untrained


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


class VlmTrainer:
    def __init__(self, model, clip_model, batch_size, lr_schedule, max_norm=1.0, weight_decay=0.001,
                 betas=(0.9, 0.999), eps=1e-8, device="cuda", t_offset=0, process_group=None, precision=None,
                 penalty=0.001):
        """model: AutoRegressiveTransformer; clip_model: the frozen CLIP image
        EncoderTransformer (sequential model), or None for the joint model
        (sequential=False, train_NWP.py); lr_schedule: one learning rate per step.
        precision: matrix-product mode ("x3" split-bf16 MFMA or "f32") of the VLM plan
        and the frozen CLIP encoder's kernels (default $GHM_PRECISION or "x3")."""
        self.device = torch.device(device)
        self.model, self.clip = model, clip_model
        self.joint = clip_model is None  # train_NWP.py: image leaves through i_embedding, no CLIP
        if self.joint == bool(model.sequential):
            raise ValueError("a sequential model needs its frozen CLIP image encoder; the joint model takes none")
        untrained = vlm_untrained(model)
        self.B = batch_size
        self.max_norm = float(max_norm)
        self.pg = process_group
        sd = dict(model.named_parameters())
        for p in list(sd.values()) + ([] if self.joint else list(clip_model.parameters())):
            require_hip(p)
        trained = [n for n in model._names if n not in untrained]
        n = sum(sd[k].numel() for k in trained)
        self.n_params = n
        self.pflat = torch.empty(n, dtype=torch.float32, device=self.device)
        self.gflat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.mflat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.vflat = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.pd, self.gd, self.md, self.vd = {}, {}, {}, {}
        off = 0
        with torch.no_grad():
            for k in trained:
                p = sd[k]
                c = p.numel()
                self.pflat[off:off + c].copy_(p.data.reshape(-1))
                p.data = self.pflat[off:off + c].view(p.shape)
                p.grad = self.gflat[off:off + c].view(p.shape)
                self.pd[k], self.gd[k] = p.data, p.grad
                self.md[k] = self.mflat[off:off + c].view(p.shape)
                self.vd[k] = self.vflat[off:off + c].view(p.shape)
                off += c
            for k in untrained:
                self.pd[k] = sd[k].data
        self.clip_p = None if self.joint else {k: v.data for k, v in clip_model.named_parameters()}
        self.T, self.P, self.V = model.n_token, model.n_i_token, model.vocab_size
        self.plan = VlmPlan(model.n_layer, model.n_token, batch_size, n_prefix=model.n_i_token,
                            num_class=model.vocab_size, n_embd=model.n_embd, normalize_attn=model.normalize_attn,
                            device=self.device, precision=precision, joint=self.joint,
                            activation=getattr(model, "activation", "softmax"),
                            layernorm=getattr(model, "layernorm", True))
        if self.joint:
            self.clip_plan = None
            self.precision = self.plan.precision
        else:
            self.clip_plan = make_encoder_plan(clip_model.n_layer, clip_model.n_token, batch_size,
                                         num_class=clip_model.vocab_size, vocab=clip_model.vocab_size,
                                         n_embd=clip_model.n_embd, normalize_attn=clip_model.normalize_attn,
                                         device=self.device, precision=precision, ln_presplit=False)
            self.precision = self.clip_plan.precision
            if self.precision == "x3":
                self.clip_plan.split_weights(self.clip_p)  # frozen: split once
        Tt = self.T - self.P
        self.yt = torch.empty(batch_size, Tt, dtype=torch.uint8, device=self.device)
        self.post = torch.empty(batch_size, Tt, self.V, dtype=torch.float32, device=self.device)
        self.betas, self.wd = betas, weight_decay
        self.consts = adam_consts(betas, eps)
        self.t_offset = t_offset
        sched = np.zeros((len(lr_schedule), 2), dtype=np.float32)
        for s, lr in enumerate(lr_schedule):
            sched[s, 0] = adam_lr_t(lr, s + 1 + t_offset, betas)
            sched[s, 1] = lr * weight_decay
        self.sched = torch.from_numpy(sched.reshape(-1)).to(self.device)
        self.n_sched = len(lr_schedule)
        self.step_ctr = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.hyper = torch.zeros(4, dtype=torch.float32, device=self.device)
        self.work = torch.zeros(1024, dtype=torch.float32, device=self.device)
        # [loss, compare, per-workgroup partials] (ghm_ce_kl_out_elems)
        self.loss_out = torch.zeros(_native.hip_lib().ghm_ce_kl_out_elems(batch_size, self.T, self.P),
                                    dtype=torch.float32, device=self.device)
        self.hist = torch.zeros(max(1, len(lr_schedule)), dtype=torch.float32, device=self.device)
        self.chist = torch.zeros_like(self.hist)
        self.graphs = None
        self.steps_done = 0
        self._setup_guide(penalty)

    def _setup_guide(self, penalty):
        """Guided VLM (train_NWP.py / train_sequential_NWP.py --guide=True,
        exp_vlm_guidedTF.sh): the host stages per-position BP targets
        (bp_nwp_posterior(guide=True), and for the joint model the image
        guided_info, packed by vlm_guide_planes); the penalty partials of every
        guided block (model.py:303-331, 1122-1144) are one launch after the forward,
        their gradients one launch per guided layer in the backward.  The sequential
        model's image blocks target the frozen CLIP feature itself
        (train_sequential_NWP.py:165: [clip_image_output] * 2), read in place from
        the CLIP encoder's output [B][V] (no host staging)."""
        self.guide = bool(getattr(self.model, "guide", False))
        self.phist = None
        if not self.guide:
            return
        Tt = self.T - self.P
        self.penalty = float(penalty)
        self.gblocks = vlm_guide_blocks(self.model, Tt, self.V)
        self.n_gelems = vlm_guide_plane_elems(self.model, Tt, self.V)
        self.gtgt = torch.zeros(self.B, self.n_gelems, dtype=torch.float32, device=self.device)
        self.gitems = [(l, b) for l in sorted(self.gblocks) for b in self.gblocks[l]]
        self.gpart = torch.zeros(len(self.gitems), self.B, dtype=torch.float32, device=self.device)
        self.gbuf = torch.zeros(3, dtype=torch.float32, device=self.device)
        self.phist = torch.zeros_like(self.hist)
        self._glists = []
        mx = int(_native.hip_lib().ghm_guide_max_blocks())
        self._gfwd = [(a, self._blk_list(self.gitems[a:a + mx])) for a in range(0, len(self.gitems), mx)]
        self._gbwd = {l: [self._blk_list([(l, b) for b in blks[a:a + mx]]) for a in range(0, len(blks), mx)]
                      for l, blks in self.gblocks.items()}

    def _blk_list(self, items):
        """Host arrays of ghm_guide_blks_{fwd,bwd}_d (kept alive: graphs replay them)."""
        n = len(items)
        H = (ctypes.c_void_p * n)(*[self.plan.H[l + 1].data_ptr() for l, _ in items])
        M = (ctypes.c_void_p * n)()
        desc = (ctypes.c_int32 * (6 * n))()
        desc64 = (ctypes.c_int64 * (2 * n))()
        for k, (_, (tok0, ntok, col, off, grp)) in enumerate(items):
            desc[6 * k:6 * k + 6] = [self.T, tok0, ntok, col, 1, self.V]
            if grp == "loss3" and not self.joint:  # the CLIP feature [B][V] (one prefix token)
                M[k] = self.clip_plan.emb.data_ptr()
                desc64[2 * k:2 * k + 2] = [self.V, 0]
            else:
                M[k] = self.gtgt.data_ptr()
                desc64[2 * k:2 * k + 2] = [self.n_gelems, off]
        lst = (H, M, desc, desc64, n)
        self._glists.append(lst)
        return lst

    def _guide_hooks(self):
        if not self.guide:
            return None
        scale = 2.0 * self.penalty / self.B
        hooks = {}
        for l in self.gblocks:
            def fn(dH, s, l=l):
                for H, M, desc, desc64, n in self._gbwd[l]:
                    _native.call("ghm_guide_blks_bwd_d", H, M, desc, desc64, n, self.plan.D, _p(dH), scale, self.B,
                                 s)
            hooks[l] = fn
        return hooks

    def _fwd_bwd(self):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        emb = None if self.joint else self.clip_plan.forward(self.clip_p, split=False)  # train_sequential_NWP.py:163
        self.plan.forward(self.pd, self.plan.xt, emb)
        _native.call("ghm_ce_kl", _p(self.plan.logits), _p(self.yt), _p(self.post), _p(self.plan.dlogits),
                     _p(self.loss_out), _p(self.hist), _p(self.chist), _p(self.step_ctr), self.B, self.T, self.P,
                     self.V, s)
        if self.guide:  # ConditionalGuidedCELoss guide branch: ploss = CE + penalty * mean_b sum ||H - target||^2
            for a, (H, M, desc, desc64, n) in self._gfwd:
                _native.call("ghm_guide_blks_fwd_d", H, M, desc, desc64, n, self.plan.D,
                             ctypes.c_void_p(self.gpart[a].data_ptr()), self.B, s)
            self.gbuf[0:1].copy_(self.loss_out[0:1])
            _native.call("ghm_guide_total", _p(self.gpart), len(self.gitems), self.B, self.penalty, _p(self.gbuf),
                         _p(self.phist), _p(self.step_ctr), s)
        self.plan.backward(self.pd, self.gd, layer_grad=self._guide_hooks())

    def _optim(self):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        b1, omb1, b2, omb2, eps = self.consts
        _native.call("ghm_clip_prepare", _p(self.gflat), self.n_params, self.max_norm, _p(self.sched),
                     self.n_sched, _p(self.step_ctr), _p(self.hyper), _p(self.work), s)
        _native.call("ghm_adamw", _p(self.pflat), _p(self.gflat), _p(self.mflat), _p(self.vflat),
                     self.n_params, _p(self.hyper), b1, omb1, b2, omb2, eps, s)

    def _allreduce(self):
        distributed.allreduce_mean_(self.gflat, group=self.pg)

    def set_batch(self, xt, yt, post, i_tokens, guide_targets=None):
        """Stage one batch: text inputs / targets uint8 [B, T-1], BP posteriors
        float32 [B, T-1, V], image leaves uint8 [B, 81] (host-pinned or device);
        guided: the packed guide targets float32 [B, n_gelems] (vlm_guide_planes; the
        sequential model's hold the text blocks only)."""
        self.plan.xt.copy_(xt, non_blocking=True)
        self.yt.copy_(yt, non_blocking=True)
        self.post.copy_(post, non_blocking=True)
        (self.plan.itok if self.joint else self.clip_plan.tokens).copy_(i_tokens, non_blocking=True)
        if self.guide:
            if guide_targets is None:
                raise ValueError("the guided VLM needs its guide targets every step")
            self.gtgt.copy_(guide_targets, non_blocking=True)

    def step(self):
        if self.steps_done >= self.n_sched:
            raise RuntimeError("schedule exhausted")
        dp = self.pg is not None or distributed.is_on()
        if self.graphs is not None:
            self.graphs[0].replay()
            if len(self.graphs) > 1:
                self._allreduce()
                self.graphs[1].replay()
        else:
            self._fwd_bwd()
            if dp:
                self._allreduce()
            self._optim()
        self.steps_done += 1

    def capture(self):
        """Capture the step into HIP graphs (after >= 1 eager step): one graph in
        a single process, fwd/bwd and optimizer graphs around the gradient
        all-reduce under data parallelism."""
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

    def loss_history(self, upto=None):
        n = self.steps_done if upto is None else upto
        return self.hist[:n].double().cpu().numpy()

    def ploss_history(self, upto=None):
        """Loss including the guide penalties (train_NWP.py ploss_history); equals
        loss_history without guidance."""
        if self.phist is None:
            return self.loss_history(upto)
        n = self.steps_done if upto is None else upto
        return self.phist[:n].double().cpu().numpy()

    def guide_penalties(self):
        """The last step's penalty terms as ConditionalGuidedCELoss returns them
        (model.py:1144-1149): [loss2, loss4, loss5, loss3] (host sync)."""
        if not self.guide:
            return [0.0, 0.0, 0.0, 0.0]
        part = self.gpart.double().cpu().numpy()
        out = {"loss2": 0.0, "loss4": 0.0, "loss5": 0.0, "loss3": 0.0}
        for k, (_, blk) in enumerate(self.gitems):
            out[blk[4]] += self.penalty * float(part[k].mean())
        return [out["loss2"], out["loss4"], out["loss5"], out["loss3"]]

    def compare_history(self, upto=None):
        n = self.steps_done if upto is None else upto
        return self.chist[:n].double().cpu().numpy()

    def fill_optimizer_state(self, optimizer):
        t = self.steps_done + self.t_offset
        for name, p in self.model.named_parameters():
            if name in self.md:
                optimizer.state[p] = {"t": t, "m": self.md[name], "v": self.vd[name]}

    def load_optimizer_state(self, optimizer):
        with torch.no_grad():
            for name, p in self.model.named_parameters():
                st = optimizer.state.get(p)
                if st and name in self.md:
                    self.md[name].copy_(st["m"])
                    self.vd[name].copy_(st["v"])
