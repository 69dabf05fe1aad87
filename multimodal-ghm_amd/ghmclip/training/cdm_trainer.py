"""Fused sequential-CDM training step on the HIP path — the hot loop of
src/ghmclip/training/train_sequential_DNS.py:141-168 (zero_grad, sample, frozen
CLIP text encoder, denoiser forward, ConditionalGuidedLsLoss / LsLoss / Compare,
backward, clip_grad_norm_, cosine LR, AdamW).

Per step, on the device (one captured graph + one optimizer graph):
  (guide=True: the BP messages of the image tree on the side stream, the guided
  penalty blocks after the loss, their gradients added into the residual stream
  before each guided layer's backward)
  side stream: ghm_bp_dns — exact BP posterior means from the staged text leaves
               and the f64 noisy observations (the "Compare" target), and the f32
               model input z (the reference computes both on the host, :145,
               data_random_GHM.py:871-882)
  main stream: frozen CLIP text EncoderPlan forward -> [B, 10] features,
               CdmPlan forward, ghm_ls_loss (loss, compare, dpred, histories),
               CdmPlan backward
  optimizer:   ghm_clip_prepare + ghm_adamw over the flat buffer of the trained
               parameters (t_embedding and _out get no gradient in the reference,
               so AdamW and the clip skip them, optimizer.py:55-56).
Data parallel (optional): the loss is a mean over samples, so ranks take equal
row shards and average gradients with one RCCL all-reduce.
"""
import ctypes

import numpy as np
import torch

from ..data.data_random_GHM import DeviceTree
from .. import _native
from . import distributed
from ..models.cdm import CdmPlan, cdm_guide_blocks, cdm_precision, cdm_untrained
from ..models.gemm_encoder import make_encoder_plan
from ..models.hip_encoder import require_hip
from ..models.optimizer import adam_consts, adam_lr_t


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


class CdmTrainer:
    def __init__(self, model, clip_model, batch_size, lr_schedule, t_templ, i_templ, sigma=1.0, max_norm=1.0,
                 weight_decay=0.001, betas=(0.9, 0.999), eps=1e-8, device="cuda", t_offset=0, process_group=None,
                 precision=None, penalty=0.1):
        """model: ConditionalDenoiseEncoderTransformer; clip_model: the frozen CLIP
        text EncoderTransformer (sequential model), or None for the joint model
        (sequential=False, train_CDNS.py: the text leaves go through t_embedding);
        lr_schedule: one learning rate per step; t_templ / i_templ: the sampler's
        transition templates [L][C][V][V]."""
        self.joint = clip_model is None
        if self.joint == bool(model.sequential):
            raise ValueError("a sequential model needs its frozen CLIP text encoder; the joint model takes none")
        self.device = torch.device(device)
        self.model, self.clip = model, clip_model
        self.B = batch_size
        self.max_norm = float(max_norm)
        self.pg = process_group
        self.sigma = float(sigma)
        self.names = list(model._names)
        sd = dict(model.named_parameters())
        untrained = cdm_untrained(model)
        for p in list(sd.values()) + ([] if self.joint else list(clip_model.parameters())):
            require_hip(p)
        trained = [n for n in self.names if n not in untrained]
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
        T, Ti = model.n_token, model.n_i_token
        self.T, self.Ti = T, Ti
        # the joint model: "f32fwd" unguided (its 30-step reference curve at f32's
        # distance, 7.8e-6 / 1.5e-5 against 7.2e-6 / 1.4e-5; step 4.66 -> 3.22 ms),
        # "f32x6" guided (the backward exact f32; 4.91 -> 4.37 ms; models/cdm.py)
        precision = cdm_precision(precision, self.joint, getattr(model, "guide", False),
                                  getattr(model, "layernorm", True))
        self.plan = CdmPlan(model.n_layer, T, Ti, batch_size, num_class=model.vocab_size, n_embd=model.n_embd,
                            normalize_attn=model.normalize_attn, device=self.device, precision=precision,
                            joint=self.joint, activation=getattr(model, "activation", "softmax"),
                            layernorm=getattr(model, "layernorm", True))
        self.precision = self.plan.precision
        if self.joint:
            self.clip_plan = None
            self.t_tok = self.plan.tok  # text leaves [B, T - T_img], read by the embedding and BP
            n_text = T - Ti
        else:
            self.clip_plan = make_encoder_plan(clip_model.n_layer, clip_model.n_token, batch_size,
                                         num_class=clip_model.vocab_size, vocab=clip_model.vocab_size,
                                         n_embd=clip_model.n_embd, normalize_attn=clip_model.normalize_attn,
                                         device=self.device, precision=self.precision, ln_presplit=False)
            if getattr(self.clip_plan, "pack", None) is not None:
                self.clip_plan.split_weights(self.clip_p)  # frozen: split once
            self.t_tok = self.clip_plan.tokens
            n_text = clip_model.n_token
        # templates [L][C][V][V], or per-edge tables of non-translation-invariant trees
        tt, it = DeviceTree.of(t_templ), DeviceTree.of(i_templ)
        if it.C ** it.L != Ti or tt.C ** tt.L != n_text:
            raise ValueError("transition templates do not match the token counts")
        self.tree = (tt.L, tt.C, it.L, it.C, tt.V)
        self.per_edge = tt.per_edge | (it.per_edge << 1)  # ghm_bp_dns: bit 0 text, bit 1 image
        self.t_trans = torch.from_numpy(tt.trans).to(self.device)
        self.i_trans = torch.from_numpy(it.trans).to(self.device)
        # staged inputs (text leaves live in the CLIP plan's token buffer)
        self.i_tok = torch.empty(batch_size, Ti, dtype=torch.uint8, device=self.device)
        self.z64 = torch.empty(batch_size, Ti, dtype=torch.float64, device=self.device)
        self.z32 = torch.empty(batch_size, Ti, dtype=torch.float32, device=self.device)
        self.post = torch.empty(batch_size, Ti, dtype=torch.float32, device=self.device)
        # optimizer constants and the per-step schedule table (as ClipTrainer)
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
        self.loss_out = torch.zeros(2, dtype=torch.float32, device=self.device)
        self.hist = torch.zeros(max(1, len(lr_schedule)), dtype=torch.float32, device=self.device)
        self.chist = torch.zeros_like(self.hist)
        self.graphs = None
        self.steps_done = 0
        self.side = torch.cuda.Stream(device=self.device)
        self._setup_guide(penalty)

    def _setup_guide(self, penalty):
        """Guided CDM (train_CDNS.py / train_sequential_DNS.py --guide=True): BP
        message buffers (image hd/qd/bu planes; the joint model's text BP_CLS
        levels), one penalty partial row per guided block, and the penalised loss
        history (ploss_history).  The sequential model's text blocks target the
        frozen CLIP text embedding (train_sequential_DNS.py:145)."""
        self.guide = bool(getattr(self.model, "guide", False))
        self.phist = None
        if not self.guide:
            return
        Lt, Ct, Li, Ci, V = self.tree
        self.penalty = float(penalty)
        self.gblocks = cdm_guide_blocks(self.model, (Lt, Ct), (Li, Ci), V)
        self.n_inodes = sum(Ci ** d for d in range(1, Li + 1)) + 1
        n_tnodes = sum(Ct ** d for d in range(Lt))
        self.imsgs = torch.zeros(self.B, 3, self.n_inodes, V, dtype=torch.float32, device=self.device)
        self.tmsgs = torch.zeros(self.B, n_tnodes, V, dtype=torch.float32, device=self.device) if self.joint else None
        # ConditionalGuidedLsLoss's diagnostic groups (model.py:1023-1040): loss2 = the
        # first Li image-guided layers, loss4 = the middle (root) one, loss5 = the
        # last Li, loss3 = the text blocks; one group id per penalty partial row
        ig = [l for l, f in enumerate(self.model.i_guided_layer_flag) if f]
        self.gpart_group = []
        for l, blks in sorted(self.gblocks.items()):
            for b in blks:
                if b[0] != "i":
                    self.gpart_group.append(3)
                else:
                    k = ig.index(l)
                    self.gpart_group.append(0 if k < Li else (1 if k == Li else 2))
        self.n_gparts = sum(len(b) for b in self.gblocks.values())
        self.gpart = torch.zeros(self.n_gparts, self.B, dtype=torch.float32, device=self.device)
        self.gloss = torch.zeros(3, dtype=torch.float32, device=self.device)
        self.phist = torch.zeros_like(self.hist)
        self._blk_lists, self._gfwd, self._gbwd = [], None, {}

    def _blk_args(self, blk):
        src, tok0, ntok, col, moff, ext = blk
        msgs = {"i": self.imsgs, "t": self.tmsgs, "c": None if self.joint else self.clip_plan.emb}[src]
        return tok0, ntok, col, _p(msgs), msgs[0].numel(), moff, ext, self.tree[4]

    def _blk_list(self, items):
        """Host arrays for ghm_guide_blks_{fwd,bwd}: items = [(layer, block), ...]
        in launch order; kept alive on self (the HIP graph replays the launch)."""
        n = len(items)
        H = (ctypes.c_void_p * n)(*[self.plan.H[l + 1].data_ptr() for l, _ in items])
        M = (ctypes.c_void_p * n)()
        desc = (ctypes.c_int32 * (6 * n))()
        desc64 = (ctypes.c_int64 * (2 * n))()
        for k, (l, blk) in enumerate(items):
            tok0, ntok, col, msgs, stride, moff, ext, V = self._blk_args(blk)
            M[k] = msgs
            desc[6 * k:6 * k + 6] = [self.T, tok0, ntok, col, ext, V]
            desc64[2 * k:2 * k + 2] = [stride, moff]
        lst = (H, M, desc, desc64, n)
        self._blk_lists.append(lst)
        return lst

    def _guide_fwd(self, s):
        """All guided blocks, in launches of at most ghm_guide_max_blocks() blocks
        (one launch for the default 26); part row k = the k-th block in layer order."""
        if self._gfwd is None:
            items = [(l, b) for l, blks in sorted(self.gblocks.items()) for b in blks]
            mx = int(_native.hip_lib().ghm_guide_max_blocks())
            self._gfwd = [(a, self._blk_list(items[a:a + mx])) for a in range(0, len(items), mx)]
        for a, (H, M, desc, desc64, n) in self._gfwd:
            _native.call("ghm_guide_blks_fwd", H, M, desc, desc64, n, ctypes.c_void_p(self.gpart[a].data_ptr()),
                         self.B, s)

    def _guide_hooks(self):
        """{layer: fn(dH, stream)} adding d(penalty)/dH_{l+1} = 2 p (H - target) / B,
        one launch per guided layer."""
        if not self.guide:
            return None
        scale = 2.0 * self.penalty / self.B
        hooks = {}
        for l, blks in self.gblocks.items():
            def fn(dH, s, l=l, blks=blks):
                if l not in self._gbwd:
                    mx = int(_native.hip_lib().ghm_guide_max_blocks())
                    self._gbwd[l] = [self._blk_list([(l, b) for b in blks[a:a + mx]])
                                     for a in range(0, len(blks), mx)]
                for H, M, desc, desc64, n in self._gbwd[l]:  # in list order: shared columns accumulate
                    _native.call("ghm_guide_blks_bwd", H, M, desc, desc64, n, _p(dH), scale, self.B, s)
            hooks[l] = fn
        return hooks

    # -- the launch sequence -----------------------------------------------------
    def _fwd_bwd(self):
        main = torch.cuda.current_stream()
        side = self.side
        Lt, Ct, Li, Ci, V = self.tree
        side.wait_stream(main)
        with torch.cuda.stream(side):
            ss = ctypes.c_void_p(side.cuda_stream)
            if self.guide:
                _native.call("ghm_bp_dns_msgs", _p(self.t_trans), _p(self.i_trans), _p(self.t_tok), _p(self.z64),
                             self.sigma, _p(self.post), _p(self.z32), _p(self.imsgs), self.B, Lt, Ct, Li, Ci, V,
                             self.per_edge, ss)
                if self.joint:  # (the sequential model's text blocks target the CLIP feature)
                    _native.call("ghm_bp_cls", _p(self.t_trans), _p(self.t_tok), _p(self.tmsgs), self.B, Lt, Ct, V,
                                 self.per_edge & 1, ss)
            else:
                _native.call("ghm_bp_dns", _p(self.t_trans), _p(self.i_trans), _p(self.t_tok), _p(self.z64),
                             self.sigma, _p(self.post), _p(self.z32), self.B, Lt, Ct, Li, Ci, V, self.per_edge, ss)
        emb = None if self.joint else self.clip_plan.forward(self.clip_p, split=False)  # train_sequential_DNS.py:141
        main.wait_stream(side)
        s = ctypes.c_void_p(main.cuda_stream)
        self.plan.forward(self.pd, self.z32, emb, 0 if emb is None else emb.shape[1])
        _native.call("ghm_ls_loss", _p(self.plan.pred), _p(self.i_tok), _p(self.post), _p(self.plan.dpred),
                     _p(self.loss_out), _p(self.hist), _p(self.chist), _p(self.step_ctr), self.B, self.Ti, s)
        if self.guide:  # ConditionalGuidedLsLoss guide branch (model.py:1023-1040)
            self._guide_fwd(s)
            self.gloss[0:1].copy_(self.loss_out[0:1])
            _native.call("ghm_guide_total", _p(self.gpart), self.n_gparts, self.B, self.penalty, _p(self.gloss),
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

    def set_batch(self, t_tokens, i_tokens, z):
        """Stage one batch: text / image leaves uint8 [B, 81] and the noisy image
        observations z float64 [B, 81] (host-pinned or device), async."""
        self.t_tok.copy_(t_tokens, non_blocking=True)
        self.i_tok.copy_(i_tokens, non_blocking=True)
        self.z64.copy_(z, non_blocking=True)

    def step(self):
        """One training step on the staged batch (async; no host sync)."""
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

    # -- host-side views -----------------------------------------------------------
    def loss_history(self, upto=None):
        """Denoising loss per step (train_sequential_DNS.py loss_history; equals
        ploss_history without guidance)."""
        n = self.steps_done if upto is None else upto
        return self.hist[:n].double().cpu().numpy()

    def ploss_history(self, upto=None):
        """Penalised loss per step (train_CDNS.py ploss_history): the loss plus the
        guided penalties when the model is guided, else the loss itself."""
        if not self.guide:
            return self.loss_history(upto)
        n = self.steps_done if upto is None else upto
        return self.phist[:n].double().cpu().numpy()

    def penalty_groups(self):
        """The last step's ConditionalGuidedLsLoss diagnostics (loss2, loss4, loss5,
        loss3): penalty x the batch mean of each group's squared Frobenius norms
        (model.py:1023-1040; train_sequential_DNS.py logs them).  Host sync."""
        if not self.guide:
            return np.zeros(4)
        part = self.gpart.double().cpu().numpy()
        out = np.zeros(4)
        for row, grp in enumerate(self.gpart_group):
            out[grp] += part[row].mean()
        return self.penalty * out

    def compare_history(self, upto=None):
        """Squared error against the BP posterior means per step (compare_history)."""
        n = self.steps_done if upto is None else upto
        return self.chist[:n].double().cpu().numpy()

    def fill_optimizer_state(self, optimizer):
        """Expose the flat moments as the reference AdamW's per-parameter state."""
        t = self.steps_done + self.t_offset
        for name, p in self.model.named_parameters():
            if name in self.md:
                optimizer.state[p] = {"t": t, "m": self.md[name], "v": self.vd[name]}

    def load_optimizer_state(self, optimizer):
        """Copy a loaded reference-format AdamW state ('m', 'v') into the flat moments."""
        with torch.no_grad():
            for name, p in self.model.named_parameters():
                st = optimizer.state.get(p)
                if st and name in self.md:
                    self.md[name].copy_(st["m"])
                    self.vd[name].copy_(st["v"])
