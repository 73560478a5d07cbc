"""BERT (base / large) pretraining on the tfk executor (BASELINE config 3: "BERT-base pretrain
TFJob ParameterServerStrategy PS=2/worker=6").

Architecture and TF variable names follow google-research/bert (modeling.py / run_pretraining.py):
post-LN encoder, GELU(tanh) FFN, masked-LM head (transform dense+GELU+LN, decoder tied to the
word embeddings + output_bias) evaluated only at the masked positions, next-sentence head on the
tanh pooler. MI355X mapping:
* q/k/v = ONE fused [3W, W] GEMM (FusedLinear); attention reads its output in place
  (ops.transformer.attention_* column views) -> no head split/merge transposes;
* bias, GELU, dropout and the residual add run in the GEMM epilogues; the GELU input is saved by
  the FFN1 epilogue (aux) and its derivative is applied in the FFN2 dgrad epilogue (dact);
* flash attention (MFMA, online softmax, dropout regenerated from a hash in backward);
* vocab padded to a multiple of 128 rows (padding rows stay zero, loss masks them).
Dropout seeds = per-(layer, site) host salt + a per-step key kept and advanced on the device, so
every mask is reproducible and a hipGraph-captured step draws fresh masks on every replay.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from ..ops import elementwise as E
from ..ops import gemm as G
from ..ops import transformer as TR
from ..ops.loss import softmax_xent
from ..runtime import streams
from ..runtime.arena import ParamArena, ParamSpec
from ..runtime.layers import Embedding, FusedLinear, LayerNorm, Linear


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    hidden_dropout: float = 0.1
    attn_dropout: float = 0.1
    ln_eps: float = 1e-12
    init_std: float = 0.02
    seq_len: int = 128
    max_predictions: int = 20
    fp8: bool = False  # all linear GEMMs (fwd, dgrad, wgrad) in MX-fp8 (e4m3 + e8m0 block scales)
    # split-K fill target for the encoder weight gradients (None = ops.gemm.TARGET_BLOCKS). Measured
    # on MI355X, base bs64x128: 512 -> 15.44 ms/step vs 16.17 at 1024 (profiles/splitk_sweep_*).
    wgrad_split_target: int | None = 512

    def __post_init__(self):
        from ..ops.elementwise import check_rate
        check_rate(self.hidden_dropout)  # representable by the kernels' 8-bit mask threshold
        check_rate(self.attn_dropout)

    @classmethod
    def base(cls):
        return cls()

    @classmethod
    def large(cls):
        return cls(hidden=1024, layers=24, heads=16, intermediate=4096)

    @classmethod
    def tiny(cls):  # tests
        return cls(vocab_size=1000, hidden=128, layers=2, heads=2, intermediate=256, max_position=64, seq_len=32,
                   max_predictions=5)


def _mix(*xs) -> int:
    h = 0x9E3779B97F4A7C15
    for x in xs:
        h = ((h ^ (x & 0xFFFFFFFFFFFFFFFF)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        h ^= h >> 31
    return h & 0x7FFFFFFFFFFFFFFF


class BertLayer:
    def __init__(self, arena: ParamArena, cfg: BertConfig, i: int):
        W, std = cfg.hidden, cfg.init_std
        pre = f"bert/encoder/layer_{i}"
        self.cfg, self.i = cfg, i
        self.qn, self.kn, self.vn = (f"{pre}/attention/self/{n}" for n in ("query", "key", "value"))
        self.qkv = FusedLinear(arena, [self.qn, self.kn, self.vn], W, W, std=std)
        self.ao = Linear(arena, f"{pre}/attention/output/dense", W, W, init="trunc_normal", std=std)
        self.ln1 = LayerNorm(arena, f"{pre}/attention/output/LayerNorm", W, cfg.ln_eps)
        self.ff1 = Linear(arena, f"{pre}/intermediate/dense", W, cfg.intermediate, init="trunc_normal", std=std)
        self.ff2 = Linear(arena, f"{pre}/output/dense", cfg.intermediate, W, init="trunc_normal", std=std)
        self.ln2 = LayerNorm(arena, f"{pre}/output/LayerNorm", W, cfg.ln_eps)
        for lin in (self.qkv, self.ao, self.ff1, self.ff2):
            lin.split_target = cfg.wgrad_split_target
        self.saved = None

    def forward(self, h, B, S, kv_len, seed: int, training: bool):
        cfg = self.cfg
        hd = cfg.hidden_dropout if training else 0.0
        ad = cfg.attn_dropout if training else 0.0
        s_attn, s_ao, s_ff = _mix(seed, 1), _mix(seed, 2), _mix(seed, 3)
        qkv = self.qkv.forward(h)
        sp = TR.AttnSpec(B, cfg.heads, S, S, (qkv, self.qkv.col(self.qn)), (qkv, self.qkv.col(self.kn)),
                         (qkv, self.qkv.col(self.vn)), kv_len=kv_len, p_drop=ad, seed=s_attn)
        o, lse = TR.attention_fwd(sp)
        s1 = self.ao.forward(o, resid=h, drop_p=hd, drop_seed=s_ao)
        h1, st1 = self.ln1.forward(s1)
        z = torch.empty(h1.shape[0], cfg.intermediate, dtype=torch.bfloat16, device=h.device)
        f = self.ff1.forward(h1, act="gelu", aux=z)
        s2 = self.ff2.forward(f, resid=h1, drop_p=hd, drop_seed=s_ff)
        h2, st2 = self.ln2.forward(s2)
        if training:
            self.saved = (h, qkv, sp, o, lse, s1, st1, h1, z, f, s2, st2, hd, s_ao, s_ff)
        return h2

    def backward(self, dh2):
        h, qkv, sp, o, lse, s1, st1, h1, z, f, s2, st2, hd, s_ao, s_ff = self.saved
        self.saved = None
        # LayerNorm backward also emits the hidden-dropout backward of its gradient (one kernel)
        # ... and the column sums of that gradient = the consuming Linear's bias gradient (no
        # separate column-sum pass; only when the bias gradients were pre-zeroed for this step)
        f2 = self.ff2.bias_sink() is not None
        ds2, dy2 = self.ln2.backward(dh2, s2, st2, drop=(hd, s_ff), consumer=self.ff2 if f2 else None)
        dz = self.ff2.backward(dy2, f, dact_src=z, dact="gelu", bias_done=f2)
        dh1 = self.ff1.backward(dz, h1, resid=ds2)
        fa = self.ao.bias_sink() is not None
        ds1, dy1 = self.ln1.backward(dh1, s1, st1, drop=(hd, s_ao), consumer=self.ao if fa else None)
        do = self.ao.backward(dy1, o, bias_done=fa)
        dqkv = torch.empty_like(qkv)
        TR.attention_bwd(sp, o, do, lse, (dqkv, self.qkv.col(self.qn)), (dqkv, self.qkv.col(self.kn)),
                         (dqkv, self.qkv.col(self.vn)))
        return self.qkv.backward(dqkv, h, resid=ds1)


class BertForPreTraining:
    def __init__(self, cfg: BertConfig | None = None):
        cfg = cfg or BertConfig.base()
        if cfg.hidden != cfg.heads * TR.HEAD_DIM:
            raise ValueError("tfk attention kernels use head_dim 64: hidden must equal heads*64")
        self.cfg = cfg
        self.name = "bert-large" if cfg.layers == 24 else "bert-base" if cfg.layers == 12 else "bert"
        self.num_classes = cfg.vocab_size
        self.training = True
        self.step = 0
        W, std = cfg.hidden, cfg.init_std
        a = self.arena = ParamArena()
        # dropout RNG: int64 [counter, key] on the device, advanced INSIDE every training step
        # (hipGraph-replayable); kernels use seed = per-site host salt + key (ops.elementwise.rng_key).
        # A checkpointed buffer, so a resumed job continues the mask sequence; rng_stream (e.g. the
        # data-parallel rank) gives each replica its own masks.
        self.rng_state = a.add_buffer("tfk/dropout_rng_state", torch.zeros(2, dtype=torch.int64))
        self.rng_stream = 0
        # registration order = forward order (the arena reverses it so backward fills grads front-to-back)
        self.word = Embedding(a, "bert/embeddings/word_embeddings", cfg.vocab_size, W, std)
        self.pos = Embedding(a, "bert/embeddings/position_embeddings", cfg.max_position, W, std)
        self.typ = Embedding(a, "bert/embeddings/token_type_embeddings", cfg.type_vocab, W, std)
        self.ln_emb = LayerNorm(a, "bert/embeddings/LayerNorm", W, cfg.ln_eps)
        self.layers = [BertLayer(a, cfg, i) for i in range(cfg.layers)]
        self.pooler = Linear(a, "bert/pooler/dense", W, W, init="trunc_normal", std=std)
        self.mlm_dense = Linear(a, "cls/predictions/transform/dense", W, W, init="trunc_normal", std=std)
        self.mlm_ln = LayerNorm(a, "cls/predictions/transform/LayerNorm", W, cfg.ln_eps)
        Vp = self.word.Vp
        self.mlm_bias = a.add(ParamSpec("cls/predictions/output_bias", (Vp,), init="zeros", decay=False,
                                        tf_shape=(cfg.vocab_size,), to_tf=lambda x, V=cfg.vocab_size: x[:V],
                                        from_tf=lambda x, Vp=Vp: np.concatenate([x, np.zeros(Vp - x.shape[0], x.dtype)])))
        # TF stores output_weights as [out=2, in=W] (no transpose)
        self.nsp = Linear(a, "cls/seq_relationship", W, 2, init="trunc_normal", std=std, kernel_name="output_weights")
        self.nsp.w.spec.to_tf = None
        self.nsp.w.spec.from_tf = None
        self.nsp.w.spec.tf_shape = (2, W)
        self.nsp.b.spec.name = "cls/seq_relationship/output_bias"
        self._wq = None
        self._fp8_lins = []
        if cfg.fp8:
            for layer in self.layers:
                for lin in (layer.qkv, layer.ao, layer.ff1, layer.ff2):
                    lin.fp8 = True
                    self._fp8_lins.append(lin)

    def to(self, device, seed: int = 1234):
        self.arena.finalize(device, seed)
        self._wq = None
        return self

    def train(self, mode: bool = True):
        self.training = mode
        return self

    # ------------------------------------------------------------------ forward
    def _encode(self, ids, tt, B, S, kv_len, seed):
        cfg = self.cfg
        hd = cfg.hidden_dropout if self.training else 0.0
        e = TR.embedding_fwd(ids, self.word.table.compute, self.pos.table.compute, S, tt, self.typ.table.compute)
        e_ln, st = self.ln_emb.forward(e)
        s_emb = _mix(seed, 0xE)
        h = E.dropout(e_ln, hd, s_emb)
        for i, layer in enumerate(self.layers):
            h = layer.forward(h, B, S, kv_len, _mix(seed, 100 + i), self.training)
        return h, (e, st, hd, s_emb)

    def _heads(self, h, B, S, mlm_pos):
        hm = TR.gather_rows(h, mlm_pos, S)  # the MLM positions' rows (HIP gather)
        zt = torch.empty_like(hm)
        t = self.mlm_dense.forward(hm, act="gelu", aux=zt)
        tl, stt = self.mlm_ln.forward(t)
        logits = G.linear_fwd(tl, self.word.table.compute, self.mlm_bias.master)  # tied decoder
        hc = TR.gather_rows(h, None, S)  # the [CLS] rows
        zp = torch.empty(B, self.cfg.hidden, dtype=torch.bfloat16, device=h.device)
        pooled = self.pooler.forward(hc, act="tanh", aux=zp)
        nsp_logits = self.nsp.forward(pooled)
        return logits, nsp_logits, (mlm_pos, hm, zt, t, tl, stt, None, hc, zp, pooled)

    def forward_backward(self, ids, tt, mlm_pos, mlm_ids, nsp_labels, loss_scale: float = 1.0):
        """One training step's forward + backward (see _forward_backward). The no-decay gradients
        (biases, LayerNorm gamma/beta) are zeroed in one fill up front and accumulated by their kernels."""
        self.arena.zero_nodecay_grads()
        E.rng_advance(self.rng_state, self.rng_stream)
        if self.cfg.fp8:
            from ..ops.fp8 import clear_saved
            from ..runtime.layers import weight_quantizer
            clear_saved()  # transposed MX operands live from this step's forward to its backward
            weight_quantizer(self, self._fp8_lins).run()  # all fp8 weights, both ways, one launch
        try:
            with E.rng_key(self.rng_state):
                return self._forward_backward(ids, tt, mlm_pos, mlm_ids, nsp_labels, loss_scale)
        finally:
            self.arena.prezeroed = False
            if self.cfg.fp8:
                from ..ops.fp8 import clear_saved
                clear_saved()  # nothing quantized in this step may leak into a later forward

    def _forward_backward(self, ids, tt, mlm_pos, mlm_ids, nsp_labels, loss_scale: float = 1.0):
        """One pretraining step's forward + backward. Returns (loss f32 [B], mlm-correct f32 [B*P])."""
        cfg = self.cfg
        B = nsp_labels.shape[0]
        S = ids.numel() // B
        P = mlm_pos.shape[1]
        self.step += 1
        seed = 0xBE27  # salt base; the per-step part is the device key (rng_state)
        h, emb_saved = self._encode(ids, tt, B, S, None, seed)
        logits, nsp_logits, hs = self._heads(h, B, S, mlm_pos)
        rows, hm, zt, t, tl, stt, cls_rows, hc, zp, pooled = hs
        V = cfg.vocab_size
        mlm_loss, dlogits, corr = softmax_xent(logits, mlm_ids.reshape(-1), scale=loss_scale / (B * P),
                                               want_correct=True, V=V)
        nsp_loss, dnsp, _ = softmax_xent(nsp_logits, nsp_labels, scale=loss_scale / B)
        # ---- heads backward (the decoder wgrad is the first writer of the word-embedding grad)
        G.linear_wgrad(dlogits, tl, self.word.table.grad)  # first writer of the tied table's grad
        G.bias_grad(dlogits, self.mlm_bias.grad, accumulate=self.arena.prezeroed)
        self.arena.grad_ready(self.mlm_bias)
        dtl = G.linear_dgrad(dlogits, self.word.table.compute)
        dt = self.mlm_ln.backward(dtl, t, stt)
        dt = E.act_bwd(dt, zt, "gelu")
        dhm = self.mlm_dense.backward(dt, hm)
        dpooled = self.nsp.backward(dnsp, pooled)
        dzp = E.act_bwd(dpooled, zp, "tanh")
        dhc = self.pooler.backward(dzp, hc)
        dh = torch.zeros_like(h)
        TR.scatter_add_rows(dh, dhm, rows, S)  # rows = the MLM positions
        TR.scatter_add_rows(dh, dhc, None, S)  # the [CLS] rows
        streams.flush()  # the heads' weight gradients behind one side-stream fork (under capture)
        # ---- encoder backward
        for layer in reversed(self.layers):
            dh = layer.backward(dh)
            streams.flush()  # this layer's weight gradients, concurrent with the next layer's dgrads
        e, st, hd, s_emb = emb_saved
        de = self.ln_emb.backward(E.dropout(dh, hd, s_emb), e, st)
        self.pos.table.grad.zero_()
        self.typ.table.grad.zero_()
        TR.embedding_bwd(ids, de, self.word.table.grad, self.pos.table.grad, S, tt,
                         self.typ.table.grad[:self.cfg.type_vocab])  # real rows only (table padded to 64)
        streams.join()  # side-stream weight gradients complete before anyone reads arena.grad
        self.arena.grad_ready(self.word.table, self.pos.table, self.typ.table)
        loss = mlm_loss.view(B, P).mean(1) + nsp_loss
        return loss, corr

    def evaluate(self, ids, tt, mlm_pos, mlm_ids, nsp_labels):
        """Returns (sum of MLM loss, number of MLM hits, number of predictions)."""
        was = self.training
        self.training = False
        B = nsp_labels.shape[0]
        S = ids.numel() // B
        h, _ = self._encode(ids, tt, B, S, None, 0)
        logits, _, _ = self._heads(h, B, S, mlm_pos)
        loss, _, corr = softmax_xent(logits, mlm_ids.reshape(-1), want_grad=False, want_correct=True,
                                     V=self.cfg.vocab_size)
        for layer in self.layers:
            layer.saved = None
        self.training = was
        return float(loss.sum()), float(corr.sum()), int(corr.numel())

    def synthetic_batch(self, batch: int, device, seed: int = 0, seq_len: int | None = None, **_):
        """Synthetic pretraining batch (full-length sequences, 2 segments, P masked positions)."""
        cfg = self.cfg
        S = seq_len or cfg.seq_len
        P = cfg.max_predictions
        g = torch.Generator().manual_seed(seed)
        ids = torch.randint(0, cfg.vocab_size, (batch, S), generator=g, dtype=torch.int32)
        tt = torch.zeros(batch, S, dtype=torch.int32)
        tt[:, S // 2:] = 1
        pos = torch.sort(torch.rand(batch, S - 1, generator=g).argsort(1)[:, :P] + 1, 1).values.to(torch.int32)
        mlm_ids = torch.gather(ids, 1, pos.long()).to(torch.int32)
        nsp = torch.randint(0, 2, (batch,), generator=g, dtype=torch.int32)
        return tuple(t.contiguous().to(device) for t in (ids.reshape(-1), tt.reshape(-1), pos, mlm_ids, nsp))

