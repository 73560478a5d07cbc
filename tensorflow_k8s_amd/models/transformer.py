"""Transformer (big / base) encoder-decoder for WMT-shaped translation (BASELINE config 5:
"Transformer-big (WMT-shape) bf16/fp8 MFMA, 8-worker ring all-reduce TFJob").

Follows tensor2tensor's transformer_big hparams: d_model 1024, 16 heads, FFN 4096 (ReLU), 6+6
layers, pre-LayerNorm residual blocks ("n" preprocess, "da" postprocess), sinusoidal timing
signal, ONE shared embedding matrix for source, target and the softmax (scaled by sqrt(d)),
label smoothing 0.1, dropouts 0.3 (residual) / 0.1 (attention, relu). Attention projections have
no bias (as in T2T). TF variable names mirror T2T's ("transformer/body/encoder/layer_0/
self_attention/multihead_attention/q/kernel", ...), so checkpoints map name-for-name.

MI355X mapping as in models/bert.py: fused q|k|v (self-attention) and k|v (encoder-decoder
attention, computed from the encoder memory) GEMMs, flash attention (causal for decoder self
attention; cross attention with Sq != Sk), dropout + residual in GEMM epilogues, the ReLU mask
applied in the FFN2 dgrad epilogue from the saved pre-activation.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from ..ops import elementwise as E
from ..ops import gemm as G
from ..ops import transformer as TR
from ..ops.loss import softmax_xent
from ..ops import fp8 as F8
from ..runtime import streams
from ..runtime.arena import ParamArena
from ..runtime.layers import Embedding, FusedLinear, LayerNorm, Linear
from .bert import _mix

def _sink(lin):
    """lin when a LayerNorm backward may reduce its bias gradient (the gradient it hands lin is lin's
    output gradient; runtime.layers.LayerNorm.backward consumer), else None."""
    return lin if lin.bias_sink() is not None else None


# fp8 training: LayerNorms and FFN GEMMs that feed only MX-fp8 GEMMs emit those GEMMs' MX operands
# themselves (ops.fp8 _register_out) instead of separate quantize passes (measured 19.21 -> 18.86 ms)
MX_PRODUCERS = True


@dataclass
class TransformerConfig:
    vocab_size: int = 33708  # t2t translate_ende_wmt32k shared subword vocabulary
    hidden: int = 1024
    enc_layers: int = 6
    dec_layers: int = 6
    heads: int = 16
    ffn: int = 4096
    dropout: float = 0.3
    attn_dropout: float = 0.1
    relu_dropout: float = 0.1
    label_smoothing: float = 0.1
    ln_eps: float = 1e-6
    src_len: int = 256
    tgt_len: int = 256
    max_len: int = 1024
    fp8: bool = False  # all linear GEMMs (fwd, dgrad, wgrad) in MX-fp8 (e4m3 + e8m0 block scales)

    def __post_init__(self):
        from ..ops.elementwise import check_rate
        for k in ("dropout", "attn_dropout", "relu_dropout"):
            check_rate(getattr(self, k))  # representable by the kernels' 8-bit mask threshold

    @classmethod
    def big(cls):
        return cls()

    @classmethod
    def base(cls):
        return cls(hidden=512, heads=8, ffn=2048, dropout=0.1)

    @classmethod
    def tiny(cls):  # tests
        return cls(vocab_size=500, hidden=128, enc_layers=2, dec_layers=2, heads=2, ffn=256, src_len=24, tgt_len=20,
                   max_len=64)


def timing_signal(length: int, channels: int) -> torch.Tensor:
    """tensor2tensor get_timing_signal_1d: [sin(p*inv_ts) | cos(p*inv_ts)], half the channels each."""
    half = channels // 2
    log_inc = math.log(1.0e4) / max(half - 1, 1)
    inv = torch.exp(torch.arange(half, dtype=torch.float64) * -log_inc)
    t = torch.arange(length, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cat([torch.sin(t), torch.cos(t)], 1).float()


class _Attn:
    """Self attention (fused q|k|v) or encoder-decoder attention (q from x, fused k|v from memory)."""

    def __init__(self, arena, pre: str, W: int, cross: bool):
        self.cross = cross
        base = f"{pre}/multihead_attention"
        self.names = {n: f"{base}/{n}" for n in "qkv"}
        if cross:
            self.q = Linear(arena, self.names["q"], W, W, bias=False, init="trunc_normal", std=W ** -0.5)
            self.kv = FusedLinear(arena, [self.names["k"], self.names["v"]], W, W, bias=False, std=W ** -0.5)
        else:
            self.qkv = FusedLinear(arena, [self.names[n] for n in "qkv"], W, W, bias=False, std=W ** -0.5)
        self.out = Linear(arena, f"{base}/output_transform", W, W, bias=False, init="trunc_normal", std=W ** -0.5)


class EncoderLayer:
    def __init__(self, arena: ParamArena, cfg: TransformerConfig, pre: str):
        W = cfg.hidden
        self.cfg = cfg
        self.ln1 = LayerNorm(arena, f"{pre}/self_attention/layer_prepostprocess/layer_norm", W, cfg.ln_eps,
                             ("layer_norm_scale", "layer_norm_bias"))
        self.att = _Attn(arena, f"{pre}/self_attention", W, cross=False)
        self.ln2 = LayerNorm(arena, f"{pre}/ffn/layer_prepostprocess/layer_norm", W, cfg.ln_eps,
                             ("layer_norm_scale", "layer_norm_bias"))
        self.ff1 = Linear(arena, f"{pre}/ffn/conv1", W, cfg.ffn, init="trunc_normal", std=W ** -0.5)
        self.ff2 = Linear(arena, f"{pre}/ffn/conv2", cfg.ffn, W, init="trunc_normal", std=cfg.ffn ** -0.5)
        self.ffn_ln = self.ln2
        self.saved = None

    @staticmethod
    def _mx(x, lin, training) -> bool:
        """fp8 training with the token count on whole MX-fp8 K-tiles: a LayerNorm whose output feeds
        only `lin` emits that GEMM's MX operands itself (no bf16 output, no quantize pass)."""
        return MX_PRODUCERS and lin.fp8 and training and (x.numel() // x.shape[-1]) % 128 == 0

    def _self_attn(self, x, B, S, kv_len, causal, seed, training):
        cfg = self.cfg
        a, st1 = self.ln1.forward(x, mx_out=self._mx(x, self.att.qkv, training))
        qkv = self.att.qkv.forward(a)
        n = self.att.names
        sp = TR.AttnSpec(B, cfg.heads, S, S, (qkv, self.att.qkv.col(n["q"])), (qkv, self.att.qkv.col(n["k"])),
                         (qkv, self.att.qkv.col(n["v"])), kv_len=kv_len, causal=causal,
                         p_drop=cfg.attn_dropout if training else 0.0, seed=_mix(seed, 1))
        o, lse = TR.attention_fwd(sp)
        x1 = self.att.out.forward(o, resid=x, drop_p=cfg.dropout if training else 0.0, drop_seed=_mix(seed, 2))
        return x1, (x, a, st1, qkv, sp, o, lse)

    # Backward plumbing of the residual dropouts: every sublayer's LayerNorm backward also writes the
    # gradient its CONSUMER's dropout backward needs (out_drop = (p, seed) of that dropout), so the
    # consumer takes it as `din` instead of running a separate dropout pass over dx.
    def _self_attn_bwd(self, dx1, saved, seed, training, din=None, out_drop=None):
        x, a, st1, qkv, sp, o, lse = saved
        n = self.att.names
        fused = din is not None and _sink(self.att.out) is not None  # din's producer reduced our bias grad
        if din is None:
            din = E.dropout(dx1, self.cfg.dropout if training else 0.0, _mix(seed, 2))
        do = self.att.out.backward(din, o, bias_done=fused)
        dqkv = torch.empty_like(qkv)
        TR.attention_bwd(sp, o, do, lse, (dqkv, self.att.qkv.col(n["q"])), (dqkv, self.att.qkv.col(n["k"])),
                         (dqkv, self.att.qkv.col(n["v"])))
        da = self.att.qkv.backward(dqkv, a)
        return self.ln1.backward(da, x, st1, dres=dx1, drop=out_drop)

    def _ffn(self, x, seed, training):
        cfg = self.cfg
        b, st = self.ffn_ln.forward(x, mx_out=self._mx(x, self.ff1, training))
        # relu: the FFN's activation backward only needs relu'(z) -> a 1-bit mask instead of bf16 z
        # (1/16 of the bytes written here and read back by ff2's dgrad epilogue)
        # (A/B same box: bf16 19.11 -> 18.70 ms/step, MX-fp8 18.04 -> 17.59)
        z = torch.empty(b.shape[0], cfg.ffn // 8, dtype=torch.uint8, device=x.device)
        # fp8 training: ff1's epilogue writes MX(f) / MX(f^T) for ff2's forward and weight gradient --
        # f itself is never read (ff2's dgrad takes relu' from z), so its bf16 store is skipped
        mx = MX_PRODUCERS and self.ff1.fp8 and self.ff2.fp8 and training and b.shape[0] % 128 == 0
        f = self.ff1.forward(b, act="relu", aux=z, drop_p=cfg.relu_dropout if training else 0.0,
                             drop_seed=_mix(seed, 5), mx_out=mx, mx_skip_c=mx and F8.MX_WGRAD)
        x2 = self.ff2.forward(f, resid=x, drop_p=cfg.dropout if training else 0.0, drop_seed=_mix(seed, 6))
        return x2, (x, b, st, z, f)

    def _ffn_bwd(self, dx2, saved, seed, training, din=None, out_drop=None):
        cfg = self.cfg
        x, b, st, z, f = saved
        fused = din is not None and _sink(self.ff2) is not None
        dy = din if din is not None else E.dropout(dx2, cfg.dropout if training else 0.0, _mix(seed, 6))
        # relu backward and the relu-dropout backward in the ff2 dgrad epilogue (forward mask regenerated)
        # ff1's bias gradient = column sums of dz, accumulated by that same epilogue; in fp8 the MX(dz)
        # copies then serve ff1's dgrad and weight gradient and the bf16 dz is never stored
        sink1 = self.ff1.bias_sink()  # (same box: bf16 18.29 -> 18.21 ms/step, MX-fp8 17.47 -> 17.32)
        mx = MX_PRODUCERS and self.ff1.fp8
        # no bf16 dz only when both its consumers take MX copies: ff1's weight gradient reads bf16 dz
        # unless it runs in MX-fp8 too (F8.MX_WGRAD)
        only = mx and F8.MX_WGRAD and sink1 is not None and (dy.numel() // dy.shape[-1]) % 128 == 0
        dz = self.ff2.backward(dy, f, dact_src=z, dact="relu", drop_p=cfg.relu_dropout if training else 0.0,
                               drop_seed=_mix(seed, 5), mx_dx=mx,  # fp8: MX(dz) for ff1
                               bias_done=fused, dx_bias=sink1, mx_dx_only=only)
        db = self.ff1.backward(dz, b, bias_done=sink1 is not None)
        return self.ffn_ln.backward(db, x, st, dres=dx2, drop=out_drop)

    def forward(self, x, B, S, kv_len, seed, training):
        x1, s1 = self._self_attn(x, B, S, kv_len, False, seed, training)
        x2, s2 = self._ffn(x1, seed, training)
        self.saved = (s1, s2, seed, training) if training else None
        return x2

    def in_drop(self, training: bool, seed: int):
        """(p, seed) of the dropout whose backward consumes this layer's output gradient first (the
        FFN output dropout), for the producer's fused LayerNorm-backward output."""
        return (self.cfg.dropout if training else 0.0, _mix(seed, 6), _sink(self.ff2))

    def backward(self, dx2, din=None, out_drop=None):
        """din: dropout(dx2) already produced by the caller's LayerNorm backward (None: computed
        here). out_drop: (p, seed) of the consumer of the returned gradient -> returns (dx, dxd)."""
        s1, s2, seed, training = self.saved
        self.saved = None
        dx1, dx1d = self._ffn_bwd(dx2, s2, seed, training, din=din,
                                  out_drop=(self.cfg.dropout if training else 0.0, _mix(seed, 2), _sink(self.att.out)))
        return self._self_attn_bwd(dx1, s1, seed, training, din=dx1d, out_drop=out_drop)


class DecoderLayer(EncoderLayer):
    def __init__(self, arena: ParamArena, cfg: TransformerConfig, pre: str):
        W = cfg.hidden
        self.cfg = cfg
        self.ln1 = LayerNorm(arena, f"{pre}/self_attention/layer_prepostprocess/layer_norm", W, cfg.ln_eps,
                             ("layer_norm_scale", "layer_norm_bias"))
        self.att = _Attn(arena, f"{pre}/self_attention", W, cross=False)
        self.ln2 = LayerNorm(arena, f"{pre}/encdec_attention/layer_prepostprocess/layer_norm", W, cfg.ln_eps,
                             ("layer_norm_scale", "layer_norm_bias"))
        self.xatt = _Attn(arena, f"{pre}/encdec_attention", W, cross=True)
        self.ln3 = LayerNorm(arena, f"{pre}/ffn/layer_prepostprocess/layer_norm", W, cfg.ln_eps,
                             ("layer_norm_scale", "layer_norm_bias"))
        self.ff1 = Linear(arena, f"{pre}/ffn/conv1", W, cfg.ffn, init="trunc_normal", std=W ** -0.5)
        self.ff2 = Linear(arena, f"{pre}/ffn/conv2", cfg.ffn, W, init="trunc_normal", std=cfg.ffn ** -0.5)
        self.ffn_ln = self.ln3
        self.saved = None

    def forward(self, y, mem, B, St, Ss, src_len, seed, training):
        cfg = self.cfg
        y1, s1 = self._self_attn(y, B, St, None, True, seed, training)
        c, st2 = self.ln2.forward(y1, mx_out=self._mx(y1, self.xatt.q, training))
        q = self.xatt.q.forward(c)
        kv = self.xatt.kv.forward(mem)
        n = self.xatt.names
        sp = TR.AttnSpec(B, cfg.heads, St, Ss, (q, 0), (kv, self.xatt.kv.col(n["k"])), (kv, self.xatt.kv.col(n["v"])),
                         kv_len=src_len, p_drop=cfg.attn_dropout if training else 0.0, seed=_mix(seed, 3))
        o2, lse2 = TR.attention_fwd(sp)
        y2 = self.xatt.out.forward(o2, resid=y1, drop_p=cfg.dropout if training else 0.0, drop_seed=_mix(seed, 4))
        y3, s3 = self._ffn(y2, seed, training)
        self.saved = (s1, (y1, c, st2, q, kv, sp, o2, lse2), s3, seed, training) if training else None
        return y3

    def backward(self, dy3, mem, dmem, din=None, out_drop=None):
        """Returns dy (or (dy, dropout(dy)) with out_drop, see EncoderLayer.backward); accumulates this
        layer's encoder-memory gradient into dmem (in place)."""
        s1, s2, s3, seed, training = self.saved
        self.saved = None
        cfg = self.cfg
        p = cfg.dropout if training else 0.0
        dy2, dy2d = self._ffn_bwd(dy3, s3, seed, training, din=din, out_drop=(p, _mix(seed, 4), _sink(self.xatt.out)))
        y1, c, st2, q, kv, sp, o2, lse2 = s2
        n = self.xatt.names
        do2 = self.xatt.out.backward(dy2d, o2, bias_done=_sink(self.xatt.out) is not None)
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        TR.attention_bwd(sp, o2, do2, lse2, (dq, 0), (dkv, self.xatt.kv.col(n["k"])), (dkv, self.xatt.kv.col(n["v"])))
        dmem.copy_(self.xatt.kv.backward(dkv, mem, resid=dmem))
        dc = self.xatt.q.backward(dq, c)
        dy1, dy1d = self.ln2.backward(dc, y1, st2, dres=dy2, drop=(p, _mix(seed, 2), _sink(self.att.out)))
        return self._self_attn_bwd(dy1, s1, seed, training, din=dy1d, out_drop=out_drop)


class Transformer:
    def __init__(self, cfg: TransformerConfig | None = None):
        cfg = cfg or TransformerConfig.big()
        if cfg.hidden != cfg.heads * TR.HEAD_DIM:
            raise ValueError("tfk attention kernels use head_dim 64: hidden must equal heads*64")
        self.cfg = cfg
        self.name = {1024: "transformer-big", 512: "transformer-base"}.get(cfg.hidden, "transformer")
        self.num_classes = cfg.vocab_size
        self.training = True
        self.step = 0
        W = cfg.hidden
        a = self.arena = ParamArena()
        # dropout RNG: int64 [counter, key] on the device, advanced INSIDE every training step
        # (hipGraph-replayable); kernels use seed = per-site host salt + key (ops.elementwise.rng_key).
        # A checkpointed buffer, so a resumed job continues the mask sequence; rng_stream (e.g. the
        # data-parallel rank) gives each replica its own masks.
        self.rng_state = a.add_buffer("tfk/dropout_rng_state", torch.zeros(2, dtype=torch.int64))
        self.rng_stream = 0
        self.emb = Embedding(a, f"transformer/symbol_modality_{cfg.vocab_size}_{W}/shared/weights", cfg.vocab_size, W,
                             std=W ** -0.5)
        self.enc = [EncoderLayer(a, cfg, f"transformer/body/encoder/layer_{i}") for i in range(cfg.enc_layers)]
        self.enc_ln = LayerNorm(a, "transformer/body/encoder/layer_prepostprocess/layer_norm", W, cfg.ln_eps,
                                ("layer_norm_scale", "layer_norm_bias"))
        self.dec = [DecoderLayer(a, cfg, f"transformer/body/decoder/layer_{i}") for i in range(cfg.dec_layers)]
        self.dec_ln = LayerNorm(a, "transformer/body/decoder/layer_prepostprocess/layer_norm", W, cfg.ln_eps,
                                ("layer_norm_scale", "layer_norm_bias"))
        self._pos = None
        self._wq = None
        self._fp8_lins = []
        if cfg.fp8:
            for layer in self.enc + self.dec:
                for lin in [layer.att.qkv, layer.att.out, layer.ff1, layer.ff2] + (
                        [layer.xatt.q, layer.xatt.kv, layer.xatt.out] if isinstance(layer, DecoderLayer) else []):
                    lin.fp8 = True
                    self._fp8_lins.append(lin)

    def to(self, device, seed: int = 1234):
        self.arena.finalize(device, seed)
        self._wq = None
        self._pos = timing_signal(self.cfg.max_len, self.cfg.hidden).to(torch.bfloat16).to(device)
        return self

    def train(self, mode: bool = True):
        self.training = mode
        return self

    def _embed(self, ids, S, seed, training):
        cfg = self.cfg
        x = TR.embedding_fwd(ids, self.emb.table.compute, self._pos, S, scale=math.sqrt(cfg.hidden))
        return E.dropout(x, cfg.dropout if training else 0.0, seed)

    def _forward(self, src, tgt_in, src_len, B, Ss, St, seed, training):
        x = self._embed(src, Ss, _mix(seed, 0xE0), training)
        for i, layer in enumerate(self.enc):
            x = layer.forward(x, B, Ss, src_len, _mix(seed, 100 + i), training)
        # fp8: the encoder memory feeds only the decoders' cross-attention K/V GEMMs, the final
        # decoder state only the tied logits GEMM -> MX outputs straight from the LayerNorm
        mx = MX_PRODUCERS and self.cfg.fp8 and training and (x.numel() // x.shape[-1]) % 128 == 0
        mem, st_m = self.enc_ln.forward(x, mx_out=mx and all(l.xatt.kv.fp8 for l in self.dec))
        y = self._embed(tgt_in, St, _mix(seed, 0xE1), training)
        for i, layer in enumerate(self.dec):
            y = layer.forward(y, mem, B, St, Ss, src_len, _mix(seed, 200 + i), training)
        yo, st_y = self.dec_ln.forward(y, mx_out=MX_PRODUCERS and self.cfg.fp8 and training
                                       and (y.numel() // y.shape[-1]) % 128 == 0)
        from ..runtime.layers import linear_forward
        logits = linear_forward(yo, self.emb.table.compute, None, self.cfg.fp8)  # tied softmax weights
        return logits, (x, mem, st_m, y, yo, st_y)

    def forward_backward(self, src, tgt_in, tgt_out, src_len, loss_scale: float = 1.0):
        """One training step's forward + backward (see _forward_backward). The no-decay gradients
        (biases, LayerNorm gamma/beta) are zeroed in one fill up front and accumulated by their kernels."""
        self.arena.zero_nodecay_grads()
        E.rng_advance(self.rng_state, self.rng_stream)
        if self.cfg.fp8:
            from ..ops.fp8 import clear_saved
            from ..runtime.layers import weight_quantizer
            clear_saved()  # transposed MX operands live from this step's forward to its backward
            # every fp8 weight (and the tied softmax table) quantized both ways in ONE launch
            weight_quantizer(self, self._fp8_lins, [self.emb.table.compute]).run()
        try:
            with E.rng_key(self.rng_state):
                return self._forward_backward(src, tgt_in, tgt_out, src_len, loss_scale)
        finally:
            self.arena.prezeroed = False
            if self.cfg.fp8:
                from ..ops.fp8 import clear_saved
                clear_saved()  # nothing quantized in this step may leak into a later forward

    def _forward_backward(self, src, tgt_in, tgt_out, src_len, loss_scale: float = 1.0):
        cfg = self.cfg
        B = src_len.shape[0]
        Ss, St = src.numel() // B, tgt_in.numel() // B
        self.step += 1
        seed = 0x7EA  # salt base; the per-step part is the device key (rng_state)
        tr = self.training
        logits, (x, mem, st_m, y, yo, st_y) = self._forward(src, tgt_in, src_len, B, Ss, St, seed, tr)
        loss, dlogits, corr = softmax_xent(logits, tgt_out, smoothing=cfg.label_smoothing,
                                           scale=loss_scale / tgt_out.numel(), want_correct=True, V=cfg.vocab_size)
        from ..runtime.layers import fp8_dy, linear_dgrad, linear_wgrad
        # fp8: MX(dlogits) and MX(dlogits^T) from ONE read of the [tokens, vocab] gradient (separate
        # row + transposing passes were 0.53 ms/step; profiles/transformer_big_fp8_bs32_1gpu_kernels_r3b.txt)
        dyq, dyt = fp8_dy(dlogits, cfg.hidden, cfg.fp8)
        linear_wgrad(dlogits, yo, self.emb.table.grad, cfg.fp8, dyt=dyt)  # first writer of the shared table's grad
        dyo = linear_dgrad(dlogits, self.emb.table.compute, cfg.fp8, dyq=dyq)
        # each LayerNorm backward also emits dropout(dx) for the dropout its gradient flows into next
        p = cfg.dropout if tr else 0.0
        nd, ne = len(self.dec), len(self.enc)
        dy, dyd = self.dec_ln.backward(dyo, y, st_y, drop=self.dec[-1].in_drop(tr, _mix(seed, 200 + nd - 1)))
        dmem = torch.zeros_like(mem)
        for i in range(nd - 1, -1, -1):
            nxt = self.dec[i - 1].in_drop(tr, _mix(seed, 200 + i - 1)) if i > 0 else (p, _mix(seed, 0xE1))
            dy, dyd = self.dec[i].backward(dy, mem, dmem, din=dyd, out_drop=nxt)
            streams.flush()  # this layer's weight gradients, concurrent with the next layer's dgrads
        scale = math.sqrt(cfg.hidden)
        TR.embedding_bwd(tgt_in, dyd, self.emb.table.grad, None, St, scale=scale)
        dx, dxd = self.enc_ln.backward(dmem, x, st_m, drop=self.enc[-1].in_drop(tr, _mix(seed, 100 + ne - 1)))
        for i in range(ne - 1, -1, -1):
            nxt = self.enc[i - 1].in_drop(tr, _mix(seed, 100 + i - 1)) if i > 0 else (p, _mix(seed, 0xE0))
            dx, dxd = self.enc[i].backward(dx, din=dxd, out_drop=nxt)
            streams.flush()
        TR.embedding_bwd(src, dxd, self.emb.table.grad, None, Ss, scale=scale)
        streams.join()  # side-stream weight gradients complete before anyone reads arena.grad
        self.arena.grad_ready(self.emb.table)
        return loss.view(B, St).mean(1), corr

    def evaluate(self, src, tgt_in, tgt_out, src_len):
        B = src_len.shape[0]
        logits, _ = self._forward(src, tgt_in, src_len, B, src.numel() // B, tgt_in.numel() // B, 0, False)
        loss, _, corr = softmax_xent(logits, tgt_out, want_grad=False, want_correct=True, V=self.cfg.vocab_size)
        return float(loss.sum()), float(corr.sum()), int(corr.numel())

    def synthetic_batch(self, batch: int, device, seed: int = 0, seq_len: int | None = None, **_):
        """WMT-shaped synthetic batch: full-length source/target token ids (shifted target)."""
        cfg = self.cfg
        Ss = seq_len or cfg.src_len
        St = seq_len or cfg.tgt_len
        g = torch.Generator().manual_seed(seed)
        src = torch.randint(2, cfg.vocab_size, (batch, Ss), generator=g, dtype=torch.int32)
        tgt = torch.randint(2, cfg.vocab_size, (batch, St + 1), generator=g, dtype=torch.int32)
        tgt[:, 0] = 0
        src_len = torch.full((batch,), Ss, dtype=torch.int32)
        return tuple(t.contiguous().to(device) for t in (src.reshape(-1), tgt[:, :-1].reshape(-1),
                                                       tgt[:, 1:].reshape(-1), src_len))
