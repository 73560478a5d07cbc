"""Plain-torch fp32 autograd references of the tfk models, driven by the SAME arena weights.
Used as the numerics oracle for the executor's hand-written backward passes."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _bn(x, gamma, beta, eps):
    # x NCHW, training-mode batch statistics (biased variance)
    mean = x.mean(dim=(0, 2, 3), keepdim=True)
    var = x.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
    return (x - mean) / torch.sqrt(var + eps) * gamma[None, :, None, None] + beta[None, :, None, None]


class _Round(torch.autograd.Function):
    """bf16 storage of an activation AND of its gradient, as the executor keeps them."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


def resnet_loss(model, x_nhwc, labels, smoothing, emulate_bf16=False):
    """Returns (loss, {param_name: leaf tensor}) with leaves in storage layout (f32). With
    emulate_bf16 the activations/weights are rounded to bf16 where the executor stores them:
    random-init deep ResNets are chaotic enough that pure-fp32 and bf16 forwards drift apart by
    ~50% at the last stage (measured), so exact-ish comparisons need the emulated reference."""
    leaves = {p.name: p.master.detach().clone().float().requires_grad_(True) for p in model.arena.params}
    rd = _Round.apply if emulate_bf16 else (lambda t: t)

    def conv(layer, h):
        w = leaves[layer.w.name].permute(0, 3, 1, 2)
        if emulate_bf16:
            w = w.to(torch.bfloat16).float()
        return rd(F.conv2d(h, w, stride=layer.stride, padding=layer.pad))

    def bn(layer, h):
        return _bn(h, leaves[layer.gamma.name], leaves[layer.beta.name], layer.eps)

    h = x_nhwc.float().permute(0, 3, 1, 2)
    h = rd(F.relu(bn(model.bn1, conv(model.conv1, h))))
    h = F.max_pool2d(h, 3, 2, 1)
    for b in model.blocks:
        o = rd(F.relu(bn(b.bn1, conv(b.conv1, h))))
        o = rd(F.relu(bn(b.bn2, conv(b.conv2, o))))
        o = bn(b.bn3, conv(b.conv3, o))
        sc = bn(b.bn_sc, conv(b.conv_sc, h)) if b.proj else h
        h = rd(F.relu(o + sc))
    f = rd(h.mean(dim=(2, 3)))
    wfc = leaves[model.fc.w.name]
    if emulate_bf16:
        wfc = wfc.to(torch.bfloat16).float()
    logits = rd(f @ wfc.t() + leaves[model.fc.b.name])
    loss = F.cross_entropy(logits, labels.long(), label_smoothing=smoothing)
    return loss, leaves


# ----------------------------------------------------------------------------- BERT (fp32 autograd)
def bert_ref_loss(model, ids, tt, mlm_pos, mlm_ids, nsp_labels):
    """fp32 torch-autograd BERT pretraining loss over the SAME arena parameters (dropout off).
    Returns (loss, {param name: grad tensor in storage layout})."""
    import torch.nn.functional as F
    cfg = model.cfg
    params = {p.name: p.master.detach().float().clone().requires_grad_(True) for p in model.arena.params}
    B = nsp_labels.shape[0]
    S = ids.numel() // B
    W, H = cfg.hidden, cfg.heads

    def lin(x, name, kernel="kernel"):
        return x @ params[f"{name}/{kernel}"].t() + params[f"{name}/bias"]

    def ln(x, name):
        return F.layer_norm(x, (W,), params[f"{name}/gamma"], params[f"{name}/beta"], cfg.ln_eps)

    gelu = lambda x: F.gelu(x, approximate="tanh")
    word = params["bert/embeddings/word_embeddings"]
    e = word[ids.long()] + params["bert/embeddings/position_embeddings"][:S].repeat(B, 1) + \
        params["bert/embeddings/token_type_embeddings"][tt.long()]
    h = ln(e, "bert/embeddings/LayerNorm")
    for i in range(cfg.layers):
        pre = f"bert/encoder/layer_{i}"
        q, k, v = (lin(h, f"{pre}/attention/self/{n}").view(B, S, H, 64).transpose(1, 2) for n in ("query", "key", "value"))
        a = torch.softmax(q @ k.transpose(-1, -2) / 8.0, -1) @ v
        o = a.transpose(1, 2).reshape(B * S, W)
        h1 = ln(lin(o, f"{pre}/attention/output/dense") + h, f"{pre}/attention/output/LayerNorm")
        f = gelu(lin(h1, f"{pre}/intermediate/dense"))
        h = ln(lin(f, f"{pre}/output/dense") + h1, f"{pre}/output/LayerNorm")
    P = mlm_pos.shape[1]
    rows = (mlm_pos.long() + torch.arange(B)[:, None] * S).reshape(-1)
    t = ln(gelu(lin(h[rows], "cls/predictions/transform/dense")), "cls/predictions/transform/LayerNorm")
    logits = (t @ word.t() + params["cls/predictions/output_bias"])[:, :cfg.vocab_size]
    mlm = F.cross_entropy(logits, mlm_ids.reshape(-1).long())
    pooled = torch.tanh(lin(h[torch.arange(B) * S], "bert/pooler/dense"))
    nsp_logits = pooled @ params["cls/seq_relationship/output_weights"].t() + params["cls/seq_relationship/output_bias"]
    nsp = F.cross_entropy(nsp_logits, nsp_labels.long())
    loss = mlm + nsp
    loss.backward()
    return float(loss.detach()), {n: t.grad for n, t in params.items()}


# ----------------------------------------------------------------------------- Transformer (fp32 autograd)
def transformer_ref_loss(model, src, tgt_in, tgt_out, src_len):
    """fp32 autograd pre-LN encoder-decoder over the same arena parameters (dropout off)."""
    import math
    import torch.nn.functional as F
    cfg = model.cfg
    P = {p.name: p.master.detach().float().clone().requires_grad_(True) for p in model.arena.params}
    B = src_len.shape[0]
    Ss, St, W, H = src.numel() // B, tgt_in.numel() // B, cfg.hidden, cfg.heads
    E = P[f"transformer/symbol_modality_{cfg.vocab_size}_{W}/shared/weights"]
    from tensorflow_k8s_amd.models.transformer import timing_signal
    pos = timing_signal(cfg.max_len, W).to(torch.bfloat16).float()

    def ln(x, name):
        return F.layer_norm(x, (W,), P[f"{name}/layer_norm/layer_norm_scale"], P[f"{name}/layer_norm/layer_norm_bias"],
                            cfg.ln_eps)

    def attn(xq, xkv, base, Sq, Sk, causal):
        q = (xq @ P[f"{base}/q/kernel"].t()).view(B, Sq, H, 64).transpose(1, 2)
        k = (xkv @ P[f"{base}/k/kernel"].t()).view(B, Sk, H, 64).transpose(1, 2)
        v = (xkv @ P[f"{base}/v/kernel"].t()).view(B, Sk, H, 64).transpose(1, 2)
        s = q @ k.transpose(-1, -2) / 8.0
        if causal:
            s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool).triu(1), float("-inf"))
        o = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B * Sq, W)
        return o @ P[f"{base}/output_transform/kernel"].t()

    def ffn(x, pre):
        h = torch.relu(x @ P[f"{pre}/ffn/conv1/kernel"].t() + P[f"{pre}/ffn/conv1/bias"])
        return h @ P[f"{pre}/ffn/conv2/kernel"].t() + P[f"{pre}/ffn/conv2/bias"]

    x = E[src.long()] * math.sqrt(W) + pos[:Ss].repeat(B, 1)
    for i in range(cfg.enc_layers):
        pre = f"transformer/body/encoder/layer_{i}"
        a = ln(x, f"{pre}/self_attention/layer_prepostprocess")
        x = x + attn(a, a, f"{pre}/self_attention/multihead_attention", Ss, Ss, False)
        x = x + ffn(ln(x, f"{pre}/ffn/layer_prepostprocess"), pre)
    mem = ln(x, "transformer/body/encoder/layer_prepostprocess")
    y = E[tgt_in.long()] * math.sqrt(W) + pos[:St].repeat(B, 1)
    for i in range(cfg.dec_layers):
        pre = f"transformer/body/decoder/layer_{i}"
        a = ln(y, f"{pre}/self_attention/layer_prepostprocess")
        y = y + attn(a, a, f"{pre}/self_attention/multihead_attention", St, St, True)
        c = ln(y, f"{pre}/encdec_attention/layer_prepostprocess")
        y = y + attn(c, mem, f"{pre}/encdec_attention/multihead_attention", St, Ss, False)
        y = y + ffn(ln(y, f"{pre}/ffn/layer_prepostprocess"), pre)
    yo = ln(y, "transformer/body/decoder/layer_prepostprocess")
    logits = (yo @ E.t())[:, :cfg.vocab_size]
    loss = F.cross_entropy(logits, tgt_out.long(), label_smoothing=cfg.label_smoothing)
    loss.backward()
    return float(loss.detach()), {n: t.grad for n, t in P.items()}
