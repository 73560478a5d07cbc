#!/usr/bin/env python3
"""Stock PyTorch-ROCm comparators for the token workloads (BASELINE configs 3 and 5), written the
way a user would without tfk: torch.nn layers (hipBLASLt GEMMs), F.scaled_dot_product_attention,
PyTorch's fused optimizer, synthetic data of the bench's exact shapes, random init.

    python tools/stock_transformer.py --model bert-base        [--precision bf16|autocast] [--compile 1]
    python tools/stock_transformer.py --model transformer-big  [--precision bf16|autocast] [--compile 1]

bert-base: 12 x (768, 12 heads, 3072 GELU) encoder, MLM head on 20 positions/sequence tied to the
30522-word embedding + NSP, batch 64 x 128. tfk trains it with LAMB; torch has no LAMB, so the
comparator uses fused AdamW (same moment traffic, no trust-ratio reduction: slightly in torch's favour).
transformer-big: 6+6 layers, d 1024, 16 heads, FFN 4096 ReLU, shared 33708 vocabulary tied to the
output projection, label smoothing 0.1, Adam(0.9, 0.98), batch 32 x (256 + 256).
precision bf16: weights/activations bf16 (fused optimizer on bf16 params); autocast: f32 master
weights under bf16 autocast (tfk's arrangement: f32 master + bf16 compute copy).
Tokens/s counts the same tokens as bench.py (BERT: B*S, Transformer: B*(S_src+S_tgt)).
"""
import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class MHA(nn.Module):
    def __init__(self, d, h, p):
        super().__init__()
        self.h, self.p = h, p
        self.qkv = nn.Linear(d, 3 * d)
        self.o = nn.Linear(d, d)

    def forward(self, x, mem=None, causal=False):
        B, S, D = x.shape
        if mem is None:
            q, k, v = self.qkv(x).view(B, S, 3, self.h, D // self.h).permute(2, 0, 3, 1, 4)
        else:
            w_q, w_kv = self.qkv.weight.split([D, 2 * D]), None
            b_q, b_kv = self.qkv.bias.split([D, 2 * D])
            q = F.linear(x, w_q[0], b_q).view(B, S, self.h, D // self.h).transpose(1, 2)
            k, v = F.linear(mem, w_q[1], b_kv).view(B, mem.shape[1], 2, self.h, D // self.h).permute(2, 0, 3, 1, 4)
        y = F.scaled_dot_product_attention(q, k, v, dropout_p=self.p if self.training else 0.0, is_causal=causal)
        return self.o(y.transpose(1, 2).reshape(B, S, D))


class Block(nn.Module):
    """Post-LN (BERT) or pre-LN (Transformer) residual block with optional cross-attention."""

    def __init__(self, d, h, ffn, p, act, pre_ln, cross=False, eps=1e-12):
        super().__init__()
        self.pre_ln = pre_ln
        self.att, self.ln1 = MHA(d, h, p), nn.LayerNorm(d, eps=eps)
        self.cross = MHA(d, h, p) if cross else None
        self.ln_c = nn.LayerNorm(d, eps=eps) if cross else None
        self.ff1, self.ff2, self.ln2 = nn.Linear(d, ffn), nn.Linear(ffn, d), nn.LayerNorm(d, eps=eps)
        self.act, self.drop = act, nn.Dropout(p)

    def _res(self, x, ln, f):
        if self.pre_ln:
            return x + self.drop(f(ln(x)))
        return ln(x + self.drop(f(x)))

    def forward(self, x, mem=None, causal=False):
        x = self._res(x, self.ln1, lambda t: self.att(t, causal=causal))
        if self.cross is not None:
            x = self._res(x, self.ln_c, lambda t: self.cross(t, mem))
        return self._res(x, self.ln2, lambda t: self.ff2(self.drop(self.act(self.ff1(t)))))


class Bert(nn.Module):
    def __init__(self, V=30522, d=768, L=12, h=12, ffn=3072, S=512):
        super().__init__()
        self.word, self.pos, self.typ = nn.Embedding(V, d), nn.Embedding(S, d), nn.Embedding(2, d)
        self.ln, self.drop = nn.LayerNorm(d, eps=1e-12), nn.Dropout(0.1)
        self.layers = nn.ModuleList([Block(d, h, ffn, 0.1, F.gelu, pre_ln=False) for _ in range(L)])
        self.mlm_dense, self.mlm_ln = nn.Linear(d, d), nn.LayerNorm(d, eps=1e-12)
        self.mlm_bias = nn.Parameter(torch.zeros(V))
        self.pooler, self.nsp = nn.Linear(d, d), nn.Linear(d, 2)

    def forward(self, ids, tt, pos, mlm_ids, nsp):
        B, S = ids.shape
        x = self.drop(self.ln(self.word(ids) + self.pos.weight[:S] + self.typ(tt)))
        for l in self.layers:
            x = l(x)
        hm = torch.gather(x, 1, pos.unsqueeze(-1).expand(-1, -1, x.shape[-1]))
        t = self.mlm_ln(F.gelu(self.mlm_dense(hm)))
        logits = F.linear(t, self.word.weight, self.mlm_bias)
        nsp_logits = self.nsp(torch.tanh(self.pooler(x[:, 0])))
        return F.cross_entropy(logits.flatten(0, 1).float(), mlm_ids.flatten()) + F.cross_entropy(nsp_logits.float(), nsp)


class TransformerBig(nn.Module):
    def __init__(self, V=33708, d=1024, L=6, h=16, ffn=4096, p=0.3):
        super().__init__()
        self.emb, self.d = nn.Embedding(V, d), d
        self.pe = nn.Parameter(torch.randn(1024, d) * 0.02, requires_grad=False)
        self.enc = nn.ModuleList([Block(d, h, ffn, p, F.relu, pre_ln=True, eps=1e-6) for _ in range(L)])
        self.dec = nn.ModuleList([Block(d, h, ffn, p, F.relu, pre_ln=True, cross=True, eps=1e-6) for _ in range(L)])
        self.ln_e, self.ln_d, self.drop = nn.LayerNorm(d, eps=1e-6), nn.LayerNorm(d, eps=1e-6), nn.Dropout(p)

    def forward(self, src, tgt_in, tgt_out):
        s = self.drop(self.emb(src) * self.d ** 0.5 + self.pe[:src.shape[1]])
        for l in self.enc:
            s = l(s)
        mem = self.ln_e(s)
        t = self.drop(self.emb(tgt_in) * self.d ** 0.5 + self.pe[:tgt_in.shape[1]])
        for l in self.dec:
            t = l(t, mem, causal=True)
        logits = F.linear(self.ln_d(t), self.emb.weight)
        return F.cross_entropy(logits.flatten(0, 1).float(), tgt_out.flatten(), label_smoothing=0.1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-base", choices=["bert-base", "transformer-big"])
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "autocast"])
    ap.add_argument("--compile", type=int, default=0)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    if a.model == "bert-base":
        B, S, P, V = a.batch or 64, 128, 20, 30522
        m = Bert().to(dev)
        batch = (torch.randint(0, V, (B, S), device=dev, generator=g), torch.randint(0, 2, (B, S), device=dev, generator=g),
                 torch.randint(0, S, (B, P), device=dev, generator=g), torch.randint(0, V, (B, P), device=dev, generator=g),
                 torch.randint(0, 2, (B,), device=dev, generator=g))
        tokens = B * S
        opt_kw = dict(lr=1e-4, weight_decay=0.01)
    else:
        B, S, V = a.batch or 32, 256, 33708
        m = TransformerBig().to(dev)
        batch = (torch.randint(0, V, (B, S), device=dev, generator=g), torch.randint(0, V, (B, S), device=dev, generator=g),
                 torch.randint(0, V, (B, S), device=dev, generator=g))
        tokens = B * 2 * S
        opt_kw = dict(lr=1e-4, betas=(0.9, 0.98), eps=1e-9, weight_decay=0.0)
    if a.precision == "bf16":
        m = m.to(torch.bfloat16)
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], fused=True, **opt_kw)
    fwd = torch.compile(m) if a.compile else m

    def step():
        opt.zero_grad(set_to_none=True)
        if a.precision == "autocast":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = fwd(*batch)
        else:
            loss = fwd(*batch)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"comparator": f"stock_pytorch_{a.precision}" + ("_compile" if a.compile else ""),
                      "model": a.model, "batch": B, "ms_per_step": round(dt * 1000, 3),
                      "tok_s": round(tokens / dt, 1), "loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()
