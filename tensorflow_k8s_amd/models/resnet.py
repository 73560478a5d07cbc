"""ResNet-50/101/152 (v1.5: stride on the 3x3 conv) for the tfk executor, NHWC bf16.

Every conv feeds its BN's batch statistics from the GEMM epilogue; the block tail
relu(bn3(y3) + bn_sc(y_sc) | + x) is ONE fused pass; backward fuses relu-mask + both BNs of the
block tail and adds the identity-shortcut gradient inside the first conv's dgrad epilogue.
Variable names follow the Keras/TF ResNet convention (conv1, bn_conv1, res2a_branch2a, ...,
fc1000) so checkpoints line up with TF-era tooling.
"""
from __future__ import annotations

import os

import torch

from ..ops import norm as BN
from ..ops import pool as PL
from ..ops.loss import softmax_xent
from ..runtime import streams
from ..runtime.arena import ParamArena
from ..runtime.layers import BatchNorm, Conv2d, Linear

# projection shortcut (forward conv, lattice dgrad) on the side stream (runtime/streams.py)
SIDE_SHORTCUT = True
# the dgrad epilogues that feed a BN backward store dz = dA * relu-mask (BNReduce premask): the
# BN-backward apply then reads no mask and an identity block's residual gradient is dz itself (no
# second output pass).
PREMASK = True
# the stem BN + relu applied inside the max-pool forward (ops.pool.maxpool_fwd bn=): no stem activation
# (A/B: TFK_POOL_BN=0)
POOL_BN = os.environ.get("TFK_POOL_BN", "1") != "0"
# the stem BN's backward reduction fused into the max-pool backward (A/B: TFK_POOL_BNR=0)
POOL_BNR = os.environ.get("TFK_POOL_BNR", "1") != "0"
DEPTHS = {18: None, 50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3]}
IN_CH_PAD = 8  # RGB padded to 8 channels -> 16-B NHWC pixels for the implicit-GEMM gather


class Bottleneck:
    def __init__(self, arena, stage: int, idx: int, cin: int, width: int, stride: int):
        tag = f"{stage}{chr(ord('a') + idx)}"
        cout = width * 4
        self.stride = stride
        self.conv1 = Conv2d(arena, f"res{tag}_branch2a", cin, width, 1)
        self.bn1 = BatchNorm(arena, f"bn{tag}_branch2a", width)
        self.conv2 = Conv2d(arena, f"res{tag}_branch2b", width, width, 3, stride=stride)
        self.bn2 = BatchNorm(arena, f"bn{tag}_branch2b", width)
        self.conv3 = Conv2d(arena, f"res{tag}_branch2c", width, cout, 1)
        self.bn3 = BatchNorm(arena, f"bn{tag}_branch2c", cout, zero_gamma=True)
        self.proj = stride != 1 or cin != cout
        if self.proj:
            self.conv_sc = Conv2d(arena, f"res{tag}_branch1", cin, cout, 1, stride=stride, pad=0)
            self.bn_sc = BatchNorm(arena, f"bn{tag}_branch1", cout)
        self.arena = arena

    def bns(self):
        return [self.bn1, self.bn2, self.bn3] + ([self.bn_sc] if self.proj else [])

    def forward(self, x, training=True):
        dev = x.device
        s1, s2, s3 = self.bn1.state(dev), self.bn2.state(dev), self.bn3.state(dev)
        sc = []
        if self.proj and SIDE_SHORTCUT:
            # the projection shortcut only needs x: on the side stream, concurrent with conv1..conv3
            ssc = self.bn_sc.state(dev)

            def shortcut():
                ysc = self.conv_sc.forward(x, ssc if training else None)
                if training:
                    self.bn_sc.finalize(ysc.numel() // ysc.shape[-1], defer=True)
                sc.append(ysc)
            streams.run_wgrad(shortcut, x)
        y1 = self.conv1.forward(x, s1 if training else None)
        if training:
            self.bn1.finalize(y1.numel() // y1.shape[-1], defer=True)
        a1 = BN.bn_apply(y1, s1, relu=True)
        y2 = self.conv2.forward(a1, s2 if training else None)
        if training:
            self.bn2.finalize(y2.numel() // y2.shape[-1], defer=True)
        a2 = BN.bn_apply(y2, s2, relu=True)
        y3 = self.conv3.forward(a2, s3 if training else None)
        if training:
            self.bn3.finalize(y3.numel() // y3.shape[-1], defer=True)
        ysc = None
        if self.proj:
            if not SIDE_SHORTCUT:
                ssc = self.bn_sc.state(dev)
                ysc = self.conv_sc.forward(x, ssc if training else None)
                if training:
                    self.bn_sc.finalize(ysc.numel() // ysc.shape[-1], defer=True)
                sc.append(ysc)
            streams.sync()
            ysc = sc[0]
            out = BN.bn_apply(y3, s3, relu=True, r=ysc, rst=ssc, mask=training)
        else:
            out = BN.bn_apply(y3, s3, relu=True, r=x, mask=training)
        if training:
            # the tail's relu mask is kept as a bitmask (1/16 of out's bytes): the tail BN-backward
            # apply and the next block's fused dgrad reduction read it instead of out
            out, mk = out
            self.saved = (x, y1, a1, y2, a2, y3, ysc, mk)
        return out

    def tail_reduce(self) -> BN.BNReduce:
        """BN-backward reduction spec of this block's tail (relu(bn3(y3) + shortcut)); fused into
        the epilogue of the NEXT block's final dgrad, which produces this block's dout."""
        x, y1, a1, y2, a2, y3, ysc, mk = self.saved
        return BN.BNReduce(y3, self.bn3.st, a=mk, y2=ysc, st2=self.bn_sc.st if self.proj else None, premask=PREMASK)

    def backward(self, dout, need_dx=True, dout_reduced=False, next_bnr: BN.BNReduce | None = None):
        """dout_reduced: the producer of dout already accumulated this block's tail BN sums.
        next_bnr: reduction spec to fuse into the dgrad that produces dx (previous block's tail)."""
        x, y1, a1, y2, a2, y3, ysc, mk = self.saved
        self.saved = None
        cnt3 = y3.numel() // y3.shape[-1]
        if self.proj:
            dy3, dysc, _ = BN.bn_backward(dout, mk, y3, self.bn3.st, self.bn3.gamma.master, self.bn3.gamma.grad,
                                          self.bn3.beta.grad, cnt3, y2=ysc, st2=self.bn_sc.st,
                                          gamma2=self.bn_sc.gamma.master, dgamma2=self.bn_sc.gamma.grad,
                                          dbeta2=self.bn_sc.beta.grad, reduced=dout_reduced,
                                          premasked=dout_reduced and PREMASK)
            dres = None
            self.arena.grad_ready(self.bn3.gamma, self.bn3.beta, self.bn_sc.gamma, self.bn_sc.beta)
        else:
            dy3, _, dres = BN.bn_backward(dout, mk, y3, self.bn3.st, self.bn3.gamma.master, self.bn3.gamma.grad,
                                          self.bn3.beta.grad, cnt3, want_dres=True, reduced=dout_reduced,
                                          premasked=dout_reduced and PREMASK)
            self.arena.grad_ready(self.bn3.gamma, self.bn3.beta)
        lattice = self.proj and self.stride > 1 and need_dx and next_bnr is not None
        tl = []
        if lattice and SIDE_SHORTCUT:
            # the strided projection's lattice dgrad only needs dysc: side stream, concurrent with the
            # conv3 -> conv2 chain, joined before conv1's dgrad epilogue adds it
            streams.run_wgrad(lambda: tl.append(self.conv_sc.lattice_dgrad(dysc, x)), dysc, x)
        # bn2/bn1 have no residual input: relu mask recomputed from y, sums fused into the dgrad epilogue
        da2 = self.conv3.backward(dy3, a2, bnr=BN.BNReduce(y2, self.bn2.st, premask=PREMASK))
        dy2, _, _ = BN.bn_backward(da2, None, y2, self.bn2.st, self.bn2.gamma.master, self.bn2.gamma.grad,
                                   self.bn2.beta.grad, y2.numel() // y2.shape[-1], relu_from_y=True, reduced=True,
                                   premasked=PREMASK)
        self.arena.grad_ready(self.bn2.gamma, self.bn2.beta)
        da1 = self.conv2.backward(dy2, a1, bnr=BN.BNReduce(y1, self.bn1.st, premask=PREMASK))
        dy1, _, _ = BN.bn_backward(da1, None, y1, self.bn1.st, self.bn1.gamma.master, self.bn1.gamma.grad,
                                   self.bn1.beta.grad, y1.numel() // y1.shape[-1], relu_from_y=True, reduced=True,
                                   premasked=PREMASK)
        self.arena.grad_ready(self.bn1.gamma, self.bn1.beta)
        if lattice:
            # strided projection: its dgrad only touches the stride lattice -> a dense GEMM over the
            # P x Q rows, added on the lattice inside conv1's dgrad epilogue (which also carries the
            # previous block's fused BN reduction) instead of a 3/4-zero strided gather
            if not SIDE_SHORTCUT:
                tl.append(self.conv_sc.lattice_dgrad(dysc, x))
            self.conv_sc.wgrad(dysc, x)
            streams.sync()
            t = tl[0]
            dx = self.conv1.backward(dy1, x, need_dx=True, resid=t, resid_stride=self.stride, bnr=next_bnr)
        elif self.proj:
            dx = self.conv1.backward(dy1, x, need_dx=need_dx)
            dx = self.conv_sc.backward(dysc, x, need_dx=need_dx, resid=dx, bnr=next_bnr)
        else:
            dx = self.conv1.backward(dy1, x, need_dx=need_dx, resid=dres, bnr=next_bnr)
        streams.flush()  # this block's deferred weight gradients behind one side-stream fork
        return dx


class ResNet:
    """ResNet v1.5 on the tfk executor. Input: NHWC bf16 [N,224,224,8] (RGB + zero pad)."""

    def __init__(self, depth: int = 50, num_classes: int = 1000, width: int = 64, label_smoothing: float = 0.1,
                 stages: list | None = None):
        if stages is None and (depth not in DEPTHS or DEPTHS[depth] is None):
            raise ValueError(f"unsupported ResNet depth {depth}")
        self.depth, self.num_classes, self.label_smoothing = depth, num_classes, label_smoothing
        self.name = f"resnet{depth}"
        a = self.arena = ParamArena()
        self.conv1 = Conv2d(a, "conv1", IN_CH_PAD, width, 7, stride=2, pad=3, cin_real=3)
        self.bn1 = BatchNorm(a, "bn_conv1", width)
        self.blocks: list[Bottleneck] = []
        cin = width
        for si, n in enumerate(stages or DEPTHS[depth]):
            w = width * (2 ** si)
            for bi in range(n):
                stride = 2 if (bi == 0 and si > 0) else 1
                self.blocks.append(Bottleneck(a, si + 2, bi, cin, w, stride))
                cin = w * 4
        self.fc = Linear(a, "fc1000", cin, num_classes, init="normal", std=0.01)
        self.feat = cin
        self.training = True

    # ------------------------------------------------------------------ setup
    def to(self, device, seed: int = 1234) -> "ResNet":
        self.arena.finalize(device, seed)
        # every BN layer's accumulators in one buffer, zeroed once per training step: the BN passes
        # then finalize their statistics themselves (ops/norm.py BNPool, FUSED_FIN)
        bns = self.batchnorms()
        self._bn_pool = BN.BNPool([bn.C for bn in bns], device)
        for bn, st in zip(bns, self._bn_pool.states):
            bn.st = st
        return self

    def batchnorms(self):
        out = [self.bn1]
        for b in self.blocks:
            out += b.bns()
        return out

    def train(self, mode: bool = True) -> "ResNet":
        self.training = mode
        for bn in self.batchnorms():
            bn.training = mode
        return self

    # ------------------------------------------------------------------ compute
    def _features(self, x):
        dev = x.device
        if self.training and getattr(self, "_bn_pool", None) is not None:
            self._bn_pool.zero()  # this step's BN statistics and backward sums accumulate from zero
        st = self.bn1.state(dev)
        y0 = self.conv1.forward(x, st if self.training else None)
        if self.training:
            self.bn1.finalize(y0.numel() // y0.shape[-1], defer=not POOL_BN)
        else:
            self._eval_stats()
        if POOL_BN:
            # the stem BN's apply runs inside the max pool: its output is read by nothing else
            p0, idx = PL.maxpool_fwd(y0, 3, 2, 1, bn=(st.scale, st.shift))
            a0 = y0.shape
        else:
            a0 = BN.bn_apply(y0, st, relu=True)
            p0, idx = PL.maxpool_fwd(a0, 3, 2, 1)
            a0 = a0.shape
        h = p0
        for b in self.blocks:
            h = b.forward(h, self.training)
        f = PL.avgpool_fwd(h)
        if self.training:
            self._saved = (x, y0, a0, idx, h.shape, f)
        return f

    def _eval_stats(self):
        for bn in self.batchnorms():
            bn.state(self.arena.device)
            bn.use_running_stats()

    def forward(self, x):
        """Eval forward -> logits bf16 [N, classes]."""
        if not self.training:
            self._eval_stats()
        f = self._features(x)
        return self.fc.forward(f)

    def forward_backward(self, x, labels, loss_scale: float = 1.0):
        """One training forward + backward. Returns (loss_sum f32[N] per-row, correct f32[N]).
        Gradients land in arena.grad (mean over the local batch)."""
        f = self._features(x)
        logits = self.fc.forward(f)
        B = logits.shape[0]
        loss, dlogits, corr = softmax_xent(logits, labels, smoothing=self.label_smoothing, scale=loss_scale / B,
                                           want_correct=True)
        df = self.fc.backward(dlogits, f)
        x0, y0, a0, idx, hshape, _ = self._saved
        self._saved = None
        dh = PL.avgpool_bwd(df, hshape)
        nb = len(self.blocks)
        for i in range(nb - 1, -1, -1):
            nxt = self.blocks[i - 1].tail_reduce() if i > 0 else None
            dh = self.blocks[i].backward(dh, dout_reduced=i < nb - 1, next_bnr=nxt)
        # a0: the stem activation's shape; the stem BN's backward sums accumulate inside the pool's
        # backward (relu mask from y0), so no separate reduction pass re-reads dx and y0
        bnr = BN.BNReduce(y0, self.bn1.st) if POOL_BNR else None
        da0 = PL.maxpool_bwd(dh, idx, a0, 3, 2, 1, bnr=bnr)
        dy0, _, _ = BN.bn_backward(da0, None, y0, self.bn1.st, self.bn1.gamma.master, self.bn1.gamma.grad,
                                   self.bn1.beta.grad, y0.numel() // y0.shape[-1], relu_from_y=True,
                                   reduced=bnr is not None)
        self.arena.grad_ready(self.bn1.gamma, self.bn1.beta)
        self.conv1.backward(dy0, x0, need_dx=False)
        streams.join()  # side-stream weight gradients complete before anyone reads arena.grad
        return loss, corr


def resnet50(**kw) -> ResNet:
    return ResNet(50, **kw)


def resnet101(**kw) -> ResNet:
    return ResNet(101, **kw)


def resnet152(**kw) -> ResNet:
    return ResNet(152, **kw)


def synthetic_imagenet(batch: int, device, image_size: int = 224, num_classes: int = 1000, seed: int = 0):
    """On-device synthetic ImageNet-shaped batch: NHWC bf16 [B,224,224,8] (3 real channels,
    uniform [-1,1)) + int32 labels. Generated by HIP kernels on GPU (no H2D)."""
    x = torch.empty(batch, image_size, image_size, IN_CH_PAD, dtype=torch.bfloat16, device=device)
    y = torch.empty(batch, dtype=torch.int32, device=device)
    if x.is_cuda:
        from ..ops._lib import lib
        lib().synth_uniform(x, batch * image_size * image_size, 3, IN_CH_PAD, -1.0, 1.0, seed)
        lib().synth_labels(y, num_classes, seed + 1)
    else:
        g = torch.Generator().manual_seed(seed)
        x.zero_()
        x[..., :3] = (torch.rand(batch, image_size, image_size, 3, generator=g) * 2 - 1).to(torch.bfloat16)
        y.copy_(torch.randint(0, num_classes, (batch,), generator=g, dtype=torch.int32))
    return x, y
