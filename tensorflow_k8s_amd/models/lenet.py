"""LeNet-5 for MNIST (BASELINE config 1: "MNIST LeNet TFJob, 1 worker").

The reference's MNIST example (examples/tf_sample, dist-mnist) is a small Keras-style convnet:
conv5x5(6)+relu -> maxpool2 -> conv5x5(16)+relu -> maxpool2 -> dense(120)+relu -> dense(84)+relu
-> dense(10). On the tfk executor: NHWC bf16 with the single input channel padded to 8 (16-B
vectors) and conv1's 6 output channels padded to 8 (padded weights stay exactly zero); bias+relu
run in the conv/linear GEMM epilogues. TF variable names: conv1/kernel [5,5,1,6], conv1/bias,
conv2/kernel [5,5,6,16], fc1/kernel [400,120], ... so checkpoints match a Keras LeNet.
"""
from __future__ import annotations

import torch

from ..ops import elementwise as E
from ..ops import pool as PL
from ..ops.loss import softmax_xent
from ..runtime import streams
from ..runtime.arena import ParamArena
from ..runtime.layers import Conv2d, Linear

IN_CH_PAD = 8


class LeNet:
    def __init__(self, num_classes: int = 10, image_size: int = 28):
        self.name = "lenet"
        self.num_classes = num_classes
        self.training = True
        a = self.arena = ParamArena()
        self.conv1 = Conv2d(a, "conv1", IN_CH_PAD, 8, 5, pad=2, cin_real=1, cout_real=6, bias=True)
        self.conv2 = Conv2d(a, "conv2", 8, 16, 5, pad=0, cin_real=6, bias=True)
        s = (image_size // 2 - 4) // 2
        self.feat = s * s * 16
        self.fc1 = Linear(a, "fc1", self.feat, 120)
        self.fc2 = Linear(a, "fc2", 120, 84)
        self.fc3 = Linear(a, "fc3", 84, num_classes)
        self._saved = None

    def to(self, device, seed: int = 1234) -> "LeNet":
        self.arena.finalize(device, seed)
        return self

    def train(self, mode: bool = True) -> "LeNet":
        self.training = mode
        return self

    def _forward(self, x):
        a1 = self.conv1.forward(x, act="relu")
        p1, i1 = PL.maxpool_fwd(a1, 2, 2, 0)
        a2 = self.conv2.forward(p1, act="relu")
        p2, i2 = PL.maxpool_fwd(a2, 2, 2, 0)
        f = p2.reshape(p2.shape[0], -1)
        h1 = self.fc1.forward(f, act="relu")
        h2 = self.fc2.forward(h1, act="relu")
        logits = self.fc3.forward(h2)
        self._saved = (x, a1, p1, i1, a2, p2, i2, f, h1, h2)
        return logits

    def forward(self, x):
        logits = self._forward(x)
        self._saved = None
        return logits

    def forward_backward(self, x, labels, loss_scale: float = 1.0):
        logits = self._forward(x)
        B = logits.shape[0]
        loss, dlogits, corr = softmax_xent(logits, labels, scale=loss_scale / B, want_correct=True)
        x, a1, p1, i1, a2, p2, i2, f, h1, h2 = self._saved
        self._saved = None
        dh2 = self.fc3.backward(dlogits, h2)
        dh1 = self.fc2.backward(E.act_bwd(dh2, h2, "relu"), h1)
        df = self.fc1.backward(E.act_bwd(dh1, h1, "relu"), f)
        dp2 = df.reshape(p2.shape)
        da2 = PL.maxpool_bwd(dp2, i2, a2.shape, 2, 2, 0)
        dp1 = self.conv2.backward(E.act_bwd(da2, a2, "relu"), p1)
        da1 = PL.maxpool_bwd(dp1, i1, a1.shape, 2, 2, 0)
        self.conv1.backward(E.act_bwd(da1, a1, "relu"), x, need_dx=False)
        streams.join()  # side-stream weight gradients complete before anyone reads arena.grad
        return loss, corr


def synthetic_mnist(batch: int, device, num_classes: int = 10, seed: int = 0, image_size: int = 28):
    """Synthetic MNIST-shaped batch: NHWC bf16 [B,28,28,8] (1 real channel in [0,1)) + int32 labels.
    Learnable: each class has a fixed random prototype image, samples are prototype + noise."""
    g = torch.Generator().manual_seed(seed)
    proto = torch.rand(num_classes, image_size, image_size, generator=torch.Generator().manual_seed(77))
    y = torch.randint(0, num_classes, (batch,), generator=g, dtype=torch.int32)
    img = (proto[y.long()] * 0.8 + 0.2 * torch.rand(batch, image_size, image_size, generator=g)).clamp(0, 1)
    x = torch.zeros(batch, image_size, image_size, IN_CH_PAD, dtype=torch.bfloat16)
    x[..., 0] = img.to(torch.bfloat16)
    return x.to(device), y.to(device)
