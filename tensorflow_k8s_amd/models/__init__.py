"""Model zoo of the BASELINE configs: LeNet (MNIST), ResNet-50/101/152 (ImageNet),
BERT-base (SQuAD-style fine-tune / MLM), Transformer-big (WMT). All run on the tfk executor:
explicit forward/backward over the flat parameter arena and the gfx950 kernel library.

``build_model(name, **kw)`` returns an un-finalized model (call ``.to(device)``);
``synthetic_batch(model, batch, device, seed)`` returns an input batch of the model's shape.
"""
from __future__ import annotations


def build_model(name: str, **kw):
    name = name.lower()
    if name in ("lenet", "mnist"):
        from .lenet import LeNet
        return LeNet(**kw)
    if name.startswith("resnet"):
        from .resnet import ResNet
        return ResNet(int(name[len("resnet"):] or 50), **kw)
    if name in ("bert", "bert-base", "bert_base", "bert-large", "bert_large"):
        from .bert import BertConfig, BertForPreTraining
        cfg = BertConfig.large() if "large" in name else BertConfig.base()
        for k, v in kw.items():
            setattr(cfg, k, v)
        return BertForPreTraining(cfg)
    if name in ("transformer", "transformer-big", "transformer_big", "transformer-base", "transformer_base"):
        from .transformer import Transformer, TransformerConfig
        cfg = TransformerConfig.base() if "base" in name else TransformerConfig.big()
        for k, v in kw.items():
            setattr(cfg, k, v)
        return Transformer(cfg)
    raise ValueError(f"unknown model {name!r}")


def synthetic_batch(model, batch: int, device, seed: int = 0, **kw):
    name = model.name
    if name == "lenet":
        from .lenet import synthetic_mnist
        return synthetic_mnist(batch, device, model.num_classes, seed)
    if name.startswith("resnet"):
        from .resnet import synthetic_imagenet
        return synthetic_imagenet(batch, device, kw.get("image_size", 224), model.num_classes, seed)
    if hasattr(model, "synthetic_batch"):
        return model.synthetic_batch(batch, device, seed, **kw)
    raise ValueError(f"no synthetic data for {name}")
