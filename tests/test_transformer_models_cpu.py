"""BERT / Transformer explicit-backward executors vs fp32 torch autograd on the same parameters
(tiny configs, dropout off), plus checkpoint naming parity with the TF models."""
import pytest
import torch

from reference_models import bert_ref_loss


def _cos(a, b):
    a, b = a.float().reshape(-1), b.float().reshape(-1)
    return float(a @ b / (a.norm() * b.norm() + 1e-20))


def test_bert_tiny_grads_match_autograd():
    from tensorflow_k8s_amd.models.bert import BertConfig, BertForPreTraining
    cfg = BertConfig.tiny()
    cfg.hidden_dropout = cfg.attn_dropout = 0.0
    m = BertForPreTraining(cfg).to("cpu", seed=5)
    batch = m.synthetic_batch(4, "cpu", seed=1)
    loss, _ = m.forward_backward(*batch)
    ref_loss, ref_g = bert_ref_loss(m, *batch)
    assert abs(float(loss.mean()) - ref_loss) / ref_loss < 2e-2
    bad = []
    for p in m.arena.params:
        g, r = p.grad, ref_g[p.name]
        if r.norm() < 1e-6:
            continue
        c = _cos(g, r)
        if c < 0.98:
            bad.append((p.name, round(c, 4)))
    assert not bad, bad


def test_bert_checkpoint_names():
    from tensorflow_k8s_amd.models.bert import BertConfig, BertForPreTraining
    m = BertForPreTraining(BertConfig.tiny())
    names = {p.name: p for p in m.arena.params}
    for n in ["bert/embeddings/word_embeddings", "bert/encoder/layer_0/attention/self/query/kernel",
              "bert/encoder/layer_1/output/LayerNorm/gamma", "cls/predictions/output_bias",
              "cls/seq_relationship/output_weights", "cls/seq_relationship/output_bias", "bert/pooler/dense/bias"]:
        assert n in names, n
    assert names["bert/embeddings/word_embeddings"].spec.tf_shape == (1000, 128)


def test_transformer_tiny_grads_match_autograd():
    from reference_models import transformer_ref_loss
    from tensorflow_k8s_amd.models.transformer import Transformer, TransformerConfig
    cfg = TransformerConfig.tiny()
    cfg.dropout = cfg.attn_dropout = cfg.relu_dropout = 0.0
    m = Transformer(cfg).to("cpu", seed=7)
    batch = m.synthetic_batch(3, "cpu", seed=2)
    loss, _ = m.forward_backward(*batch)
    ref_loss, ref_g = transformer_ref_loss(m, *batch)
    assert abs(float(loss.mean()) - ref_loss) / ref_loss < 2e-2, (float(loss.mean()), ref_loss)
    bad = []
    for p in m.arena.params:
        g, r = p.grad, ref_g[p.name]
        if r.norm() < 1e-6:
            continue
        c = _cos(g, r)
        if c < 0.98:
            bad.append((p.name, round(c, 4)))
    assert not bad, bad


def test_transformer_trains_with_dropout():
    from tensorflow_k8s_amd.models.transformer import Transformer, TransformerConfig
    from tensorflow_k8s_amd.runtime.optimizer import AdamW
    m = Transformer(TransformerConfig.tiny()).to("cpu", seed=1)
    opt = AdamW(m.arena, 2e-3, weight_decay=0.0)
    batch = m.synthetic_batch(4, "cpu", seed=3)
    losses = []
    for _ in range(6):
        loss, _ = m.forward_backward(*batch)
        opt.step()
        losses.append(float(loss.mean()))
    assert losses[-1] < losses[0]


def test_transformer_fp8_forward_close_to_bf16():
    """MX-fp8 forward GEMMs (CPU reference of the quantized product) keep the loss and the
    gradients close to the bf16 model."""
    from tensorflow_k8s_amd.models.transformer import Transformer, TransformerConfig
    res = {}
    for fp8 in (False, True):
        cfg = TransformerConfig(vocab_size=500, hidden=128, enc_layers=1, dec_layers=1, heads=2, ffn=256, src_len=16,
                                tgt_len=16, max_len=32, dropout=0.0, attn_dropout=0.0, relu_dropout=0.0, fp8=fp8)
        m = Transformer(cfg).to("cpu", seed=4)
        loss, _ = m.forward_backward(*m.synthetic_batch(2, "cpu", seed=1))
        res[fp8] = (float(loss.mean()), m.arena.grad.clone())
    assert abs(res[True][0] - res[False][0]) / res[False][0] < 0.02
    assert _cos(res[True][1], res[False][1]) > 0.98


def test_transformer_fp8_mx_producers_match_separate_quantization():
    """fp8 training with 128-token batches: LayerNorms / FFN GEMMs that emit their consumers' MX
    operands (models.transformer MX_PRODUCERS, ops.fp8 _register_out; bf16 outputs skipped) give the
    same loss and gradients, bit for bit, as quantizing every GEMM input in a separate pass."""
    import tensorflow_k8s_amd.models.transformer as TM
    from tensorflow_k8s_amd.ops import fp8 as F8
    res = {}
    orig = F8.clear_saved
    seen = []

    def clear_and_count():  # the step clears its caches on exit: count the MX registrations first
        seen.append(len(F8._XQ))
        orig()
    F8.clear_saved = clear_and_count
    for prod in (False, True):
        TM.MX_PRODUCERS = prod
        try:
            cfg = TM.TransformerConfig(vocab_size=500, hidden=128, enc_layers=1, dec_layers=2, heads=2, ffn=256,
                                       src_len=64, tgt_len=64, max_len=128, dropout=0.1, attn_dropout=0.1,
                                       relu_dropout=0.1, fp8=True)
            m = TM.Transformer(cfg).to("cpu", seed=4)
            seen.clear()
            loss, _ = m.forward_backward(*m.synthetic_batch(2, "cpu", seed=1))
            res[prod] = (loss.clone(), m.arena.grad.clone(), max(seen))
        finally:
            TM.MX_PRODUCERS = True
            F8.clear_saved = orig if prod else clear_and_count
    assert not F8._XQ and not F8._SAVED and not F8._WQ  # nothing survives the step
    assert res[True][2] > res[False][2]  # producers registered their MX outputs
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])


@pytest.mark.parametrize("which", ["bert", "transformer"])
def test_layernorm_backward_bias_fusion_matches_column_sums(which, monkeypatch):
    """LayerNorm backward reducing its consumer Linear's bias gradient (runtime.layers LayerNorm.backward
    consumer) gives the same gradients as the consumers' own column-sum passes."""
    import tensorflow_k8s_amd.runtime.layers as L
    res = {}
    for fused in (True, False):
        if not fused:
            monkeypatch.setattr(L.Linear, "bias_sink", lambda self: None)
        if which == "bert":
            from tensorflow_k8s_amd.models.bert import BertConfig, BertForPreTraining
            cfg = BertConfig(vocab_size=300, hidden=128, layers=2, heads=2, intermediate=256, max_position=64,
                             seq_len=32, max_predictions=5)
            m = BertForPreTraining(cfg).to("cpu", seed=3)
        else:
            from tensorflow_k8s_amd.models.transformer import Transformer, TransformerConfig
            cfg = TransformerConfig(vocab_size=300, hidden=128, enc_layers=2, dec_layers=2, heads=2, ffn=256,
                                    src_len=16, tgt_len=16, max_len=32)
            m = Transformer(cfg).to("cpu", seed=3)
        loss, _ = m.forward_backward(*m.synthetic_batch(2, "cpu", seed=1))
        res[fused] = (loss.clone(), m.arena.grad.clone())
        monkeypatch.undo()
    assert torch.equal(res[True][0], res[False][0])
    torch.testing.assert_close(res[True][1], res[False][1], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mx_wgrad", [True, False])
def test_transformer_fp8_mx_wgrad_switch_finite_and_tracks_bf16(mx_wgrad, monkeypatch):
    """fp8 training with MX producers and either weight-gradient precision (ops.fp8.MX_WGRAD, bench.py
    --mx-wgrad): every gradient is finite and tracks the bf16 model. The CPU reference poisons the bf16
    values of MX-only outputs with NaN (ops.fp8._poison_no_c), so a bf16 consumer of one -- the
    round-5 ff1 weight gradient reading the never-stored dz -- fails here instead of on the GPU."""
    import tensorflow_k8s_amd.models.transformer as TM
    from tensorflow_k8s_amd.ops import fp8 as F8
    monkeypatch.setattr(F8, "MX_WGRAD", mx_wgrad)
    res = {}
    for fp8 in (False, True):
        cfg = TM.TransformerConfig(vocab_size=500, hidden=128, enc_layers=1, dec_layers=1, heads=2, ffn=256,
                                   src_len=64, tgt_len=64, max_len=128, dropout=0.1, attn_dropout=0.1,
                                   relu_dropout=0.1, fp8=fp8)
        m = TM.Transformer(cfg).to("cpu", seed=4)
        loss, _ = m.forward_backward(*m.synthetic_batch(2, "cpu", seed=1))
        res[fp8] = (float(loss.mean()), m.arena.grad.clone())
    assert torch.isfinite(res[True][1]).all()
    assert abs(res[True][0] - res[False][0]) / res[False][0] < 0.02
    assert _cos(res[True][1], res[False][1]) > 0.98


def test_mx_only_output_refuses_bf16_consumers():
    """An MX-only GEMM output (mx_skip_c) raises when a bf16 consumer reaches it."""
    from tensorflow_k8s_amd.ops import fp8 as F8
    x = torch.randn(128, 128).bfloat16()
    w = torch.randn(128, 128).bfloat16()
    try:
        y = F8.linear_fwd_mx(x, w, mx_out=True, mx_skip_c=True)
        assert torch.isnan(y.float()).all()
        with pytest.raises(RuntimeError, match="mx_skip_c"):
            F8.check_stored(y)
        with pytest.raises(RuntimeError, match="mx_skip_c"):
            F8.linear_dgrad_mx(y, w)
    finally:
        F8.clear_saved()
