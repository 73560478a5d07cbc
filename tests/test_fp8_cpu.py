"""CPU tier of the MX-fp8 bookkeeping (ops/fp8.py): the per-step quantization caches that let one
tensor feed several fp8 GEMMs (the encoder memory -> every decoder layer's cross-attention K/V) and
the grouped weight quantizer, on the exact CPU reference quantizer."""
import torch

from tensorflow_k8s_amd.ops import fp8 as F8


def test_shared_input_quantized_once_and_saved_per_use():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(128, 256, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(128, 256, generator=g) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(256, 256, generator=g) * 0.05).to(torch.bfloat16)
    F8.clear_saved()
    y1 = F8.linear_fwd_mx(x, w1, save=True)
    assert len(F8._XQ) == 1
    y2 = F8.linear_fwd_mx(x, w2, save=True)
    assert len(F8._XQ) == 1  # the second GEMM reused x's quantization
    t1, t2 = F8.take_t(x), F8.take_t(x)
    assert t1 is not None and t1 is t2  # one MX(x^T), handed to both weight gradients
    assert F8.take_t(x) is None
    F8.clear_saved()
    # same outputs as quantizing afresh
    assert torch.equal(y2, F8.linear_fwd_mx(x, w2))
    assert torch.equal(y1, F8.linear_fwd_mx(x, w1))
    # evaluation forwards (save=False) never consult or fill the cache
    F8.linear_fwd_mx(x, w1)
    assert not F8._XQ
    F8.clear_saved()


def test_group_quantizer_cpu_registers_weights():
    g = torch.Generator().manual_seed(1)
    ws = [(torch.randn(*sh, generator=g) * 0.05).to(torch.bfloat16) for sh in [(128, 256), (256, 128), (96, 64)]]
    gq = F8.GroupQuantizer(ws)
    F8.clear_saved()
    gq.run()
    for w, ((q, s), (qt, st)) in zip(ws, gq.out):
        (q1, s1), (qt1, st1) = F8.mx_quantize_dual(w)
        assert torch.equal(q, q1) and torch.equal(s, s1) and torch.equal(qt, qt1) and torch.equal(st, st1)
    x = torch.randn(128, 256, generator=g).to(torch.bfloat16)
    y = F8.linear_fwd_mx(x, ws[0], save=True)
    assert F8.take_t(ws[0]) is gq.out[0][1]  # the grouped MX(w^T) goes to the dgrad
    F8.clear_saved()
    assert torch.equal(y, F8.linear_fwd_mx(x, ws[0]))
    F8.clear_saved()
